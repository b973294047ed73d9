# Round 5: long seeded fuzz runs: the batch/strict irregular vote corpus (new `batch` mode,
# 60 seeds over Straus / Pippenger / fused one-call sizes) and 60 more irregular-committee
# certificate seeds (60..119).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 700 python -u tools/fuzz_long.py 0 60 batch > $O/fuzz_batch.json 2> $O/fuzz_batch.err || { tail -20 $O/fuzz_batch.err; exit 1; }
cut -c1-600 $O/fuzz_batch.json
timeout -k 10 900 python -u tools/fuzz_long.py 60 60 irregular > $O/fuzz_irregular.json 2> $O/fuzz_irregular.err || { tail -20 $O/fuzz_irregular.err; exit 1; }
cut -c1-600 $O/fuzz_irregular.json
