# Round 5: the long fuzz campaigns at scale: 2,000 batch/strict seeds (60..2059) and 1,000
# irregular-committee certificate seeds (120..1119).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 500 python -u tools/fuzz_long.py 60 2000 batch > $O/fuzz_batch.json 2> $O/fuzz_batch.err || { tail -20 $O/fuzz_batch.err; exit 1; }
cut -c1-600 $O/fuzz_batch.json
timeout -k 10 500 python -u tools/fuzz_long.py 120 1000 irregular > $O/fuzz_irregular.json 2> $O/fuzz_irregular.err || { tail -20 $O/fuzz_irregular.err; exit 1; }
cut -c1-600 $O/fuzz_irregular.json
