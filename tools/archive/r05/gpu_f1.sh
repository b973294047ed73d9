# Round 5: more batch/strict irregular-signer fuzz seeds (2,060..6,059).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f1; mkdir -p $O
timeout -k 10 1000 python -u tools/fuzz_long.py 2060 4000 batch > $O/fuzz_batch.json 2> $O/fuzz_batch.err || { tail -20 $O/fuzz_batch.err; exit 1; }
cut -c1-600 $O/fuzz_batch.json
