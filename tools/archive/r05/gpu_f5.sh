# Round 5 (session 2): batch/strict irregular-signer fuzz on the final tree (seeds 6,060..7,059).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f5; mkdir -p $O
timeout -k 10 400 python -u tools/fuzz_long.py 6060 1000 batch > $O/fuzz_batch.json 2> $O/fuzz_batch.err || { tail -20 $O/fuzz_batch.err; exit 1; }
cut -c1-600 $O/fuzz_batch.json
