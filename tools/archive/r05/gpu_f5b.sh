# Round 5 (session 2): batch/strict irregular-signer fuzz on the final tree (seeds 7,060..9,059).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f5; mkdir -p $O
timeout -k 10 500 python -u tools/fuzz_long.py 7060 2000 batch > $O/fuzz_batch_7060.json 2> $O/fuzz_batch_7060.err || { tail -20 $O/fuzz_batch_7060.err; exit 1; }
cut -c1-600 $O/fuzz_batch_7060.json
