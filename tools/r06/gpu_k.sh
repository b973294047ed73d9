# Round 6: more differential fuzz on the final tree: irregular committees (small-job kernel,
# bulk keyed pipeline, per-certificate path; injected and random coefficients) and the
# batch / strict corpus, each bounded.
set -o pipefail
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r06k}; mkdir -p $O
timeout -k 10 500 python -u tools/fuzz_long.py 30000 150 irregular > $O/fuzz_irregular.json 2> $O/fuzz_irregular.err || { tail -20 $O/fuzz_irregular.err; exit 1; }
cut -c1-500 $O/fuzz_irregular.json
timeout -k 10 400 python -u tools/fuzz_long.py 20300 600 batch > $O/fuzz_batch.json 2> $O/fuzz_batch.err || { tail -20 $O/fuzz_batch.err; exit 1; }
cut -c1-500 $O/fuzz_batch.json
