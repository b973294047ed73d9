# Round 5: the 1,000-seed irregular-committee campaign again (seeds 120..1119) with the
# widened possible-verdict search (r05q's one flag, seed 236 certificate 57, is a verdict of
# probability 251/2048 that the 64 sampled coefficient sets missed).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 700 python -u tools/fuzz_long.py 120 1000 irregular > $O/fuzz_irregular.json 2> $O/fuzz_irregular.err || { tail -20 $O/fuzz_irregular.err; exit 1; }
cut -c1-700 $O/fuzz_irregular.json
