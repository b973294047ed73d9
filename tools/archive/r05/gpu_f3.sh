# Round 5: the irregular-committee fuzz again after the per-committee key-comb widths (20-bit
# tables for N <= 16): seeds 3,120..4,119; and the plain certificate fuzz (seeds 0..199).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f3; mkdir -p $O
timeout -k 10 600 python -u tools/fuzz_long.py 3120 1000 irregular > $O/fuzz_irregular.json 2> $O/fuzz_irregular.err || { tail -20 $O/fuzz_irregular.err; exit 1; }
cut -c1-500 $O/fuzz_irregular.json
timeout -k 10 500 python -u tools/fuzz_long.py 0 200 > $O/fuzz_plain.json 2> $O/fuzz_plain.err || { tail -20 $O/fuzz_plain.err; exit 1; }
cut -c1-400 $O/fuzz_plain.json
