# Round 5 (session 2): more irregular-committee certificate fuzz seeds (4,120..6,119).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f4; mkdir -p $O
timeout -k 10 1000 python -u tools/fuzz_long.py 4120 2000 irregular > $O/fuzz_irregular.json 2> $O/fuzz_irregular.err || { tail -20 $O/fuzz_irregular.err; exit 1; }
cut -c1-700 $O/fuzz_irregular.json
