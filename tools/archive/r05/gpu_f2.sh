# Round 5: more irregular-committee certificate fuzz seeds (1,120..3,119).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f2; mkdir -p $O
timeout -k 10 1000 python -u tools/fuzz_long.py 1120 2000 irregular > $O/fuzz_irregular.json 2> $O/fuzz_irregular.err || { tail -20 $O/fuzz_irregular.err; exit 1; }
cut -c1-700 $O/fuzz_irregular.json
