# Round 6: differential fuzz after the small-job done-flag fix (flag words cleared before the
# launch, process-unique sequence numbers): irregular committees over the small-job kernel,
# the bulk keyed pipeline and the per-certificate path, new seeds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ag; mkdir -p $O
timeout -k 10 500 python -u tools/fuzz_long.py 40000 150 irregular > $O/fuzz_irregular.json 2> $O/fuzz_irregular.err || { tail -20 $O/fuzz_irregular.err; exit 1; }
cut -c1-600 $O/fuzz_irregular.json
