#!/bin/bash
# GPU-box helper: config-2 certificate stream (all-valid and 1 % invalid legs) at fixed merged
# group sizes (NW_CERT_GROUP_VOTES) and with merging off (NW_CERT_MERGE=0), then one kernel
# trace of a small-group run, to price a group's tail against its votes.
#   bash tools/group_sweep.sh OUTDIR [VOTES...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/group_sweep}
shift
SIZES=${*:-"32768 4096 1024 512"}
mkdir -p "$OUT"
ARGS="--workload cert --committees ${COMMITTEES:-4,10,50,100} --cert-steps 2"
for v in $SIZES; do
  NW_CERT_GROUP_VOTES=$v timeout -k 10 240 python3 -u bench.py $ARGS > "$OUT/v$v.json" 2> "$OUT/v$v.err" \
    || { echo "votes $v failed"; tail -5 "$OUT/v$v.err"; exit 1; }
  echo "votes $v ok"
done
NW_CERT_MERGE=0 timeout -k 10 240 python3 -u bench.py $ARGS > "$OUT/merge0.json" 2> "$OUT/merge0.err" \
  || { echo "merge0 failed"; exit 1; }
echo "merge0 ok"
if [ -n "$TRACE_VOTES" ]; then
  NW_CERT_GROUP_VOTES=$TRACE_VOTES timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/trace" -o p -- python3 bench.py --workload cert --committees ${TRACE_N:-100} --cert-steps 2 \
    > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo "trace failed"; exit 1; }
  echo "trace ok"
fi
