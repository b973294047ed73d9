#!/bin/bash
# Per-phase split of k_verify_strict, step 2 (GPU box): SQ_INSTS_VALU (+ its INT64 / INT32
# parts) of one bench-size launch of the full kernel and of each phase-cut build
# (tools/r06/phases/stop<k>, tools/strict_phases.sh), one rocprofv3 --pmc pass each. The cut builds'
# statuses are digests, not verdicts, so their bench parity fails by design (rc 1 is
# expected; anything else stops the script). Summary: tools/strict_phases_summary.py.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/strict_phases}
ARGS="--items-per-gpu 1048576 --steps 1 --warmup 0 --no-cpu-baseline --no-sha --no-cert --no-batch --no-wire --no-worker --no-service"
mkdir -p $OUT
for v in full stop1 stop2 stop3 stop4 stop5 stop6; do
  lib=narwhal_amd/libnarwhal_amd.so
  [ $v != full ] && lib=tools/r06/phases/$v/libnarwhal_amd.so
  NW_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_WAVES \
    --output-format csv -d $OUT/$v -o p -- python bench.py $ARGS > $OUT/$v.log 2>&1
  rc=$?
  echo "pass $v rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
