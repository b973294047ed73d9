#!/bin/bash
# PMC passes for the strict-verify kernel only (one counter group per rocprofv3 run, as the
# MI355X guide prescribes). Usage (GPU box): bash tools/pmc_strict.sh OUTDIR
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_strict}
ARGS="--items-per-gpu 1048576 --steps 1 --warmup 0 --no-cpu-baseline --no-sha --no-cert --no-batch"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o p \
    -- python bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
mkdir -p $OUT
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE
