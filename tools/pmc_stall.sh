#!/bin/bash
# Stall breakdown of the config-4 strict kernel (GPU box): one PMC pass of the SQ wave-state
# counters (WAIT_ANY = parked on s_waitcnt/barrier, WAIT_INST_ANY = issue stall,
# ACTIVE_INST_ANY = issuing; MI355X_MICROARCH.md §rocprofv3 PMC slots) and one GRBM pass.
#   bash tools/pmc_stall.sh OUTDIR [LIB]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_stall}
[ -n "$2" ] && export NW_LIB=$2
ARGS="--items-per-gpu 4194304 --steps 1 --warmup 0 --no-cpu-baseline --no-sha --no-cert --no-batch --no-wire --no-service --no-worker"
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o p \
    -- python3 bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.log
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_THREAD_CYCLES_VALU && \
run sq2 SQ_WAVES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM \
  SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_LEVEL_WAVES && \
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
