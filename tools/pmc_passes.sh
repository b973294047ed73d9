#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, as the MI355X
# guide prescribes). Output: gpurun_out/pmc_<name>/p_counter_collection.csv
# Usage (on the GPU box): bash tools/pmc_passes.sh [extra bench args]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ARGS="--items-per-gpu 1048576 --steps 1 --warmup 0 --no-cpu-baseline --sha-batches 8192 $*"
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_$name -o p \
    -- python bench.py $ARGS > gpurun_out/pmc_$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1; echo "list rc=$?"
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT && \
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
