#!/bin/bash
# VALU instruction mix of the config-4 strict kernel (GPU box): 32- vs 64-bit integer VALU
# instructions (v_mad_u64_u32 / 64-bit shifts count as INT64), all VALU, and the SQ cycle
# counters, one rocprofv3 --pmc pass (8 SQ counters), for DESIGN.md's issue-time budget.
#   bash tools/pmc_mix.sh OUTDIR
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_mix}
ARGS="--items-per-gpu 4194304 --steps 1 --warmup 0 --no-cpu-baseline --no-sha --no-cert --no-batch --no-wire --no-service --no-worker"
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 \
  SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d $OUT/mix -o p -- python3 bench.py $ARGS > $OUT/mix.json 2> $OUT/mix.log
echo "pass mix rc=$?"
