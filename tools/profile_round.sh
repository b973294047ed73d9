#!/bin/bash
# GPU-box helper: the round's profile set, each step under its own time limit, stopping at
# the first failure (no retries).
#   1. rocprofv3 --kernel-trace --stats of the default bench.py run (all legs)
#   2. PMC passes, one counter group per rocprofv3 run (MI355X_MICROARCH.md: FETCH_SIZE and
#      WRITE_SIZE cannot share a pass), over one untimed-warmup-free bench step of the
#      config-4 strict leg and the config-3 SHA-512 leg at their full bench sizes, so the
#      per-dispatch counters are per bench launch; then the same over one config-1
#      verify_batch step (the Pippenger kernels, 64 resident 10k batches).
# Usage (on the GPU box): bash tools/profile_round.sh TAG   -> gpurun_out/prof_TAG/
# Summarise here with: python tools/profile_summary.py gpurun_out/prof_TAG profiles/TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-run}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
PMC_ARGS="--steps 1 --warmup 0 --no-cert --no-batch --no-wire --no-service --no-worker --no-cpu-baseline"

timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_available.txt" 2>&1
echo "list rc=$?"

timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o p \
  -- python3 bench.py --no-cpu-baseline > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.log" \
  || { echo "trace pass failed"; exit 1; }
echo "trace pass ok"

pmc() {
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$name" -o p \
    -- python3 bench.py $PMC_ARGS > "$OUT/pmc_$name.json" 2> "$OUT/pmc_$name.log"
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
pmc fetch FETCH_SIZE && \
pmc write WRITE_SIZE && \
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
  SQ_BUSY_CYCLES SQ_WAIT_INST_ANY && \
pmc grbm GRBM_GUI_ACTIVE GRBM_COUNT && \
PMC_ARGS="--workload batch --steps 1 --warmup 0 --no-cpu-baseline" && \
pmc batch_fetch FETCH_SIZE && \
pmc batch_write WRITE_SIZE && \
pmc batch_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
  SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
