#!/bin/bash
# GPU-box helper: PMC passes of config 1's one-call path (tools/ab_batch_latency.py: 10k
# verify_batch calls through the host entry point -> k_pip_points_sorted + k_pip_tail_fused),
# one rocprofv3 run per counter group, each under its own time limit, stopping at the first
# failure. Summarise with: python tools/pmc_config1_summary.py OUTDIR profiles/TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_config1}
mkdir -p "$OUT"
run() {  # run NAME [rocprofv3 args...]
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o p -- \
    python3 tools/ab_batch_latency.py 40 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "config1 $name rc=$rc"
  return $rc
}
run fetch --pmc FETCH_SIZE && \
run write --pmc WRITE_SIZE && \
run tcc --pmc TCC_HIT_sum TCC_MISS_sum && \
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU || exit 1
