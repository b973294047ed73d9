#!/bin/bash
# GPU-box helper: kernel trace + PMC passes of the config-2 certificate kernels, per
# committee size and grouping mode, each rocprofv3 run under its own time limit, stopping at
# the first failure (no retries).
#   bash tools/pmc_cert.sh OUTDIR N [N ...]
# Modes (MODES="big keyed" by default): "keyed" = all-valid stream with the default policy
# (k_votes_keyed + verify_batch of failed certificates only), "big" = the same stream with
# NW_CERT_KEYED=0 (merged Pippenger groups: k_grp_keys, k_pip_*). One bench step (plus its warmup call) at the full 1M-certificate
# size, so per-dispatch counters are per bench launch.
# Summarise with: python tools/pmc_cert_summary.py OUTDIR profiles/TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_cert}; shift
mkdir -p "$OUT"
ARGS="--workload cert --no-sha --no-batch --no-wire --no-cpu-baseline --cert-steps 1 --cert-invalid 0 --cert-payload-committees="

run() {  # run NAME N MODE [rocprofv3 args...]
  local name=$1 n=$2 mode=$3; shift 3
  local envk=1
  [ "$mode" = big ] && envk=0
  NW_CERT_KEYED=$envk timeout -s KILL 240 rocprofv3 "$@" --output-format csv \
    -d "$OUT/${mode}_n${n}_$name" -o p -- python3 bench.py $ARGS --committees "$n" \
    > "$OUT/${mode}_n${n}_$name.json" 2> "$OUT/${mode}_n${n}_$name.log"
  local rc=$?
  echo "$mode N=$n $name rc=$rc"
  return $rc
}

for N in "$@"; do
  for MODE in ${MODES:-big keyed}; do
    run trace "$N" "$MODE" --kernel-trace --stats && \
    run fetch "$N" "$MODE" --pmc FETCH_SIZE && \
    run write "$N" "$MODE" --pmc WRITE_SIZE && \
    run tcc "$N" "$MODE" --pmc TCC_HIT_sum TCC_MISS_sum && \
    run sq "$N" "$MODE" --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT && \
    run grbm "$N" "$MODE" --pmc GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
  done
done
