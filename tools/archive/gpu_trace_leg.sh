#!/bin/bash
# GPU-box helper: rocprofv3 kernel trace (+ HIP API and copy trace) of one bench leg.
#   bash tools/gpu_trace_leg.sh OUTDIR LEG [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=$1; LEG=$2; shift 2
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --stats \
  --output-format csv -d "$OUT/$LEG" -o p -- python3 bench.py --workload $LEG --no-cpu-baseline "$@" \
  > "$OUT/$LEG.json" 2> "$OUT/$LEG.log"
rc=$?; echo "trace $LEG rc=$rc"; exit $rc
