#!/bin/bash
# GPU-box helper: kernel trace of the config-2 legs alone, one committee size per run.
#   bash tools/gpu_cert_trace.sh OUTDIR N [N ...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/cert_trace}; shift
mkdir -p $OUT
for N in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/n$N -o p \
    -- python3 bench.py --workload cert --committees $N --no-sha --no-batch --no-wire \
    --no-cpu-baseline --cert-steps 2 --cert-invalid 0 > $OUT/n$N.json 2> $OUT/n$N.log || { echo "trace N=$N failed"; exit 1; }
  echo "trace N=$N ok"
done
