#!/bin/bash
# GPU-box helper: kernel trace of the config-2 1 %-invalid leg alone for one committee size.
#   bash tools/gpu_cert_trace_inv.sh OUTDIR N
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/cert_trace_inv}; N=${2:-4}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/n$N -o p \
  -- python3 bench.py --workload cert --committees $N --no-sha --no-batch --no-wire \
  --no-cpu-baseline --cert-steps 3 > $OUT/n$N.json 2> $OUT/n$N.log || { echo "trace N=$N failed"; exit 1; }
echo "trace N=$N ok"
