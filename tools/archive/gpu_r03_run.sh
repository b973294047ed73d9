#!/bin/bash
# GPU-box helper (round 3): the -m gpu suite, then the bench legs named in LEGS
# (cert, service, strict, batch, wire, full), each step under its own time limit, stopping at the
# first failure.   LEGS="cert service" bash tools/gpu_r03_run.sh OUTDIR
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r03}; mkdir -p "$OUT"
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
for L in $LEGS; do
  case $L in
    full) A="" ;;
    cert) A="--workload cert --no-cpu-baseline" ;;
    service) A="--workload service --no-cpu-baseline" ;;
    strict) A="--workload strict --no-sha --no-cert --no-batch --no-wire --no-service --no-cpu-baseline" ;;
    batch) A="--workload batch --no-cpu-baseline" ;;
    wire) A="--workload strict --no-sha --no-cert --no-batch --no-service --no-cpu-baseline" ;;
    *) echo "unknown leg $L"; exit 2 ;;
  esac
  timeout -k 10 500 python -u bench.py $A > "$OUT/bench_$L.json" 2> "$OUT/bench_$L.log"
  rc=$?; echo "bench $L rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$L.log"; exit $rc; }
done
