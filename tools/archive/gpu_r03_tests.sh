#!/bin/bash
# GPU-box helper: the -m gpu suite, the certificate-service latency leg, and config 2 with
# the default policy (keyed vote checks; MERGED=1: also the merged-group policy) and with
# variant builds (VARIANTS="name ..." = exp/<name>/libnarwhal_amd.so).
#   bash tools/gpu_r03_tests.sh OUTDIR [pytest -k expr]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r03}; mkdir -p "$OUT"
K=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  ${K:+-k "$K"} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload service > "$OUT/bench_service.json" 2> "$OUT/bench_service.log"
rc=$?; echo "service bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload cert --no-cpu-baseline > "$OUT/bench_cert.json" 2> "$OUT/bench_cert.log"
rc=$?; echo "cert bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ -n "$MERGED" ] && { NW_CERT_KEYED=0 timeout -k 10 300 python -u bench.py --workload cert --no-cpu-baseline > "$OUT/bench_cert_merged.json" 2> "$OUT/bench_cert_merged.log"
rc=$?; echo "merged-groups cert bench rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for V in $VARIANTS; do
  NW_LIB=exp/$V/libnarwhal_amd.so timeout -k 10 300 python -u bench.py --workload cert \
    --no-cpu-baseline > "$OUT/bench_cert_keyed_$V.json" 2> "$OUT/bench_cert_keyed_$V.log"
  rc=$?; echo "keyed cert bench $V rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
