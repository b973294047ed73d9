#!/bin/bash
# GPU-box helper: GPU parity tests, a strict-only bench line and the strict-kernel PMC
# passes, each step under its own time limit; stops at the first failure.
# Usage (on the GPU box): bash tools/gpu_strict_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cert --no-batch --no-sha --no-cpu-baseline \
  > gpurun_out/bench_strict_$TAG.json 2> gpurun_out/bench_strict_$TAG.log || { echo "bench failed"; exit 1; }
bash tools/pmc_strict.sh gpurun_out/pmc_strict_$TAG
