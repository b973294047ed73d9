#!/bin/bash
# GPU box: A/B the strict kernel builds given as arguments (tools/strict_variants.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/strict_variants.py --reps ${REPS:-3} --steps ${STEPS:-3} "$@" \
  > gpurun_out/variants.json 2> gpurun_out/variants.err
rc=$?
cat gpurun_out/variants.json
tail -3 gpurun_out/variants.err
exit $rc
