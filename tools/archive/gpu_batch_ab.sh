#!/bin/bash
# GPU box: batch tests, then config-1 latency/throughput for the in-tree build and variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_messages.py -x -q --timeout 200 --timeout-method thread > gpurun_out/batch_tests.log 2>&1 || { tail -30 gpurun_out/batch_tests.log; exit 1; }
tail -2 gpurun_out/batch_tests.log
for L in narwhal_amd/libnarwhal_amd.so "$@"; do
  NW_LIB=$L timeout -k 10 200 python bench.py --workload batch --steps 5 --no-cpu-baseline > gpurun_out/ab_batch.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_batch.json').read().splitlines()[-1])['verify_batch_10k'];print(sys.argv[1], round(d['latency_ms'],4), round(d['verifies_per_s_resident']/1e6,1), d['parity'])" $L
done
