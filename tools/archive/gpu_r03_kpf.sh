#!/bin/bash
# GPU-box helper: message/fan-out/service tests, keyed-prefetch A/B on config 2, and the
# service's host timing breakdown at N = 50 under high load.
set -o pipefail
O=gpurun_out/kpf; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_messages.py tests/test_gpu_fanout.py \
  tests/test_service.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload cert --no-cpu-baseline --cert-invalid 0 \
  > $O/pf.json 2> $O/pf.log || exit 1
NW_LIB=exp/nokpf/libnarwhal_amd.so timeout -k 10 400 python -u bench.py --workload cert \
  --no-cpu-baseline --cert-invalid 0 > $O/nopf.json 2>> $O/pf.log || exit 1
NW_SERVICE_DEBUG=1 timeout -k 10 200 python -u bench.py --workload service --no-cpu-baseline \
  --service-committees 50 --service-rates 100000,1000000 > $O/svc_dbg.json 2> $O/svc_dbg.log
grep "service:" $O/svc_dbg.log
