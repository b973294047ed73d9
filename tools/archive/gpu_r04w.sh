# Quorum on wave 0 beside the header digest (small-job kernel): parity tests, stamps, service.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_small.py tests/test_gpu_messages.py tests/test_service.py > gpurun_out/r04w_tests.log 2>&1 || { tail -30 gpurun_out/r04w_tests.log; exit 1; }
tail -1 gpurun_out/r04w_tests.log
timeout -k 10 200 python -u tools/small_stamps.py > gpurun_out/r04w_stamps.txt 2>&1 || exit 1
grep "blocking\|slots=35 " gpurun_out/r04w_stamps.txt | cut -c1-330
NW_SERVICE_DEBUG=1 timeout -k 10 250 python -u bench.py --workload service --service-rates 1000,10000,100000,1000000,1000000 > gpurun_out/r04w_service.json 2> gpurun_out/r04w_service.err || exit 1
