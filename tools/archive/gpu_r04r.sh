set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_service.py > gpurun_out/r04r_tests.log 2>&1; tail -2 gpurun_out/r04r_tests.log
NW_SERVICE_DEBUG=1 timeout -k 10 300 python -u bench.py --workload service --service-rates 1000,10000,100000,1000000,1000000,1000000,1000000 > gpurun_out/r04r_service.json 2> gpurun_out/r04r_service.err || exit 1
grep "service:" gpurun_out/r04r_service.err
