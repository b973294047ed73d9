# Tail-block loads issued together (header SHA in the small-job kernel) + service eager A/B.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_service.py > gpurun_out/r04v_tests.log 2>&1; tail -1 gpurun_out/r04v_tests.log
timeout -k 10 200 python -u tools/small_stamps.py > gpurun_out/r04v_stamps.txt 2>&1 || exit 1
grep "blocking\|slots=35 " gpurun_out/r04v_stamps.txt | cut -c1-330
timeout -k 10 200 python -u bench.py --workload sha --steps 5 > gpurun_out/r04v_sha.json 2> gpurun_out/r04v_sha.err || exit 1
for e in 2 1; do
  NW_SERVICE_EAGER=$e NW_SERVICE_DEBUG=1 timeout -k 10 250 python -u bench.py --workload service --service-rates 1000,10000,100000,1000000,1000000 > gpurun_out/r04v_service_e$e.json 2> gpurun_out/r04v_service_e$e.err || exit 1
done
