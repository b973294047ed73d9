set -o pipefail
timeout -k 10 60 ./tools/ubench_h2d 10000 200 > gpurun_out/r04k_h2d.json && timeout -k 10 60 ./tools/ubench_h2d 35000 100 >> gpurun_out/r04k_h2d.json && cat gpurun_out/r04k_h2d.json || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_service.py tests/test_gpu_batch.py > gpurun_out/r04k_tests.log 2>&1; tail -3 gpurun_out/r04k_tests.log
for f in 1 0 1 0; do NW_BATCH_FORK=$f timeout -k 10 60 python -u tools/ab_batch_latency.py 400 2>&1 | sed "s/^/fork=$f /" || exit 1; done | tee gpurun_out/r04k_ab_fork.txt
NW_SERVICE_DEBUG=1 timeout -k 10 200 python -u bench.py --workload service --service-rates 1000,10000,100000,1000000,1000000 > gpurun_out/r04k_service.json 2> gpurun_out/r04k_service.err; tail -4 gpurun_out/r04k_service.err
timeout -k 10 200 python -u bench.py --workload worker --worker-rates 50 > gpurun_out/r04k_worker.json 2> gpurun_out/r04k_worker.err; tail -2 gpurun_out/r04k_worker.err
