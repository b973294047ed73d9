set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch.py > gpurun_out/r04ab_tests.log 2>&1 || { tail -30 gpurun_out/r04ab_tests.log; exit 1; }
tail -1 gpurun_out/r04ab_tests.log
for i in 1 2; do timeout -k 10 60 python -u tools/ab_batch_latency.py 400 || exit 1; done
