set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_fuzz.py > gpurun_out/r04ag_tests.log 2>&1 || { tail -40 gpurun_out/r04ag_tests.log; exit 1; }
tail -1 gpurun_out/r04ag_tests.log
NW_PIP_FUSE_STAMPS=1 timeout -k 10 60 python -u tools/ab_batch_latency.py 60 > gpurun_out/r04ag_stamps.txt 2>&1 || { tail -5 gpurun_out/r04ag_stamps.txt; exit 1; }
tail -4 gpurun_out/r04ag_stamps.txt
for f in 1 0 1 0; do NW_PIP_FUSE=$f timeout -k 10 60 python -u tools/ab_batch_latency.py 400 2>&1 | sed "s/^/fuse=$f /" || exit 1; done | tee gpurun_out/r04ag_ab.txt
