set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_fuzz.py > gpurun_out/r04aj_tests.log 2>&1 || { tail -40 gpurun_out/r04aj_tests.log; exit 1; }
tail -1 gpurun_out/r04aj_tests.log
NW_PIP_FUSE_STAMPS=1 timeout -k 10 60 python -u tools/ab_batch_latency.py 40 > gpurun_out/r04aj_stamps.txt 2>&1 || { tail -5 gpurun_out/r04aj_stamps.txt; exit 1; }
tail -6 gpurun_out/r04aj_stamps.txt
for k in 4 1 2 8 4 1 2 8; do NW_PIP_SORT_SPLIT=$k timeout -k 10 60 python -u tools/ab_batch_latency.py 400 2>&1 | sed "s/^/split=$k /" || exit 1; done | tee gpurun_out/r04aj_ab.txt
NW_PIP_FUSE=0 timeout -k 10 60 python -u tools/ab_batch_latency.py 400 2>&1 | sed "s/^/fuse=0 /" | tee -a gpurun_out/r04aj_ab.txt
