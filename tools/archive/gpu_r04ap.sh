set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_fuzz.py > gpurun_out/r04ap_tests.log 2>&1 || { tail -40 gpurun_out/r04ap_tests.log; exit 1; }
tail -1 gpurun_out/r04ap_tests.log
NW_PIP_FUSE_HEAD=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py -k "fused or config1" > gpurun_out/r04ap_tests_nohead.log 2>&1 || { tail -40 gpurun_out/r04ap_tests_nohead.log; exit 1; }
tail -1 gpurun_out/r04ap_tests_nohead.log
for i in 1 2 3; do timeout -k 10 60 python -u tools/ab_batch_latency.py 400 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04ap_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_batch_latency.py 200 > $GRAFT_REPO_ROOT/gpurun_out/r04ap_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04ap_prof.log; exit 1; }
echo done
