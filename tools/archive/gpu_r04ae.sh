set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py > gpurun_out/r04ae_tests.log 2>&1 || { tail -40 gpurun_out/r04ae_tests.log; exit 1; }
tail -1 gpurun_out/r04ae_tests.log
for cfg in "1 98304" "0 0" "1 0" "1 98304" "0 0" "1 0"; do
  set -- $cfg
  NW_PIP_FUSE=$1 NW_PIP_FUSE_LDS=$2 timeout -k 10 60 python -u tools/ab_batch_latency.py 400 2>&1 | sed "s/^/fuse=$1 lds=$2 /" || exit 1
done | tee gpurun_out/r04ae_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04ae_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_batch_latency.py 200 > $GRAFT_REPO_ROOT/gpurun_out/r04ae_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04ae_prof.log; exit 1; }
echo done
