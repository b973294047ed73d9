set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/r04af_tests.log 2>&1 || { tail -40 gpurun_out/r04af_tests.log; exit 1; }
tail -1 gpurun_out/r04af_tests.log
for f in 1 0 1 0; do NW_PIP_FUSE=$f timeout -k 10 60 python -u tools/ab_batch_latency.py 400 2>&1 | sed "s/^/fuse=$f /" || exit 1; done | tee gpurun_out/r04af_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04af_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_batch_latency.py 200 > $GRAFT_REPO_ROOT/gpurun_out/r04af_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04af_prof.log; exit 1; }
echo done
