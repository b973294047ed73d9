set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_fuzz.py > gpurun_out/r04ac_tests.log 2>&1 || { tail -30 gpurun_out/r04ac_tests.log; exit 1; }
tail -1 gpurun_out/r04ac_tests.log
NW_PIP_PREFETCH=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch.py > gpurun_out/r04ac_tests_pf3.log 2>&1 || { tail -30 gpurun_out/r04ac_tests_pf3.log; exit 1; }
tail -1 gpurun_out/r04ac_tests_pf3.log
for cfg in "1 99" "2 99" "3 99" "1 3" "3 3" "1 5" "3 5" "1 99" "3 99"; do
  set -- $cfg
  NW_PIP_PREFETCH=$1 NW_PIP_LG=$2 timeout -k 10 60 python -u tools/ab_batch_latency.py 400 2>&1 | sed "s/^/pf=$1 lg=$2 /" || exit 1
done | tee gpurun_out/r04ac_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04ac_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_batch_latency.py 200 > $GRAFT_REPO_ROOT/gpurun_out/r04ac_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04ac_prof.log; exit 1; }
NW_PIP_PREFETCH=3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04ac_prof_pf3 -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_batch_latency.py 200 > $GRAFT_REPO_ROOT/gpurun_out/r04ac_prof_pf3.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04ac_prof_pf3.log; exit 1; }
echo done
