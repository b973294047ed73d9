# Round 6: the -m gpu suite ended with "corrupted size vs. prev_size" (glibc heap check) at
# the pytest process's exit in r06f. Each GPU test file in its own process, stopping at the
# first non-zero exit, to find the file whose process shows it; then the suite in one process.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
for f in test_gpu_batch test_gpu_small test_service test_gpu_messages test_gpu_parity test_gpu_memory test_gpu_streams test_gpu_fanout test_wire test_worker test_gpu_fuzz test_gpu_distributed test_gpu_hedge test_gpu_small_vram test_gpu_fused_abort test_bench_line; do
  timeout -k 10 400 python -u -m pytest tests/$f.py -m gpu -q --timeout 280 --timeout-method thread > $O/$f.log 2>&1
  rc=$?
  echo "$f rc=$rc $(tail -1 $O/$f.log | cut -c1-120)"
  if [ $rc -ne 0 ]; then tail -15 $O/$f.log; exit 1; fi
  if grep -q "corrupted\|double free\|dumped core" $O/$f.log; then echo "heap message in $f"; exit 1; fi
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > $O/gputests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 $O/gputests.log
