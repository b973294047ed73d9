# Round 6: the small-job flag words poisoned with the job's own sequence number
# (NW_TEST_STALE_FLAGS=1) — the GPU test with the product library (must pass), then the small-job
# parity file against a negative-control build without the host's clearing memset
# (tools/r06/build_var.sh noclear -DNW_NO_FLAG_CLEAR nw_jobs.cpp; expected to FAIL).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ae; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_small_vram.py -v --timeout 300 --timeout-method thread -k "STALE or SMALL_DONE" > $O/stale_product.log 2>&1 || { tail -30 $O/stale_product.log; exit 1; }
tail -3 $O/stale_product.log
NW_LIB=tools/r06/var/noclear/libnarwhal_amd.so NW_TEST_STALE_FLAGS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -q --timeout 120 --timeout-method thread > $O/stale_noclear.log 2>&1
rc=$?
echo "negative control rc=$rc (1 = tests failed, as expected)"
tail -5 $O/stale_noclear.log
