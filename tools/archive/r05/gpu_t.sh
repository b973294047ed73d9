# Round 5: packed per-lane strict tables as the default: same-process A/B (the unpacked
# build, the packed variant with the 40 KB prefetch slots, the new default), the strict and
# batch GPU tests, smoke, then the strict launch's HBM traffic (FETCH_SIZE / WRITE_SIZE
# passes, one bench-size launch each).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 400 python -u tools/strict_variants.py --reps 4 --steps 4 var/unpacked/libnarwhal_amd.so narwhal_amd/libnarwhal_amd.so var/pack/libnarwhal_amd.so > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_messages.py tests/test_gpu_distributed.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
A="--steps 1 --warmup 0 --no-sha --no-cert --no-batch --no-wire --no-service --no-worker --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- python3 bench.py $A > $O/pmc_fetch.json 2> $O/pmc_fetch.log || { tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- python3 bench.py $A > $O/pmc_write.json 2> $O/pmc_write.log || { tail -5 $O/pmc_write.log; exit 1; }
echo pmc ok
