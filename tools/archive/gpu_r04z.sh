# Round 4 final check: the -m gpu suite, smoke(), the default bench line (N=1), a kernel
# trace of the same bench. Each step under its own limit; stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r04z_gputests.log 2>&1 || { tail -30 gpurun_out/r04z_gputests.log; exit 1; }
tail -2 gpurun_out/r04z_gputests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04z_smoke.log 2>&1 || { tail -20 gpurun_out/r04z_smoke.log; exit 1; }
tail -1 gpurun_out/r04z_smoke.log
T0=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/r04z_bench.json 2> gpurun_out/r04z_bench.err || { tail -20 gpurun_out/r04z_bench.err; exit 1; }
echo "bench seconds: $(( $(date +%s) - T0 ))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04z_trace -o p -- python3 bench.py --no-cpu-baseline > gpurun_out/r04z_bench_traced.json 2> gpurun_out/r04z_bench_traced.log || { echo "trace failed"; exit 1; }
echo "trace ok"
