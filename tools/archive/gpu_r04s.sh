# Round 4 full check: the -m gpu suite, smoke(), the default bench line, its rocprof summary.
set -o pipefail
export TMPDIR=/tmp
: timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04s_gputests.log 2>&1 || { tail -30 gpurun_out/r04s_gputests.log; exit 1; }
: tail
: timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04s_smoke.log 2>&1 || { tail -20 gpurun_out/r04s_smoke.log; exit 1; }
: tail
T0=$(date +%s); timeout -k 10 600 python -u bench.py > gpurun_out/r04s_bench.json 2> gpurun_out/r04s_bench.err || { tail -20 gpurun_out/r04s_bench.err; exit 1; }
echo "bench seconds: $(( $(date +%s) - T0 ))"
