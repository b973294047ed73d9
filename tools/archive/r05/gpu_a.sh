# Round 5, first check: the -m gpu suite (incl. bench --gpus 2 and the worker modes), the
# default bench line (N=1) with its compact output. Each step under its own limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
T0=$(date +%s)
NW_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench seconds: $(( $(date +%s) - T0 )) line bytes: $(wc -c < $O/bench.json)"
