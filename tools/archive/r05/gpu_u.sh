# Round 5: the full -m gpu suite, smoke and the default bench line on the packed-table tree,
# then the kernel trace of the same bench command (rocprofv3 --kernel-trace --stats).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
NW_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); s=d['summary']; print(d['value'], d['parity'], d['roofline']['frac'], d['roofline']['traffic'], s['batch10k'], s['cert_stream_Mcerts_s'], s['sha512']['GB_s'], s['service']['N50'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o p -- python3 bench.py --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.log || { tail -5 $O/bench_traced.log; exit 1; }
echo trace ok
