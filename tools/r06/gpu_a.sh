# Round 6, first GPU check: the new GPU tests (16-bit key-comb fallback, the 8-rank gloo
# bench rehearsal), the full -m gpu suite, smoke and the default bench line (its
# cpu_baseline legs now the dalek-equivalent restatement).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hedge.py tests/test_gpu_memory.py tests/test_bench_line.py -m gpu -v --timeout 280 --timeout-method thread > $O/newtests.log 2>&1 || { tail -60 $O/newtests.log; exit 1; }
tail -6 $O/newtests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
NW_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); s=d['summary']; print(len(open('$O/bench.json').read()), d['value'], d['parity'], d['roofline']['frac'], d['cpu_baseline'], s['batch10k'], s['cert_stream_Mcerts_s'], s['cert_cpu_certs_s'], s['sha512']['GB_s'], s['service'])"
