# Round 5 round-end check on the final tree: the -m gpu suite, smoke, the default bench line,
# then the profile set (kernel trace of the default bench + PMC passes, tools/profile_round.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05final2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
NW_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); s=d['summary']; print(d['value'], d['parity'], d['roofline']['frac'], s['batch10k'], s['cert_stream_Mcerts_s'], s['sha512']['GB_s'])"
bash tools/profile_round.sh r05final2
