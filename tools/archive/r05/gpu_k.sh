# Round 5 mid-round check: the whole -m gpu suite, the long irregular-committee fuzz
# (60 seeds), the default bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 900 python -u tools/fuzz_long.py 0 60 irregular > $O/fuzz_irregular.json 2> $O/fuzz_irregular.err || { tail -20 $O/fuzz_irregular.err; exit 1; }
cut -c1-600 $O/fuzz_irregular.json
NW_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['parity'], d['summary']['batch10k'], d['summary']['service'])"
