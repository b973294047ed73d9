# GPU-box helper: the whole -m gpu suite, then the default bench line (N=1).
#   bash tools/gpu_full.sh TAG   -> gpurun_out/gputests_TAG.log, gpurun_out/bench_TAG.json
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1 || { tail -40 gpurun_out/gputests_$TAG.log; exit 1; }
tail -2 gpurun_out/gputests_$TAG.log
NW_DEBUG_GROUPS=1 timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 - $TAG <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/bench_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print('strict', round(d['value']/1e6,2), 'parity', d['parity'], 'sha', round(d['sha512']['GB_per_s'],1))
for leg in ('cert_stream','cert_stream_invalid'):
  for n,v in d[leg].items(): print(leg,n,round(v['certs_per_s']/1e6,2), v.get('vs_all_valid'), v['parity'])
b=d['verify_batch_10k']; print('batch10k', round(b['latency_ms'],3), round(b['verifies_per_s_resident']/1e6,1))
PY
