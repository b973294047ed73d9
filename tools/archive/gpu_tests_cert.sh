set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 400 python bench.py --workload cert --no-cpu-baseline > gpurun_out/cert.json 2> gpurun_out/cert.err || { tail -20 gpurun_out/cert.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/cert.json').read().splitlines()[-1])
for k in ['cert_stream','cert_stream_invalid']:
  for N,r in d[k].items(): print(k,N,round(r['certs_per_s']/1e6,2),r['parity'],r.get('vs_all_valid'))"
