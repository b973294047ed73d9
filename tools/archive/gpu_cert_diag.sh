set -o pipefail
mkdir -p gpurun_out
export NW_DEBUG_GROUPS=1
timeout -k 10 400 python bench.py --workload cert --committees 4,10,50,100 --no-cpu-baseline > gpurun_out/cert.json 2> gpurun_out/cert.err || { tail -20 gpurun_out/cert.err; exit 1; }
grep narwhal_amd gpurun_out/cert.err | head -30
python3 -c "
import json
for f in ['gpurun_out/cert.json']:
  d=json.loads(open(f).read().splitlines()[-1])
  for k in ['cert_stream','cert_stream_invalid']:
    for N,r in d[k].items(): print(f,k,N,round(r['certs_per_s']/1e6,2),r['parity'],r.get('vs_all_valid'))"
