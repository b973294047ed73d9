# Round 6: sustained load with the final defaults (small jobs on 16-bit combs, done flags,
# retiring jobs, hedge): N = 50 at 10^6 certs/s for 10 s, done flags on vs off, alternating,
# two pairs (round 5's sustained runs collapsed in about half the cases).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
for i in 1 2; do
  for v in 1 0; do
    NW_SMALL_DONE=$v NW_BENCH_DETAIL=$O/svc_${v}_$i.json timeout -k 10 240 python -u bench.py --workload service --service-committees 50 --service-rates 1000000 --service-seconds 10 --service-max-certs 10000000 > $O/svc_${v}_$i.line 2> $O/svc_${v}_$i.err || { tail -20 $O/svc_${v}_$i.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/svc_${v}_$i.json'))['service_latency']
for k,v in d.items():
  for x in v['loads']:
    print('done=$v run $i', k, int(x['offered_certs_per_s']), x.get('certs'), {kk: (round(vv,3) if isinstance(vv,float) else vv) for kk,vv in x.items() if kk in ('achieved_certs_per_s','p50_ms','p90_ms','p99_ms','max_ms','hedged','host_first','producer_lag_max_ms','pipeline_jobs')})
"
  done
done
