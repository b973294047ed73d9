# Round 5: the default bench twice with the service's per-job timeline and the job staging
# growth log (NW_SERVICE_DEBUG=<path>), an extra 10^6 run per committee: where does the
# occasional 30-45 ms service stall at 10^6 certs/s come from.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
for r in 1 2; do
NW_SERVICE_DEBUG=$PWD/$O/svc$r NW_BENCH_DETAIL=$O/detail$r.json timeout -k 10 300 python -u bench.py --service-rates 1000,10000,100000,1000000,1000000 > $O/bench$r.json 2> $O/bench$r.err || { tail -20 $O/bench$r.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/detail$r.json'))
for k,v in d['service_latency'].items():
  for x in v['loads']:
    print(k, int(x['offered_certs_per_s']), 'p50 %.2f p90 %.2f p99 %.2f max %.2f'%(x['p50_ms'],x['p90_ms'],x['p99_ms'],x['max_ms']), 'jobs',x['jobs'], 'lagmax %.2f callmax %.0f first10 %.2f'%(x['producer_lag_max_ms'],x['call_max_us'],x['slowest1pct_in_first_tenth']))
"
done
