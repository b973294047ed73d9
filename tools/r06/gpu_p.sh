# Round 6: N = 50 at 10^3 certs/s hedges ~1 % of its requests (device jobs > 1 ms spread over
# the run, not at its start). Are the 20-bit committee combs (47 GB at N = 50, random table
# pages per vote) the cause? The service leg with NW_KEY_WIDTH=16 (3.4 GB) against the
# default, alternating, two pairs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p; mkdir -p $O
for i in 1 2; do
  for w in 16 0; do
    if [ $w = 16 ]; then export NW_KEY_WIDTH=16; else unset NW_KEY_WIDTH; fi
    NW_BENCH_DETAIL=$O/svc_${w}_$i.json timeout -k 10 300 python -u bench.py --workload service > $O/svc_${w}_$i.line 2> $O/svc_${w}_$i.err || { tail -20 $O/svc_${w}_$i.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/svc_${w}_$i.json'))['service_latency']
for k,v in d.items():
  for x in v['loads']:
    print('width=$w run $i', k, int(x['offered_certs_per_s']), {kk: (round(vv,3) if isinstance(vv,float) else vv) for kk,vv in x.items() if kk in ('p50_ms','p99_ms','max_ms','hedged','host_first','host_only_batches','producer_lag_max_ms')})
"
  done
done
