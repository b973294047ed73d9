# Round 6: small jobs finish on their workgroups' done flags (NW_SMALL_DONE, default) instead
# of the completion event: the small-job GPU files both ways, then the service leg against
# NW_SMALL_DONE=0, alternating, two pairs.
set -o pipefail
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r06s}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_small.py tests/test_gpu_messages.py tests/test_service.py tests/test_gpu_fuzz.py tests/test_gpu_hedge.py tests/test_gpu_small_vram.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    NW_SMALL_DONE=$v NW_BENCH_DETAIL=$O/svc_${v}_$i.json timeout -k 10 300 python -u bench.py --workload service > $O/svc_${v}_$i.line 2> $O/svc_${v}_$i.err || { tail -20 $O/svc_${v}_$i.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/svc_${v}_$i.json'))['service_latency']
for k,v in d.items():
  for x in v['loads']:
    print('done=$v run $i', k, int(x['offered_certs_per_s']), {kk: (round(vv,3) if isinstance(vv,float) else vv) for kk,vv in x.items() if kk in ('p50_ms','p90_ms','p99_ms','max_ms','hedged','producer_lag_max_ms')})
"
  done
done
