# Service sustained load: jobs prewarmed to max_items; alternating 20 s N = 50 service runs
# with max_items 32,768 vs 1,048,576 units (a backlogged batch's size bound).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05mi; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_service.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3 4; do
  for mi in 32768 1048576; do
    NW_BENCH_DETAIL=$O/svc_m${mi}_$i.json timeout -k 10 170 python -u bench.py --workload service --service-committees 50 --service-rates 10000,1000000 --service-seconds 20 --service-max-certs 20000000 --service-max-items $mi > $O/svc_m${mi}_$i.line 2> $O/svc_m${mi}_$i.err || { tail -20 $O/svc_m${mi}_$i.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/svc_m${mi}_$i.json'))['service_latency']['N50']
print('max_items=$mi run $i', [(int(x['offered_certs_per_s']), round(x['p50_ms'],3), round(x['p90_ms'],3), round(x['p99_ms'],3), round(x['max_ms'],2), x['pipeline_jobs'], round(x['certs_per_job'],1), round(x['producer_lag_max_ms'],2)) for x in d['loads']], d['parity'])
"
  done
done
