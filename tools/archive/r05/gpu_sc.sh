# Service tail A/B: the small-job kernel over pinned host memory (default) vs device copies
# (NW_SMALL_COPY=1). Parity of the small-job and service tests with copies, the completion
# stall probe (device / pinned-host kernel / H2D copy interleaved), then alternating 20 s
# N = 50 service runs at 10^4 and 10^6 certificates/s.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05sc; mkdir -p $O
NW_SMALL_COPY=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py tests/test_service.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_copy.log 2>&1 || { tail -40 $O/tests_copy.log; exit 1; }
tail -2 $O/tests_copy.log
for i in 1 2 3; do
  timeout -k 10 170 python -u tools/stall_probe.py 120 mixed > $O/probe_$i.jsonl 2> $O/probe_$i.err || { tail -5 $O/probe_$i.err; exit 1; }
  python3 -c "
import json
for l in open('$O/probe_$i.jsonl'):
    d=json.loads(l); print({k:v for k,v in d.items() if not isinstance(v,list)}, 'slow', len(d.get('slow',[])))
" || true
done
for i in 1 2 3 4; do
  for c in 0 1; do
    NW_SMALL_COPY=$c NW_BENCH_DETAIL=$O/svc_c${c}_$i.json timeout -k 10 170 python -u bench.py --workload service --service-committees 50 --service-rates 10000,1000000 --service-seconds 20 --service-max-certs 20000000 > $O/svc_c${c}_$i.line 2> $O/svc_c${c}_$i.err || { tail -20 $O/svc_c${c}_$i.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/svc_c${c}_$i.json'))['service_latency']['N50']
print('copy=$c run $i', [(int(x['offered_certs_per_s']), round(x['p50_ms'],3), round(x['p99_ms'],3), round(x['max_ms'],2), x['pipeline_jobs'], round(x['producer_lag_max_ms'],2)) for x in d['loads']], d['parity'])
"
  done
done
