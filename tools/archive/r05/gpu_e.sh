# Round 5: config-1 inputs read straight from the pinned buffer + self-clearing fused
# counters (tests, latency A/B against NW_BATCH_PINNED=0); a 20 s completion-stall probe
# with a trivial kernel; the 20 s 10^4 N=50 service run again with prewarmed job counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_small.py tests/test_gpu_fanout.py tests/test_gpu_streams.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0 1 0; do
NW_BATCH_PINNED=$v NW_BENCH_DETAIL=$O/batch_$v.json timeout -k 10 300 python -u bench.py --workload batch --steps 10 --no-cpu-baseline > /dev/null 2> $O/batch_$v.err || { tail -20 $O/batch_$v.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/batch_$v.json'))['verify_batch_10k']; print('pinned=$v config1 latency ms %.4f mean %.4f %s' % (d['latency_ms'], d['latency_ms_mean'], d['parity']))"
done
timeout -k 10 120 python -u tools/stall_probe.py 20 > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cut -c1-600 $O/probe.json
NW_SERVICE_DEBUG=$PWD/$O/svc NW_BENCH_DETAIL=$O/svc_detail.json timeout -k 10 300 python -u bench.py --workload service --service-committees 50 --service-rates 10000 --service-seconds 20 --service-max-certs 200000 > $O/svc.json 2> $O/svc.err || { tail -20 $O/svc.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/svc_detail.json'))
for k,v in d['service_latency'].items():
  for x in v['loads']:
    print(k, int(x['offered_certs_per_s']), 'p50 %.2f p90 %.2f p99 %.2f max %.2f'%(x['p50_ms'],x['p90_ms'],x['p99_ms'],x['max_ms']), 'jobs',x['jobs'])
"
