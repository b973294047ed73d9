# Round 5: (1) lp_mul by one row rotate per term (nw_lp.hpp NW_LP_ROR): the batch and
# small-job GPU tests, config-1 latency; (2) 20 s of steady 10^4 N=50 certificates/s through
# the service with the per-job timeline: are the rare 5-30 ms completion stalls periodic?
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_small.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NW_BENCH_DETAIL=$O/batch_detail.json timeout -k 10 300 python -u bench.py --workload batch --steps 20 --no-cpu-baseline > $O/batch.json 2> $O/batch.err || { tail -20 $O/batch.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/batch_detail.json'))['verify_batch_10k']; print('config1 latency ms', d['latency_ms'], 'mean', d['latency_ms_mean'], 'resident M/s', d['verifies_per_s_resident']/1e6, d['parity'])"
NW_PIP_FUSE_STAMPS=1 timeout -k 10 200 python -u bench.py --workload batch --steps 3 --no-cpu-baseline > /dev/null 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
grep -E "^\[(head|fuse)\]" $O/stamps.err | tail -6
NW_SERVICE_DEBUG=$PWD/$O/svc NW_BENCH_DETAIL=$O/svc_detail.json timeout -k 10 300 python -u bench.py --workload service --service-committees 50 --service-rates 10000 --service-seconds 20 --service-max-certs 200000 > $O/svc.json 2> $O/svc.err || { tail -20 $O/svc.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/svc_detail.json'))
for k,v in d['service_latency'].items():
  for x in v['loads']:
    print(k, int(x['offered_certs_per_s']), 'p50 %.2f p90 %.2f p99 %.2f max %.2f'%(x['p50_ms'],x['p90_ms'],x['p99_ms'],x['max_ms']), 'jobs',x['jobs'])
"
