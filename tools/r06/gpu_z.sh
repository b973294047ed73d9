# Round 6: r06x's sequence again (10 s of N = 50 at 10^6 natively, then the asyncio legs, whose
# 10^4 leg reported parity FAIL there), now with the asyncio leg's first mismatches recorded.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
for i in 1 2; do
  NW_BENCH_DETAIL=$O/svc_$i.json timeout -k 10 240 python -u bench.py --workload service --service-committees 50 --service-rates 1000000 --service-seconds 10 --service-max-certs 10000000 > $O/svc_$i.line 2> $O/svc_$i.err || true
  python3 -c "
import json
d=json.load(open('$O/svc_$i.json'))['service_latency']['N50']
for x in d['loads']: print('native', {k: x.get(k) for k in ('certs','p50_ms','p99_ms','max_ms','hedged','host_first','parity')})
for x in d['python_asyncio']['loads']: print('asyncio', {k: x.get(k) for k in ('offered_certs_per_s','certs','jobs','parity','mismatches','first_mismatches')})
" || exit 1
done
