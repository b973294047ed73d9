# Round 5 (session 2) round-end check: sustained 20 s N = 50 service runs at 10^6/s with the
# cgroup's CPU throttling recorded (bench.py cgroup_cpu_stat), then the full -m gpu suite,
# smoke and the default bench line of the final tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05final4; mkdir -p $O
cat /sys/fs/cgroup/cpu.max > $O/cgroup.txt 2>&1 || true
nproc >> $O/cgroup.txt 2>&1 || true
for i in 1 2 3; do
  NW_BENCH_DETAIL=$O/svc_$i.json timeout -k 10 170 python -u bench.py --workload service --service-committees 50 --service-rates 1000000 --service-seconds 20 --service-max-certs 20000000 > $O/svc_$i.line 2> $O/svc_$i.err || { tail -20 $O/svc_$i.err; exit 1; }
  python3 -c "
import json
x=json.load(open('$O/svc_$i.json'))['service_latency']['N50']['loads'][0]
print('run $i', {k: (round(v,3) if isinstance(v,float) else v) for k,v in x.items() if k in ('p50_ms','p90_ms','p99_ms','max_ms','producer_lag_max_ms','pipeline_jobs','cgroup_cpus_used','cgroup_throttled_periods','cgroup_throttled_ms','producer_cpu_per_wall','producer_ivcsw')})
"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
NW_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); s=d['summary']; print(len(open('$O/bench.json').read()), d['value'], d['parity'], d['roofline']['frac'], s['batch10k'], s['cert_stream_Mcerts_s'], s['sha512']['GB_s'], s['service'])
dd=json.load(open('$O/bench_detail.json'))['service_latency']
for k,v in dd.items():
  print(k, [(int(x['offered_certs_per_s']), x.get('cgroup_throttled_periods'), round(x.get('cgroup_throttled_ms') or 0,1), round(x.get('cgroup_cpus_used') or 0,2)) for x in v['loads']])
"
