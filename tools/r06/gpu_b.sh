# Round 6: the service with the reworked hedge (device batches always hedged, host-only
# batches budgeted, 6 threads), twice; the host path's rate on the box's cores; the strict
# kernel's per-phase split (PMC of the phase-cut builds); then the BAR stall probe (last:
# the one step that may fault on the host side).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 120 python -u tools/host_path_rate.py 4,10,50,100 > $O/host_path_rate.json 2> $O/host_path_rate.err || { tail -20 $O/host_path_rate.err; exit 1; }
cat $O/host_path_rate.json
for i in 1 2; do
  NW_BENCH_DETAIL=$O/svc_$i.json timeout -k 10 300 python -u bench.py --workload service > $O/svc_$i.line 2> $O/svc_$i.err || { tail -20 $O/svc_$i.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/svc_$i.json'))['service_latency']
for k,v in d.items():
  for x in v['loads']:
    print('run $i', k, int(x['offered_certs_per_s']), {kk: (round(vv,3) if isinstance(vv,float) else vv) for kk,vv in x.items() if kk in ('p50_ms','p99_ms','max_ms','hedged','host_first','host_only_batches','producer_lag_max_ms','pipeline_jobs')})
"
done
timeout -k 10 1200 bash tools/strict_phases_pmc.sh $O/strict_phases > $O/strict_phases.log 2>&1 || { tail -20 $O/strict_phases.log; exit 1; }
cat $O/strict_phases.log
python3 tools/strict_phases_summary.py $O/strict_phases $O/strict_phases.json || true
timeout -k 10 60 ./tools/ubench/bar_probe 30 > $O/bar_probe.jsonl 2> $O/bar_probe.err; echo "bar_probe rc=$?"
cat $O/bar_probe.jsonl | cut -c1-600
