# Sustained 20 s N = 50 service runs at 10^6/s with the per-job timeline (NW_SERVICE_DEBUG),
# summarised per second by tools/service_timeline.py (the raw CSVs are not kept).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05tl; mkdir -p $O
for i in 1 2 3 4; do
  NW_SERVICE_DEBUG=$PWD/$O/tl_$i NW_BENCH_DETAIL=$O/svc_$i.json timeout -k 10 170 python -u bench.py --workload service --service-committees 50 --service-rates 1000000 --service-seconds 20 --service-max-certs 20000000 > $O/svc_$i.line 2> $O/svc_$i.err || { tail -20 $O/svc_$i.err; exit 1; }
  python3 -c "
import json
x=json.load(open('$O/svc_$i.json'))['service_latency']['N50']['loads'][0]
print('run $i', {k: (round(v,3) if isinstance(v,float) else v) for k,v in x.items() if k in ('p50_ms','p90_ms','p99_ms','max_ms','producer_lag_max_ms','pipeline_jobs','call_max_us','calls_over_20us','cgroup_throttled_periods')})
"
  # one CSV per service the run created: the native load's (the most jobs) is the one kept
  best=$(for f in $O/tl_$i.*.csv; do case $f in *.grow.csv) ;; *) echo "$(wc -l < $f) $f";; esac; done | sort -n | tail -1 | cut -d' ' -f2)
  python3 tools/service_timeline.py $best --bin 0.5 > $O/tl_$i.summary.json || exit 1
  rm -f $O/tl_$i.*.csv
  python3 -c "
import json
d=json.load(open('$O/tl_$i.summary.json'))
print('jobs', d['jobs'], d['by_submitter'], d['stages_us'])
for r in d['per_bin']:
    if r['wait_us'][1] > 2000 or r['submit_us'][1] > 2000 or r['device_us'][1] > 2000 or r['certs_per_job'] > 300: print(r)
"
done
