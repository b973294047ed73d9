# Round 5: (1) do the service's 1-10 ms HIP-side stalls (every thread that calls HIP freezes,
# a clock-only thread does not, profiles/r05f) depend on streams sharing the 4 hardware
# queues? 20 s at 10^4 N=50 certs/s with GPU_MAX_HW_QUEUES 4 (default) and 16;
# (2) config-1 latency with the poll-before-block wait (NW_WAIT_SPIN_US=5000 default vs 0).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
for q in 4 16; do
GPU_MAX_HW_QUEUES=$q NW_LOADGEN_GAPS=$PWD/$O/gaps_$q.csv NW_SERVICE_DEBUG=$PWD/$O/svc_q$q NW_BENCH_DETAIL=$O/svc_q$q.json timeout -k 10 300 python -u bench.py --workload service --service-committees 50 --service-rates 10000 --service-seconds 20 --service-max-certs 200000 > /dev/null 2> $O/svc_q$q.err || { tail -20 $O/svc_q$q.err; exit 1; }
python3 -c "
import json
x=json.load(open('$O/svc_q$q.json'))['service_latency']['N50']['loads'][0]
print('queues=$q', 'p50 %.3f p99 %.3f max %.2f lagmax %.2f callmax %.0f' % (x['p50_ms'], x['p99_ms'], x['max_ms'], x['producer_lag_max_ms'], x['call_max_us']))
"
done
for sp in 5000 0 5000 0; do
NW_WAIT_SPIN_US=$sp NW_BENCH_DETAIL=$O/batch_$sp.json timeout -k 10 300 python -u bench.py --workload batch --steps 10 --no-cpu-baseline > /dev/null 2> $O/batch_$sp.err || { tail -20 $O/batch_$sp.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/batch_$sp.json'))['verify_batch_10k']; print('spin=$sp config1 latency ms %.4f mean %.4f %s' % (d['latency_ms'], d['latency_ms_mean'], d['parity']))"
done
