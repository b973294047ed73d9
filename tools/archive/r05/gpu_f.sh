# Round 5: (1) host facts that can stall a process (NUMA balancing, THP, CPU quota);
# (2) 20 s of 10^4 N=50 certificates/s with a clock-gap monitor thread beside the service's
# per-job timeline: do the device "stalls" coincide with the whole process not running?
# (3) config 1 with the fused launches' LDS reservation at 96 / 64 / 48 KB (1 / 2 / 3
# workgroups per CU), stamps on.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
{ echo "numa_balancing $(cat /proc/sys/kernel/numa_balancing 2>&1)"; echo "thp $(cat /sys/kernel/mm/transparent_hugepage/enabled 2>&1)"; echo "thp_defrag $(cat /sys/kernel/mm/transparent_hugepage/defrag 2>&1)"; echo "cpu.max $(cat /sys/fs/cgroup/cpu.max 2>&1)"; echo "cpu.stat"; cat /sys/fs/cgroup/cpu.stat 2>&1; echo "nproc $(nproc)"; } > $O/host.txt
cat $O/host.txt
NW_LOADGEN_GAPS=$PWD/$O/gaps.csv NW_SERVICE_DEBUG=$PWD/$O/svc NW_BENCH_DETAIL=$O/svc_detail.json timeout -k 10 300 python -u bench.py --workload service --service-committees 50 --service-rates 10000 --service-seconds 20 --service-max-certs 200000 > $O/svc.json 2> $O/svc.err || { tail -20 $O/svc.err; exit 1; }
echo "cpu.stat after"; cat /sys/fs/cgroup/cpu.stat 2>&1
wc -l $O/gaps.csv || true
for lds in 98304 65536 49152; do
NW_PIP_FUSE_LDS=$lds NW_BENCH_DETAIL=$O/batch_$lds.json timeout -k 10 300 python -u bench.py --workload batch --steps 10 --no-cpu-baseline > /dev/null 2> $O/batch_$lds.err || { tail -20 $O/batch_$lds.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/batch_$lds.json'))['verify_batch_10k']; print('lds=$lds config1 latency ms %.4f mean %.4f %s' % (d['latency_ms'], d['latency_ms_mean'], d['parity']))"
NW_PIP_FUSE_LDS=$lds NW_PIP_FUSE_STAMPS=1 timeout -k 10 200 python -u bench.py --workload batch --steps 3 --no-cpu-baseline > /dev/null 2> $O/stamps_$lds.err || { tail -20 $O/stamps_$lds.err; exit 1; }
grep -E "^\[(head|fuse)\]" $O/stamps_$lds.err | tail -4
done
