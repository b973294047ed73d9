# Round 5: batch / small-job GPU tests on the lp code (two MAC chains, old carry); config-1
# latency: one MAC chain (var/ch1) vs two (in-tree); the Horner wave at issue priority 3
# (var/p3) with 1 / 2 / 3 workgroups per CU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_small.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # $1 label, env assignments follow via env
NW_BENCH_DETAIL=$O/b.json timeout -k 10 300 python -u bench.py --workload batch --steps 10 --no-cpu-baseline > /dev/null 2> $O/b.err || { tail -20 $O/b.err; return 1; }
python3 -c "import json; d=json.load(open('$O/b.json'))['verify_batch_10k']; print('$1 config1 latency ms %.4f mean %.4f resident %.1f M/s %s' % (d['latency_ms'], d['latency_ms_mean'], d['verifies_per_s_resident']/1e6, d['parity']))"
}
for r in 1 2; do
NW_LIB=$PWD/var/ch1/libnarwhal_amd.so run "chains=1" || exit 1
run "chains=2" || exit 1
done
for lds in 98304 65536 49152; do
NW_PIP_FUSE_LDS=$lds run "lds=$lds prio=0" || exit 1
NW_PIP_FUSE_LDS=$lds NW_LIB=$PWD/var/p3/libnarwhal_amd.so run "lds=$lds prio=3" || exit 1
done
