# Round 5: (1) the stall probe with device / pinned-read / H2D-copy operations interleaved
# (the same host conditions for all three), 30 s; (2) config-1 latency for the lp carry /
# MAC-chain variants (var/c1: old carry, one chain; var/c2: new carry, one chain; in-tree:
# new carry, two chains), alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 200 python -u tools/stall_probe.py 30 mixed > $O/probe_mixed.json 2> $O/probe_mixed.err || { tail -20 $O/probe_mixed.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/probe_mixed.json'))
for k in ('device','pinned','copy'): print(k, 'p50 %.3f p99 %.3f max %.2f n_over_1ms %d' % (d[k]['p50_ms'], d[k]['p99_ms'], d[k]['max_ms'], len(d[k]['over_1ms'])), d[k]['over_1ms'][:8])
"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_small.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for v in var/c1 var/c2 narwhal_amd; do
NW_LIB=$PWD/$v/libnarwhal_amd.so NW_BENCH_DETAIL=$O/b.json timeout -k 10 300 python -u bench.py --workload batch --steps 10 --no-cpu-baseline > /dev/null 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json'))['verify_batch_10k']; print('$v config1 latency ms %.4f mean %.4f resident %.1f M/s %s' % (d['latency_ms'], d['latency_ms_mean'], d['verifies_per_s_resident']/1e6, d['parity']))"
done; done
# (3) the Horner wave at issue priority 3 (var/p3) with 1 / 2 / 3 workgroups per CU
for lds in 98304 65536 49152; do for v in narwhal_amd var/p3; do
NW_PIP_FUSE_LDS=$lds NW_LIB=$PWD/$v/libnarwhal_amd.so NW_BENCH_DETAIL=$O/b.json timeout -k 10 300 python -u bench.py --workload batch --steps 10 --no-cpu-baseline > /dev/null 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json'))['verify_batch_10k']; print('lds=$lds $v config1 latency ms %.4f mean %.4f resident %.1f M/s %s' % (d['latency_ms'], d['latency_ms_mean'], d['verifies_per_s_resident']/1e6, d['parity']))"
done; done
