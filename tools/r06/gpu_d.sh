# Round 6: inputs written by the CPU into host-mapped fine-grained VRAM (NW_SMALL_VRAM for the
# small-job kernel, NW_BATCH_VRAM for config 1's lone fused batch): parity files in child
# processes, then config-1 one-call latency and the service leg A/B (alternating), then the
# strict ladder's addition variants (NW_ADD_NEGC, NW_PF_SWAP) in one process.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 590 --timeout-method thread tests/test_gpu_small_vram.py > $O/vram_tests.log 2>&1 || { tail -40 $O/vram_tests.log; exit 1; }
tail -4 $O/vram_tests.log
for i in 1 2 3; do
  for v in 0 1; do
    NW_BATCH_VRAM=$v NW_BENCH_DETAIL=$O/batch_${v}_$i.json timeout -k 10 200 python -u bench.py --workload batch --no-cpu-baseline > $O/batch_${v}_$i.line 2> $O/batch_${v}_$i.err || { tail -20 $O/batch_${v}_$i.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/batch_${v}_$i.json'))
b=d['verify_batch_10k']
print('batch vram=$v run $i', {k: b.get(k) for k in ('latency_ms','latency_ms_mean','verifies_per_s_resident')}, 'parity', d['parity'])
"
  done
done
for i in 1 2; do
  for v in 0 1; do
    NW_SMALL_VRAM=$v NW_BENCH_DETAIL=$O/svc_${v}_$i.json timeout -k 10 300 python -u bench.py --workload service > $O/svc_${v}_$i.line 2> $O/svc_${v}_$i.err || { tail -20 $O/svc_${v}_$i.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/svc_${v}_$i.json'))['service_latency']
for k,v in d.items():
  for x in v['loads']:
    print('svc vram=$v run $i', k, int(x['offered_certs_per_s']), {kk: (round(vv,3) if isinstance(vv,float) else vv) for kk,vv in x.items() if kk in ('p50_ms','p99_ms','max_ms','hedged','host_first','producer_lag_max_ms','pipeline_jobs')})
"
  done
done
timeout -k 10 400 python -u tools/strict_variants.py --reps 6 narwhal_amd/libnarwhal_amd.so tools/r06/var/negc/libnarwhal_amd.so tools/r06/var/swapnegc/libnarwhal_amd.so > $O/negc_ab.jsonl 2> $O/negc_ab.err || { tail -20 $O/negc_ab.err; exit 1; }
cat $O/negc_ab.jsonl
