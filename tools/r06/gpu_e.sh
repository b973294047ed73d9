# Round 6: more same-box evidence before choosing defaults — the strict ladder variants
# (NW_ADD_NEGC / NW_PF_SWAP) at 10 rounds, the service leg with small-job inputs in VRAM
# (NW_SMALL_VRAM) three more alternating pairs, config 1 with the new default (inputs in
# VRAM) against NW_BATCH_VRAM=0 twice more.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 500 python -u tools/strict_variants.py --reps 10 narwhal_amd/libnarwhal_amd.so tools/r06/var/swapnegc/libnarwhal_amd.so tools/r06/var/negc/libnarwhal_amd.so > $O/negc_ab.jsonl 2> $O/negc_ab.err || { tail -20 $O/negc_ab.err; exit 1; }
cat $O/negc_ab.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 890 --timeout-method thread tests/test_gpu_small_vram.py > $O/vram_tests.log 2>&1 || { tail -40 $O/vram_tests.log; exit 1; }
tail -5 $O/vram_tests.log
for i in 1 2 3; do
  for v in g 1 0; do
    if [ $v = g ]; then export NW_BATCH_GATE=1 NW_BATCH_VRAM=1; else export NW_BATCH_GATE=0 NW_BATCH_VRAM=$v; fi
    NW_BENCH_DETAIL=$O/batch_${v}_$i.json timeout -k 10 200 python -u bench.py --workload batch --no-cpu-baseline > $O/batch_${v}_$i.line 2> $O/batch_${v}_$i.err || { tail -20 $O/batch_${v}_$i.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/batch_${v}_$i.json'))
b=d['verify_batch_10k']
print('batch mode=$v run $i', {k: b.get(k) for k in ('latency_ms','latency_ms_mean','verifies_per_s_resident')}, 'parity', d['parity'])
"
  done
done
unset NW_BATCH_GATE NW_BATCH_VRAM
for i in 1 2 3; do
  for v in 1 0; do
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
