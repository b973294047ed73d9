# Round 6: the host path in 51-bit limbs (nw_host_f51.hpp) — its rate on the box's cores, the
# forced-hedge GPU test — the service with the hedge twice, then the BAR probe (is fine-grained
# VRAM CPU-mapped; 60 s of pinned / VRAM / device reads interleaved). Also the NW_PF_SWAP A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 120 python -u tools/host_path_rate.py 4,10,50,100 > $O/host_path_rate.json 2> $O/host_path_rate.err || { tail -20 $O/host_path_rate.err; exit 1; }
cat $O/host_path_rate.json
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hedge.py > $O/hedge_test.log 2>&1 || { tail -30 $O/hedge_test.log; exit 1; }
tail -3 $O/hedge_test.log
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
timeout -k 10 300 python -u tools/strict_variants.py --reps 6 narwhal_amd/libnarwhal_amd.so tools/r06/var/swap/libnarwhal_amd.so > $O/swap_ab.jsonl 2> $O/swap_ab.err || { tail -20 $O/swap_ab.err; exit 1; }
cat $O/swap_ab.jsonl
timeout -k 10 100 ./tools/ubench/bar_probe 60 > $O/bar_probe.jsonl 2> $O/bar_probe.err; echo "bar_probe rc=$?"
cat $O/bar_probe.jsonl | cut -c1-900
