# Round 6: config 1 returning on the fused tail's done word (NW_BATCH_SPIN=1) instead of the
# launch's completion event: the batch parity files with it, then alternating one-call
# latency (default vs spin, three pairs, host-side stamps on).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 890 --timeout-method thread tests/test_gpu_small_vram.py > $O/vram_tests.log 2>&1 || { tail -40 $O/vram_tests.log; exit 1; }
tail -7 $O/vram_tests.log
for i in 1 2 3; do
  for v in 1 0; do
    NW_BATCH_SPIN=$v NW_BATCH_STAMPS=1 NW_BENCH_DETAIL=$O/batch_${v}_$i.json timeout -k 10 200 python -u bench.py --workload batch --no-cpu-baseline > $O/batch_${v}_$i.line 2> $O/batch_${v}_$i.err || { tail -20 $O/batch_${v}_$i.err; exit 1; }
    python3 - <<PY
import re, statistics as st, json
L=open('$O/batch_${v}_$i.err').read().splitlines()
wai=[float(m.group(1)) for l in L if (m:=re.search(r'wait ([0-9.]+) us', l))]
b=json.load(open('$O/batch_${v}_$i.json'))
print('spin=$v run $i latency', round(b['verify_batch_10k']['latency_ms'],4), 'mean', round(b['verify_batch_10k']['latency_ms_mean'],4), 'wait p50', st.median(wai) if wai else None, 'parity', b['parity'])
PY
  done
done
