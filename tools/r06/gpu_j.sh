# Round 6: where config 1's one call spends its host-side time (NW_BATCH_STAMPS: the input
# writes into host-mapped VRAM, the launch call, the wait), default path and pinned path.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
for v in 1 0; do
  NW_BATCH_STAMPS=1 NW_BATCH_VRAM=$v NW_BENCH_DETAIL=$O/batch_$v.json timeout -k 10 200 python -u bench.py --workload batch --no-cpu-baseline > $O/batch_$v.line 2> $O/batch_$v.err || { tail -20 $O/batch_$v.err; exit 1; }
  python3 - <<PY
import re, statistics as st
L=open('$O/batch_$v.err').read().splitlines()
ins=[float(m.group(1)) for l in L if (m:=re.search(r'n=10000 vram=\d gate=\d inputs ([0-9.]+) us', l))]
lau=[float(m.group(1)) for l in L if (m:=re.search(r'n=10000 .* launch ([0-9.]+) us', l))]
wai=[float(m.group(1)) for l in L if (m:=re.search(r'wait ([0-9.]+) us', l))]
import json
b=json.load(open('$O/batch_$v.json'))['verify_batch_10k']
print('vram=$v calls', len(ins), 'inputs p50', st.median(ins), 'launch p50', st.median(lau), 'wait p50', st.median(wai[-len(ins):]) if wai else None, 'latency', b['latency_ms'])
PY
done
