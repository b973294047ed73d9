#!/bin/bash
# GPU box: kernel trace of the config-1 leg (one-call latency path + resident batches).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_batch -o p \
  -- python3 bench.py --workload batch --steps 3 --no-cpu-baseline > gpurun_out/trace_batch.json 2> gpurun_out/trace_batch.log || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/trace_batch/**/p_kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(list)
for r in rows:
    g = int(r.get('Grid_Size_X', r.get('Grid_Size', 0)) or 0)
    agg[(r['Kernel_Name'][:40], g)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for (k, g), v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:30]:
    v.sort()
    print(f"{k:40s} grid={g:9d} n={len(v):4d} med_us={v[len(v)//2]:9.1f} min_us={v[0]:9.1f}")
PY
