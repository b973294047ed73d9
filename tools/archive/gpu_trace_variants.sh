#!/bin/bash
# GPU box: per-kernel times of the config-1 leg for several library builds (rocprofv3).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in "$@"; do
  tag=$(echo $L | tr '/' '_')
  NW_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tv_$tag -o p \
    -- python3 bench.py --workload batch --steps 2 --no-cpu-baseline > gpurun_out/tv_$tag.json 2>/dev/null
  echo "== $L rc=$?"
  python3 - "$tag" <<'PY'
import csv, glob, collections, sys
f = glob.glob(f'gpurun_out/tv_{sys.argv[1]}/**/p_kernel_trace.csv', recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    g = int(r.get('Grid_Size_X', 0) or 0)
    if 'pip' in r['Kernel_Name'] or 'iota' in r['Kernel_Name']:
        agg[(r['Kernel_Name'].split('(')[0][-14:], g)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for (k, g), v in sorted(agg.items()):
    v.sort(); print(f"  {k:16s} grid={g:8d} n={len(v):3d} med_us={v[len(v)//2]:8.1f}")
PY
done
