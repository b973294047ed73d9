#!/bin/bash
# GPU-box helper for launch-bound experiments: the config-2 (N = 4, 100) and config-1 legs of
# bench.py against the in-tree library ("def") and variant builds exp/<v>/libnarwhal_amd.so
# (built here beforehand with one kernel's __launch_bounds__ changed), loaded via NW_LIB.
# Results: gpurun_out/sw/{c,b}_<v>.json. Stops at the first failing run.
set -o pipefail
mkdir -p gpurun_out/sw
C="python bench.py --workload cert --committees 4,100 --no-cpu-baseline"
B="python bench.py --workload batch --steps 5 --no-cpu-baseline"
for v in ${SWEEP:-def f g h}; do
  if [ $v = def ]; then L=narwhal_amd/libnarwhal_amd.so; else L=exp/$v/libnarwhal_amd.so; fi
  NW_LIB=$L timeout -k 10 200 $C > gpurun_out/sw/c_$v.json 2>/dev/null || exit 1
  NW_LIB=$L timeout -k 10 120 $B > gpurun_out/sw/b_$v.json 2>/dev/null || exit 1
done
