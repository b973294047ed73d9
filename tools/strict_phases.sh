#!/bin/bash
# Per-phase split of k_verify_strict's work, step 1 (here, CPU): build
# the phase-cut variants of the library (nw_strict.hpp NW_STRICT_STOP = 1..6), each with only
# nw_kernels.o recompiled and linked against the in-tree build's other objects, into
# tools/r06/phases/stop<k>/libnarwhal_amd.so. Step 2 (GPU box): tools/strict_phases_pmc.sh.
set -e
cd "$(dirname "$0")/.."
make -s -j8 narwhal_amd/libnarwhal_amd.so
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Inarwhal_amd/csrc -Wall -Wno-unused-function"
OBJS=$(ls build/*.o | grep -v nw_kernels.o)
for k in 1 2 3 4 5 6; do
  (mkdir -p tools/r06/phases/stop$k && \
   /opt/rocm/bin/hipcc $HIPFLAGS -DNW_STRICT_STOP=$k -c narwhal_amd/csrc/nw_kernels.hip -o tools/r06/phases/stop$k/nw_kernels.o && \
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/r06/phases/stop$k/libnarwhal_amd.so tools/r06/phases/stop$k/nw_kernels.o $OBJS && \
   echo "built tools/r06/phases/stop$k") &
  if [ $k = 3 ]; then wait; fi
done
wait
