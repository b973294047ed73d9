#!/bin/bash
# A kernel variant of the library for tools/strict_variants.py: nw_kernels.hip recompiled
# with extra flags and linked against the in-tree build's other objects, into
# tools/r06/var/<name>/libnarwhal_amd.so (gpurun carries it; exp/ is not carried).
#   bash tools/r06/build_var.sh NAME "-DFOO=1"
set -e
cd "$(dirname "$0")/../.."
NAME=$1; FLAGS=$2
make -s -j8 narwhal_amd/libnarwhal_amd.so
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Inarwhal_amd/csrc -Wall -Wno-unused-function"
OBJS=$(ls build/*.o | grep -v nw_kernels.o)
D=tools/r06/var/$NAME; mkdir -p $D
/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c narwhal_amd/csrc/nw_kernels.hip -o $D/nw_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libnarwhal_amd.so $D/nw_kernels.o $OBJS
echo "built $D ($FLAGS)"
