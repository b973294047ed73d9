#!/bin/bash
# A variant of the library (tools/strict_variants.py, negative controls): one source file
# (default nw_kernels.hip) recompiled with extra flags and linked against the in-tree build's
# other objects, into tools/r06/var/<name>/libnarwhal_amd.so (gpurun carries it).
#   bash tools/r06/build_var.sh NAME "-DFOO=1" [nw_jobs.cpp]
set -e
cd "$(dirname "$0")/../.."
NAME=$1; FLAGS=$2; SRC=${3:-nw_kernels.hip}; OBJ=${SRC%.*}.o
make -s -j8 narwhal_amd/libnarwhal_amd.so
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Inarwhal_amd/csrc -Wall -Wno-unused-function"
OBJS=$(ls build/*.o | grep -v "/$OBJ")
D=tools/r06/var/$NAME; mkdir -p $D
/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -x hip -c narwhal_amd/csrc/$SRC -o $D/$OBJ
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libnarwhal_amd.so $D/$OBJ $OBJS
echo "built $D ($FLAGS)"
