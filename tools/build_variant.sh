#!/bin/bash
# Build a variant of libnarwhal_amd.so into exp/<name>/ with extra compiler flags
# (e.g. -DNW_STRICT_WAVES=2), for tools/strict_variants.py / NW_LIB experiments.
#   bash tools/build_variant.sh NAME "-DFOO=1 -DBAR"
set -e
cd "$(dirname "$0")/.."
NAME=$1
FLAGS=$2
mkdir -p exp/$NAME/build
make -s -j8 LIB=exp/$NAME/libnarwhal_amd.so BUILD=exp/$NAME/build \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Inarwhal_amd/csrc -Wall -Wno-unused-function $FLAGS" \
  exp/$NAME/libnarwhal_amd.so
echo "built exp/$NAME/libnarwhal_amd.so ($FLAGS)"
