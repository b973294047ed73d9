#!/bin/bash
# GPU-box helper: PMC counters of k_verify_strict for two library builds in one process
# (tools/strict_variants.py, all-valid and mixed corpora), one counter group per pass.
#   bash tools/pmc_ab.sh OUTDIR LIB_B      (LIB_A = the in-tree library)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_ab}
LIBB=$2
mkdir -p $OUT
ARGS="--items 4194304 --reps 1 --steps 1"
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o p \
    -- python3 tools/strict_variants.py $ARGS $EXTRA narwhal_amd/libnarwhal_amd.so $LIBB > $OUT/$name.json 2> $OUT/$name.log
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
EXTRA=--all-valid pass valid_sq SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS && \
EXTRA=--all-valid pass valid_fetch FETCH_SIZE && \
EXTRA= pass mixed_sq SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS
