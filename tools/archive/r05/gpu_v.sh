# Round 5: stall breakdown of the packed-table strict kernel (tools/pmc_stall.sh).
set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_stall.sh gpurun_out/r05v
