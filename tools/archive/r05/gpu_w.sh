# Round 5: the strict ladder's digit words in LDS (NW_LDS_DIGITS=1: no scratch array read per
# addition) A/B against the in-tree kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 400 python -u tools/strict_variants.py --reps 4 --steps 4 narwhal_amd/libnarwhal_amd.so var/ldsdig/libnarwhal_amd.so > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.json
