# Round 5: per-lane strict tables packed into 128-byte entries (NW_PACK_TAB=1: one line per
# lookup instead of two) A/B against the in-tree kernel, then its HBM traffic (one PMC pass
# pair over one bench-size strict launch each).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 400 python -u tools/strict_variants.py --reps 4 --steps 4 narwhal_amd/libnarwhal_amd.so var/pack/libnarwhal_amd.so > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.json
