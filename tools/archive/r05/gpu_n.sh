# Round 5: paired field products (fe_sq2 / fe_mul2: four MAC chains) in ge_dbl (NW_PAIR=1),
# ge_add_any (2) and both (3), same-process A/B against the in-tree strict kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 400 python -u tools/strict_variants.py --reps 4 --steps 4 narwhal_amd/libnarwhal_amd.so var/pair1/libnarwhal_amd.so var/pair2/libnarwhal_amd.so var/pair3/libnarwhal_amd.so > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.json
