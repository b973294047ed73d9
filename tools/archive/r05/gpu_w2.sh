# Round 5: the strict kernel at 2 waves/SIMD (no spills) A/B, after the packed tables and the
# LDS digit words.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w2; mkdir -p $O
timeout -k 10 400 python -u tools/strict_variants.py --reps 4 --steps 4 narwhal_amd/libnarwhal_amd.so var/w2/libnarwhal_amd.so > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.json
