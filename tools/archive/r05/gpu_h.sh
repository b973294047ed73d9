# Round 5: (1) stall probe: trivial device kernel / the engine's kernel reading PINNED host
# memory / a 64 KB H2D copy, 20 s each at ~10^4 per second; (2) strict kernel at 3 waves per
# SIMD (default, 59 VGPR spill slots) vs 2 waves (no spills), same process, same corpus.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 200 python -u tools/stall_probe.py 20 device pinned copy > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cut -c1-400 $O/probe.jsonl
timeout -k 10 400 python -u tools/strict_variants.py --reps 3 --steps 4 narwhal_amd/libnarwhal_amd.so var/w2/libnarwhal_amd.so > $O/strict_w2_ab.jsonl 2> $O/strict_w2_ab.err || { tail -20 $O/strict_w2_ab.err; exit 1; }
cat $O/strict_w2_ab.jsonl
