# GPU-box helper: same-process strict A/B on the mixed corpus and on an all-valid corpus.
#   bash tools/gpu_ab2.sh LIB [LIB ...]   (the in-tree library is always the first variant)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/strict_variants.py --reps 3 --steps 5 narwhal_amd/libnarwhal_amd.so $* > gpurun_out/ab_mixed.json 2> gpurun_out/ab_mixed.err || { tail -20 gpurun_out/ab_mixed.err; exit 1; }
cat gpurun_out/ab_mixed.json
timeout -k 10 300 python -u tools/strict_variants.py --all-valid --reps 3 --steps 5 narwhal_amd/libnarwhal_amd.so $* > gpurun_out/ab_valid.json 2> gpurun_out/ab_valid.err || { tail -20 gpurun_out/ab_valid.err; exit 1; }
cat gpurun_out/ab_valid.json
