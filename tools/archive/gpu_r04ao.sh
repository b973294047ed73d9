set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/strict_variants.py --reps 5 narwhal_amd/libnarwhal_amd.so var/ilp/libnarwhal_amd.so > gpurun_out/r04ao_strict_ab.json 2> gpurun_out/r04ao_strict_ab.log || { tail -5 gpurun_out/r04ao_strict_ab.log; exit 1; }
cat gpurun_out/r04ao_strict_ab.json
