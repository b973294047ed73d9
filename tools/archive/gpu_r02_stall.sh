set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_stall.sh gpurun_out/pmc_stall_r02a && \
timeout -k 10 300 python -u tools/strict_variants.py --reps 2 --steps 3 narwhal_amd/libnarwhal_amd.so narwhal_amd/libnarwhal_amd.so > gpurun_out/sv_sanity.json 2> gpurun_out/sv_sanity.err; rc=$?; cat gpurun_out/sv_sanity.json; tail -3 gpurun_out/sv_sanity.err; exit $rc
