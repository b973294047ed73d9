set -o pipefail
mkdir -p gpurun_out
for s in 1 0 1 0; do HSA_ENABLE_SDMA=$s timeout -k 10 60 python -u tools/ab_batch_latency.py 400 2>&1 | sed "s/^/sdma=$s /" || exit 1; done | tee gpurun_out/r04ad_sdma.txt
