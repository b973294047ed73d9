set -o pipefail
mkdir -p gpurun_out
NW_PIP_FUSE_STAMPS=1 timeout -k 10 60 python -u tools/ab_batch_latency.py 40 > gpurun_out/r04aj_stamps.txt 2>&1 || { tail -5 gpurun_out/r04aj_stamps.txt; exit 1; }
tail -8 gpurun_out/r04aj_stamps.txt
