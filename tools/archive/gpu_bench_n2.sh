#!/bin/bash
# GPU-box helper: a 2-rank rehearsal of the driver's multi-GPU bench (every leg, small
# sizes) with both ranks sharing the box's one GPU over gloo (NW_BENCH_BACKEND=gloo).
set -o pipefail
mkdir -p gpurun_out
NW_BENCH_BACKEND=gloo timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 \
  --warmup 1 --items-per-gpu 1000000 --certs 100000 --cert-unique 16384 --committees 4,100 \
  --batch-many 8 --wire-frames 8192 --sha-batches 4096 --service-rates 1000,10000 \
  --service-seconds 0.5 --cpu-seconds 3 > gpurun_out/b_n2.json 2> gpurun_out/b_n2.err \
  || { tail -30 gpurun_out/b_n2.err; exit 1; }
echo DONE
