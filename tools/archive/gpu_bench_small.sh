set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --items-per-gpu 1000000 --certs 100000 --cert-unique 16384 --batch-many 8 --wire-frames 8192 --sha-batches 4096 --cpu-seconds 3 > gpurun_out/b_small.json 2> gpurun_out/b_small.err || { tail -30 gpurun_out/b_small.err; exit 1; }
NW_BENCH_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --items-per-gpu 1000000 --no-sha --no-batch --no-wire --certs 100000 --cert-unique 16384 --committees 4,100 > gpurun_out/b_n2.json 2> gpurun_out/b_n2.err || { tail -30 gpurun_out/b_n2.err; exit 1; }
echo DONE
