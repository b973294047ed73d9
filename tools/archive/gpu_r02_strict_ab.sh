set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1 || { tail -30 gpurun_out/gpu_parity.log; exit 1; }
tail -1 gpurun_out/gpu_parity.log
timeout -k 10 400 python -u tools/strict_variants.py --reps 3 --steps 5 narwhal_amd/libnarwhal_amd.so $* > gpurun_out/strict_ab.json 2> gpurun_out/strict_ab.err || { tail -20 gpurun_out/strict_ab.err; exit 1; }
cat gpurun_out/strict_ab.json
