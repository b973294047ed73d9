set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests3.log 2>&1 || { tail -30 gpurun_out/gputests3.log; exit 1; }
tail -2 gpurun_out/gputests3.log
timeout -k 10 300 python -u tools/strict_variants.py --reps 3 --steps 5 narwhal_amd/libnarwhal_amd.so exp/mac2/libnarwhal_amd.so > gpurun_out/ab_mac5.json 2> gpurun_out/ab_mac5.err || { tail -20 gpurun_out/ab_mac5.err; exit 1; }
cat gpurun_out/ab_mac5.json
TRACE_VOTES=1024 TRACE_N=100 bash tools/group_sweep.sh gpurun_out/gsweep 32768 4096 1024 512
