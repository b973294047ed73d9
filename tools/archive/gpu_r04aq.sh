set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/fuzz_long.py 1000 200 > gpurun_out/r04aq_fuzz.json 2> gpurun_out/r04aq_fuzz.log || { tail -5 gpurun_out/r04aq_fuzz.log; exit 1; }
cat gpurun_out/r04aq_fuzz.json
