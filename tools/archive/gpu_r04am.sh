set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_config1.sh gpurun_out/r04am_pmc || exit 1
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --workload strict --no-cpu-baseline > gpurun_out/r04am_strict_$i.json 2> gpurun_out/r04am_strict_$i.err || { tail -5 gpurun_out/r04am_strict_$i.err; exit 1; }
  tail -c 300 gpurun_out/r04am_strict_$i.json
done
