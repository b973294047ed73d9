# Service ingest A/B at 1M certs/s offered: r04l's locking (plain mutex, any small batch
# inline) vs spin-then-lock + first-request inline vs plain mutex + first-request inline.
set -o pipefail
for cfg in "NW_SERVICE_SPIN=0 NW_SERVICE_INLINE_ANY=1" "NW_SERVICE_SPIN=256" "NW_SERVICE_SPIN=0"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 200 python -u bench.py --workload service --service-rates 1000000,1000000,1000000 > gpurun_out/r04p_$tag.json 2> gpurun_out/r04p_$tag.err || exit 1
  echo "$cfg done"
done
