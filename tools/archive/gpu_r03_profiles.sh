#!/bin/bash
# GPU-box helper (round 3): the committed profile set of the final tree, stopping at the
# first failure: rocprof trace of the default bench + config-4/3/1 PMC passes
# (profile_round.sh), the strict kernel's VALU mix and stall passes, and the config-2
# keyed-vote PMC passes at N = 100 and 4.   bash tools/gpu_r03_profiles.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r03}
bash tools/profile_round.sh $TAG && \
bash tools/pmc_mix.sh gpurun_out/prof_$TAG/mix && \
bash tools/pmc_stall.sh gpurun_out/prof_$TAG/stall && \
MODES=keyed bash tools/pmc_cert.sh gpurun_out/prof_$TAG/cert 100 4
rc=$?
# summarise on the box (the raw traces exceed gpurun's 64 MiB copy-back), keep the summaries
S=gpurun_out/sum_$TAG; mkdir -p $S
cp profiles/traffic.json $S/traffic.json
python3 tools/profile_summary.py gpurun_out/prof_$TAG $S/$TAG > $S/profile_summary.log 2>&1
python3 tools/pmc_strict_json.py gpurun_out/prof_$TAG/mix gpurun_out/prof_$TAG/stall $S/$TAG
python3 tools/pmc_cert_summary.py gpurun_out/prof_$TAG/cert $S/$TAG > $S/cert_summary.log 2>&1
for f in gpurun_out/prof_$TAG/cert/keyed_n*_trace/p_kernel_stats.csv; do
  n=$(basename $(dirname $f)); cp $f $S/$TAG/${n}_kernel_stats.csv; done
rm -rf gpurun_out/prof_$TAG
exit $rc
