# Round 4: strict specialisation A/B (same process), stall PMC, config-2 PMC on the shipped
# 24-bit-B build (keyed default path), then the N=50 service repeat with producer lateness.
set -o pipefail
timeout -k 10 400 python -u tools/strict_variants.py --reps 5 narwhal_amd/libnarwhal_amd.so exp/unspec/libnarwhal_amd.so > gpurun_out/r04n_strict_ab.json 2> gpurun_out/r04n_strict_ab.log || { tail -5 gpurun_out/r04n_strict_ab.log; exit 1; }
cat gpurun_out/r04n_strict_ab.json
bash tools/pmc_stall.sh gpurun_out/r04n_stall || exit 1
MODES=keyed bash tools/pmc_cert.sh gpurun_out/r04n_cert 4 100 || exit 1
NW_SERVICE_DEBUG=1 timeout -k 10 250 python -u bench.py --workload service --service-committees 50 --service-rates 1000000,1000000,1000000,1000000 > gpurun_out/r04m_service.json 2> gpurun_out/r04m_service.err; tail -4 gpurun_out/r04m_service.err
