# Round 4: strict VALU mix (pairs with r04n's stall passes), config-2 PMC refresh (keyed
# default path, 24-bit B comb, P = 0 stream only), N=50 service repeats after the
# spin-then-lock / first-request inline change.
set -o pipefail
bash tools/pmc_mix.sh gpurun_out/r04o_mix || exit 1
MODES=keyed bash tools/pmc_cert.sh gpurun_out/r04o_cert 4 50 100 || exit 1
NW_SERVICE_DEBUG=1 timeout -k 10 250 python -u bench.py --workload service --service-rates 1000,10000,100000,1000000,1000000,1000000 > gpurun_out/r04o_service.json 2> gpurun_out/r04o_service.err; tail -6 gpurun_out/r04o_service.err
