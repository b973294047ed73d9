set -o pipefail
NW_SERVICE_DEBUG=1 timeout -k 10 200 python -u bench.py --workload service --service-rates 1000000,1000000,1000000,1000000 > gpurun_out/r04q_service.json 2> gpurun_out/r04q_service.err || exit 1
grep "service:" gpurun_out/r04q_service.err
NW_SERVICE_DEBUG=1 timeout -k 10 200 python -u bench.py --workload service --service-committees 50 --service-producers 8 --service-rates 1000000,1000000,1000000 > gpurun_out/r04q_service_p8.json 2> gpurun_out/r04q_service_p8.err || exit 1
