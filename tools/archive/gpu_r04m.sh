set -o pipefail
NW_SERVICE_DEBUG=1 timeout -k 10 250 python -u bench.py --workload service --service-committees 50 --service-rates 1000000,1000000,1000000,1000000 > gpurun_out/r04m_service.json 2> gpurun_out/r04m_service.err; tail -4 gpurun_out/r04m_service.err
