# Round 5: the irregular-committee fuzz tests, then the service at 10^6 certs/s six times per
# committee with the per-job CSV timeline (NW_SERVICE_DEBUG=<path>).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py tests/test_worker.py -m gpu -v --timeout 200 --timeout-method thread -k "irregular or worker" > $O/fuzz.log 2>&1 || { tail -60 $O/fuzz.log; exit 1; }
tail -3 $O/fuzz.log
NW_SERVICE_DEBUG=$PWD/$O/svc NW_BENCH_DETAIL=$O/service_detail.json timeout -k 10 400 python -u bench.py --workload service --service-committees 4,50 --service-rates 1000000,1000000,1000000,1000000,1000000,1000000 > $O/service.json 2> $O/service.err || { tail -20 $O/service.err; exit 1; }
grep "narwhal_amd" $O/service.err | tail -30
ls $O | head -40
