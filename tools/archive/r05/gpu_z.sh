# Round 5: config-2 fallback launches bounded (k_bv_combine grid-stride over the device count,
# k_bv_chunks empty workgroups leave before their LDS fill, k_grp_count one atomic per
# workgroup): GPU tests of the certificate / batch paths, then cert-stream A/B against the
# previous build (alternating runs, N = 4 and 10).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_messages.py tests/test_gpu_batch.py tests/test_gpu_fuzz.py tests/test_gpu_small.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--workload cert --committees 4,10 --cert-invalid 0.01 --cert-payload-committees= --no-cpu-baseline"
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then L=var/prev/libnarwhal_amd.so; else L=narwhal_amd/libnarwhal_amd.so; fi
    NW_LIB=$L timeout -k 10 300 python -u bench.py $A > $O/cert_${v}_$r.json 2> $O/cert_${v}_$r.err || { tail -20 $O/cert_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/cert_${v}_$r.json')); print('$v', {k: round(x['certs_per_s']/1e6,2) for k,x in d['cert_stream'].items()}, {k: round(x['certs_per_s']/1e6,2) for k,x in d['cert_stream_invalid'].items()}, d['parity'])"
  done
done
