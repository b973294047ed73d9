# Round 6: config 4 in two passes (k_strict_triage + k_verify_strict_pre, NW_STRICT_TRIAGE
# default on): the strict parity files, then the strict bench leg alternating with the
# one-pass kernel (NW_STRICT_TRIAGE=0), three rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aj; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_streams.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--no-cert --no-batch --no-wire --no-service --no-worker --no-sha --no-cpu-baseline"
for i in 1 2 3; do
  for cfg in tri one; do
    if [ $cfg = one ]; then E="NW_STRICT_TRIAGE=0"; else E="NW_X=0"; fi
    env $E NW_BENCH_DETAIL=$O/strict_${cfg}_$i.json timeout -k 10 300 python -u bench.py $A > $O/strict_${cfg}_$i.line 2> $O/strict_${cfg}_$i.err || { tail -5 $O/strict_${cfg}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/strict_${cfg}_$i.line').read()); r=d['roofline']
print('$cfg $i', round(d['value']/1e6,2), 'M/s', d['parity'], 'kernel', r.get('kernel'), round(r.get('kernel_ms') or 0,2), 'ms')" || exit 1
  done
done
