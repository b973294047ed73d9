# Round 6: k_strict_triage's occupancy (rolled A/R loop): 4 waves/SIMD (default build) against
# 3 / 5 / 6 (tools/r06/build_var.sh triW -DNW_TRIAGE_WAVES=W), the strict bench leg
# alternating, two rounds; the strict parity file once on the default build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06an; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--no-cert --no-batch --no-wire --no-service --no-worker --no-sha --no-cpu-baseline"
for i in 1 2; do
  for cfg in w4 w3 w5 w6; do
    if [ $cfg = w4 ]; then E="NW_X=0"; else E="NW_LIB=tools/r06/var/tri${cfg#w}/libnarwhal_amd.so"; fi
    env $E NW_BENCH_DETAIL=$O/s_${cfg}_$i.json timeout -k 10 300 python -u bench.py $A > $O/s_${cfg}_$i.line 2> $O/s_${cfg}_$i.err || { tail -5 $O/s_${cfg}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/s_${cfg}_$i.line').read()); r=d['roofline']
print('$cfg $i', round(d['value']/1e6,2), 'M/s', d['parity'], round(r.get('kernel_ms') or 0,2), 'ms')" || exit 1
  done
done
