# Round 6: the small-job done flags after the fix (flags zeroed before launch, process-unique
# sequence numbers; r06aa: mismatches in 4 of 8 runs with done flags, 0 of 4 without). Six
# default runs, 10 s at 10^6 certs/s each; the parity string of each run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ab; mkdir -p $O
for i in 1 2 3 4 5 6; do
  for cfg in def; do
    case $cfg in
      def) E="";;
      done0) E="NW_SMALL_DONE=0";;
      keyw0) E="NW_SMALL_KEYW16=0";;
    esac
    env $E NW_BENCH_DETAIL=$O/svc_${cfg}_$i.json timeout -k 10 150 python -u bench.py --workload service --service-committees 50 --service-rates 1000000 --service-seconds 10 --service-max-certs 10000000 > $O/svc_${cfg}_$i.line 2> $O/svc_${cfg}_$i.err
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "run $cfg $i rc=$rc"; tail -5 $O/svc_${cfg}_$i.err; exit 1; fi
    python3 -c "
import json
d=json.load(open('$O/svc_${cfg}_$i.json'))['service_latency']['N50']
x=d['loads'][0]; a=d['python_asyncio']['loads']
print('$cfg $i native', x.get('parity'), 'p99', round(x['p99_ms'],3), 'hedged', x.get('hedged'), '| asyncio', [y.get('parity') for y in a], [y.get('first_mismatches') for y in a if y.get('first_mismatches')])
" || exit 1
  done
done
