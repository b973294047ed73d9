# Round 6: config 1's one-call latency with the argument pointers built once (the timed region
# holds the C call only), three bench runs of the batch leg.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ad; mkdir -p $O
for i in 1 2 3; do
  NW_BENCH_DETAIL=$O/batch_$i.json timeout -k 10 200 python -u bench.py --workload batch > $O/batch_$i.line 2> $O/batch_$i.err || { tail -5 $O/batch_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/batch_$i.json')); b=d.get('batch10k') or d
print('$i', {k: b[k] for k in ('latency_ms','latency_ms_mean','verifies_per_s_resident','parity') if k in b})" || exit 1
done
