# Round 5: config-3 SHA-512 throughput vs batches resident (one lane per batch: 65,536 batches
# = one wave per SIMD; 131,072 = two; 262,144 = four).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
for nb in 65536 131072 262144; do
  timeout -k 10 300 python -u bench.py --workload sha --sha-batches $nb --steps 5 --warmup 2 --no-cpu-baseline > $O/sha_$nb.json 2> $O/sha_$nb.err || { tail -20 $O/sha_$nb.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sha_$nb.json')); print($nb, d['value'], d['roofline']['kernel_ms'], d['parity'])"
done
