# Round 6: differential fuzz of the two-pass strict path (k_strict_triage +
# k_verify_strict_pre): the batch / strict corpus over new seeds (every strict verdict
# against the oracle), bounded.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06am; mkdir -p $O
timeout -k 10 500 python -u tools/fuzz_long.py 50000 600 batch > $O/fuzz_batch.json 2> $O/fuzz_batch.err || { tail -20 $O/fuzz_batch.err; exit 1; }
cut -c1-600 $O/fuzz_batch.json
