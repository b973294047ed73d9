# Round 6: the profile set of the final tree (kernel trace of the default bench + PMC passes,
# tools/profile_round.sh), then differential fuzz on the final tree (batch / strict corpus
# over Straus, Pippenger and fused one-call sizes; irregular committees), each step bounded.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 900 bash tools/profile_round.sh r06g > $O/profile_round.log 2>&1 || { tail -20 $O/profile_round.log; exit 1; }
tail -5 $O/profile_round.log
timeout -k 10 280 python -u tools/fuzz_long.py 20000 300 batch > $O/fuzz_batch.json 2> $O/fuzz_batch.err || { tail -20 $O/fuzz_batch.err; exit 1; }
cut -c1-400 $O/fuzz_batch.json
