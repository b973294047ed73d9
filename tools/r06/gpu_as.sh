# Round 6: the profile set of the final tree (triage checks in the shared strict_triage):
# parity files, the round's profile set on it (kernel trace of the default bench + PMC
# traffic passes), then its VALU mix and stall fractions (the bench line's issue-bound peak).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06as; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_streams.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 bash tools/profile_round.sh r06as > $O/profile_round.log 2>&1 || { tail -20 $O/profile_round.log; exit 1; }
tail -9 $O/profile_round.log
bash tools/pmc_mix.sh $O/mix > $O/mix.out 2>&1; tail -2 $O/mix.out
grep -q "rc=0" $O/mix.out || exit 1
bash tools/pmc_stall.sh $O/stall > $O/stall.out 2>&1; tail -3 $O/stall.out
