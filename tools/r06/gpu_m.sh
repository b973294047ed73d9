# Round 6: the final strict kernel's VALU mix and stall fractions (for the bench line's
# issue-bound peak, which came from round 2's kernel until now). Stops at the first pass
# whose rocprofv3 did not exit 0.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
bash tools/pmc_mix.sh $O/mix > $O/mix.out 2>&1; tail -2 $O/mix.out
grep -q "rc=0" $O/mix.out || exit 1
bash tools/pmc_stall.sh $O/stall > $O/stall.out 2>&1; tail -3 $O/stall.out
