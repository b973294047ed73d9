# Round 6: the final strict kernel's VALU mix and stall fractions (for the bench line's
# issue-bound peak, which came from round 2's kernel until now).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
bash tools/pmc_mix.sh $O/mix > $O/mix.out 2>&1; tail -2 $O/mix.out
bash tools/pmc_stall.sh $O/stall > $O/stall.out 2>&1; tail -2 $O/stall.out
