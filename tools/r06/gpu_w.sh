# Round 6: the table-doubling build of k_verify_strict's per-lane tables (NW_TAB_DBL=1: four
# doublings + three mixed additions instead of one doubling + six additions) against the
# shipped build, one process, 8 rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 400 python -u tools/strict_variants.py --reps 8 narwhal_amd/libnarwhal_amd.so tools/r06/var/tabdbl/libnarwhal_amd.so > $O/tabdbl_ab.jsonl 2> $O/tabdbl_ab.err || { tail -20 $O/tabdbl_ab.err; exit 1; }
cat $O/tabdbl_ab.jsonl
