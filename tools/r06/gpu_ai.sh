# Round 6: config 1's one-call timeline on the final tree (NW_PIP_FUSE_STAMPS=1: head and fused
# tail workgroup stamps per call; 30 calls) for the next step's target.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ai; mkdir -p $O
NW_PIP_FUSE_STAMPS=1 timeout -k 10 120 python -u tools/r06/c1_ab.py 30 > $O/c1_stamps.json 2> $O/c1_stamps.txt || { tail -5 $O/c1_stamps.txt; exit 1; }
cat $O/c1_stamps.json; tail -9 $O/c1_stamps.txt
