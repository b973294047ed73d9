# Config 1 one call: fine stamps inside window 31's parts and the Horner's W_31 fold.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s1; mkdir -p $O
NW_PIP_FUSE_STAMPS=1 timeout -k 10 200 python -u bench.py --workload batch --steps 3 --no-cpu-baseline > /dev/null 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
grep -E "^\[(head|fuse|fuse31|horner)\]" $O/stamps.err | tail -8
grep -E "^\[part31\]" $O/stamps.err | tail -10
