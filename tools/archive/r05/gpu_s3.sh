# Config 1 fused tail split A/B: stamps and one-call latency, alternating NW_PIP_FUSE_SPLIT.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s3; mkdir -p $O
for ws in 24 32 24 32; do
  NW_PIP_FUSE_SPLIT=$ws NW_PIP_FUSE_STAMPS=1 timeout -k 10 200 python -u bench.py --workload batch --steps 3 --no-cpu-baseline > /dev/null 2> $O/stamps_$ws.err || { tail -20 $O/stamps_$ws.err; exit 1; }
  echo "ws=$ws"; grep -E "^\[(fuse|horner)\]" $O/stamps_$ws.err | tail -4
done
for ws in 24 32 24 32 24 32; do
  NW_PIP_FUSE_SPLIT=$ws timeout -k 10 120 python -u tools/ab_batch_latency.py 1000 > $O/ab_$ws.txt 2>&1 || { tail -5 $O/ab_$ws.txt; exit 1; }
  echo "ws=$ws $(tail -1 $O/ab_$ws.txt)"
done
