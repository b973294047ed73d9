# (r05s2) Batch GPU tests with windows 24..31 at twice the bucket lanes, then the one-call
# latency over NW_PIP_FUSE_SPLIT = 24 32 24 32 16 20 28 (tools/ab_batch_latency.py 400) and
# NW_PIP_FUSE_STAMPS=1 at the default split (reverted afterwards: no measurable gain).
