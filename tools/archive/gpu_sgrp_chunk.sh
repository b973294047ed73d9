#!/bin/bash
# GPU-box helper: config-2 1 %-invalid leg at N=4 and N=10 for several small-group chunk sizes.
set -o pipefail
mkdir -p gpurun_out
for C in default 32 48 64; do
  if [ $C = default ]; then unset NW_SGRP_CHUNK; else export NW_SGRP_CHUNK=$C; fi
  timeout -k 10 300 python3 bench.py --workload cert --committees 4,10 --no-cpu-baseline \
    --cert-steps 3 > gpurun_out/sgrp_chunk_$C.json 2> gpurun_out/sgrp_chunk_$C.err || exit 1
  python3 -c "
import json,sys;d=json.loads(open('gpurun_out/sgrp_chunk_$C.json').read().strip().splitlines()[-1])
print('$C', {k:round(v['certs_per_s']/1e6,2) for k,v in d['cert_stream_invalid'].items()}, d['parity'])"
done
