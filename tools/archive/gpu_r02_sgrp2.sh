set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NW_DEBUG_GROUPS=1 timeout -k 10 300 python -u bench.py --workload cert --cert-steps 3 > gpurun_out/cert_sgrp.json 2> gpurun_out/cert_sgrp.err || { tail -20 gpurun_out/cert_sgrp.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/cert_sgrp.json').read().strip().splitlines()[-1])
for leg in ('cert_stream','cert_stream_invalid'):
  for n,v in d[leg].items(): print(leg,n,round(v['certs_per_s']/1e6,2), v.get('vs_all_valid'), v['parity'])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sgtrace100 -o p -- python3 bench.py --workload cert --committees 100 --cert-steps 3 > gpurun_out/sgtrace100.json 2> gpurun_out/sgtrace100.err || { echo trace failed; exit 1; }
echo trace ok
