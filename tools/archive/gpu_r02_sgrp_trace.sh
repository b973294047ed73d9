set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_messages.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_sgrp.log 2>&1 || { tail -40 gpurun_out/gputests_sgrp.log; exit 1; }
tail -2 gpurun_out/gputests_sgrp.log
NW_DEBUG_GROUPS=1 timeout -k 10 300 python -u bench.py --workload cert --cert-steps 3 > gpurun_out/cert_sgrp.json 2> gpurun_out/cert_sgrp.err || { tail -20 gpurun_out/cert_sgrp.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/cert_sgrp.json').read().strip().splitlines()[-1])
for leg in ('cert_stream','cert_stream_invalid'):
  for n,v in d[leg].items(): print(leg,n,round(v['certs_per_s']/1e6,2), v.get('vs_all_valid'), v['parity'])
PY
for N in 4 100; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sgtrace$N -o p -- python3 bench.py --workload cert --committees $N --cert-steps 3 > gpurun_out/sgtrace$N.json 2> gpurun_out/sgtrace$N.err || { echo trace failed; exit 1; }
done
echo traces ok
