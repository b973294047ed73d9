# Round 5: key-major vote sort from 32 keys: the certificate / service GPU tests, then config 2
# (N = 4, 10, 50, 100) with NW_VOTES_KEY_MAJOR unset (the new rule) vs forced off.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05kw3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_messages.py tests/test_service.py tests/test_gpu_fuzz.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--workload cert --cert-invalid 0 --cert-payload-committees= --no-cpu-baseline --committees 50"
for r in 1 2; do
  for v in off new; do
    unset NW_VOTES_KEY_MAJOR
    if [ $v = off ]; then export NW_VOTES_KEY_MAJOR=0; fi
    timeout -k 10 400 python -u bench.py $A > $O/cert_${v}_$r.json 2> $O/cert_${v}_$r.err || { tail -20 $O/cert_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/cert_${v}_$r.json')); s=d['summary']; print('$v', s['cert_stream_Mcerts_s'], d['parity'])"
  done
done
