# Round 5: committee key-comb width per committee (20 bits up to 16 keys, 16 above): the -m gpu
# suite, then config 2 with NW_KEY_WIDTH=16 forced vs the per-committee choice, alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05kw; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
A="--workload cert --cert-invalid 0.01 --cert-payload-committees= --no-cpu-baseline"
for r in 1 2; do
  for v in w16 auto; do
    if [ $v = w16 ]; then export NW_KEY_WIDTH=16; else unset NW_KEY_WIDTH; fi
    timeout -k 10 400 python -u bench.py $A > $O/cert_${v}_$r.json 2> $O/cert_${v}_$r.err || { tail -20 $O/cert_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/cert_${v}_$r.json')); s=d['summary']; print('$v', s['cert_stream_Mcerts_s'], s['cert_stream_invalid_Mcerts_s'], d['parity'])"
  done
done
