# Round 5: 20-bit committee-key combs for mid-size committees with the key-major vote sort
# forced (NW_VOTES_KEY_MAJOR=1) vs the 16-bit default, N = 50 and 100, alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05kw2; mkdir -p $O
A="--workload cert --cert-invalid 0 --cert-payload-committees= --no-cpu-baseline --committees 50,100"
for r in 1 2; do
  for v in w16 w20s w16s; do
    unset NW_KEY_WIDTH NW_VOTES_KEY_MAJOR
    if [ $v = w20s ]; then export NW_KEY_WIDTH=20 NW_VOTES_KEY_MAJOR=1; fi
    if [ $v = w16s ]; then export NW_VOTES_KEY_MAJOR=1; fi
    timeout -k 10 400 python -u bench.py $A > $O/cert_${v}_$r.json 2> $O/cert_${v}_$r.err || { tail -20 $O/cert_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/cert_${v}_$r.json')); s=d['summary']; print('$v', s['cert_stream_Mcerts_s'], d['parity'])"
  done
done
