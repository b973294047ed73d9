# Round 5: the default bench again with the key-table allocation log (the P = 32 / N = 4 leg
# ran at 57 M certs/s in r05final2's round-end bench and at 151-153 alone).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p32c; mkdir -p $O
NW_KEYTAB_LOG=1 NW_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); s=d['summary']; print(d['value'], s['cert_stream_Mcerts_s'], s.get('cert_stream_p32_Mcerts_s'), s['batch10k'])"
grep -a "keytab" $O/bench.err | tail -20
