# Round 5: the full config-2 sequence of the default bench (N = 4, 10, 50, 100 with 1 %
# invalid and alternating legs, then P = 32 at N = 4 and 100), per-committee width vs 16-bit,
# with the device's free memory logged at each key-table allocation (NW_KEYTAB_LOG=1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p32b; mkdir -p $O
A="--workload cert --no-cpu-baseline"
NW_KEYTAB_LOG=1 timeout -k 10 500 python -u bench.py $A > $O/auto.json 2> $O/auto.err || { tail -20 $O/auto.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/auto.json')); s=d['summary']; print('auto', s['cert_stream_Mcerts_s'], s.get('cert_stream_p32_Mcerts_s'))"
grep -a "keytab" $O/auto.err | tail -20
