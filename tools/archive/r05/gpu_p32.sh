# Round 5: the P = 32 certificate leg at N = 4 regressed in the round-end bench (57 vs 143 M
# certs/s): its kernel trace with the per-committee width, and the leg with NW_KEY_WIDTH=16.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p32; mkdir -p $O
A="--workload cert --cert-invalid 0 --committees 100 --cert-payload-committees 4,100 --no-cpu-baseline"
NW_KEY_WIDTH=16 timeout -k 10 300 python -u bench.py $A > $O/w16.json 2> $O/w16.err || { tail -20 $O/w16.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/w16.json')); print('w16', d['summary'].get('cert_stream_p32_Mcerts_s'))"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o p -- python3 bench.py $A > $O/auto.json 2> $O/auto.err || { tail -20 $O/auto.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/auto.json')); print('auto', d['summary'].get('cert_stream_p32_Mcerts_s'))"
