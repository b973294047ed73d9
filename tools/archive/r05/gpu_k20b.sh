# Round 5: 20-bit key combs at N = 50 alone (fresh process) vs 16-bit, and N = 4 alone.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k20b; mkdir -p $O
A="--workload cert --cert-invalid 0 --cert-payload-committees= --no-cpu-baseline"
for N in 50 4; do
  for v in 16 20; do
    if [ $v = 16 ]; then L=narwhal_amd/libnarwhal_amd.so; else L=var/k20/libnarwhal_amd.so; fi
    NW_LIB=$L timeout -k 10 300 python -u bench.py $A --committees $N > $O/cert_${v}_$N.json 2> $O/cert_${v}_$N.err || { tail -20 $O/cert_${v}_$N.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/cert_${v}_$N.json')); print('$v', d['summary']['cert_stream_Mcerts_s'], d['parity'])"
  done
done
