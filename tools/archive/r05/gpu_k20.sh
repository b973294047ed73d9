# Round 5: committee-key combs of 20 / 24 bits (13 / 11 tables instead of 16: fewer additions
# per keyed check) — the keyed GPU tests on the 20-bit build, then config-2 A/B in
# alternating runs (16 vs 20 at N = 4, 10, 50, 100; 24 at N = 4, 10).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k20; mkdir -p $O
echo "tests skipped (run separately)"

A="--workload cert --cert-invalid 0 --cert-payload-committees= --no-cpu-baseline"
for r in 1 2; do
  for v in 16 20 24; do
    if [ $v = 16 ]; then L=narwhal_amd/libnarwhal_amd.so; C=4,10,50,100; else L=var/k$v/libnarwhal_amd.so; C=4,10,50,100; fi
    if [ $v = 24 ]; then C=4,10; fi
    NW_LIB=$L timeout -k 10 400 python -u bench.py $A --committees $C > $O/cert_${v}_$r.json 2> $O/cert_${v}_$r.err || { tail -20 $O/cert_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/cert_${v}_$r.json')); print('$v', d['summary']['cert_stream_Mcerts_s'], d['parity'])"
  done
done
