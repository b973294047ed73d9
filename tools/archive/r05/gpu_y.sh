# Round 5: config-2 kernel breakdown per committee size (kernel trace of the cert leg alone).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
for N in 4 100; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_N$N -o p -- python3 bench.py --workload cert --committees $N --cert-invalid 0 --cert-payload-committees "" --no-cpu-baseline > $O/cert_N$N.json 2> $O/cert_N$N.err || { tail -20 $O/cert_N$N.err; exit 1; }
  echo "N$N ok"
done
