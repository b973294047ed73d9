# Round 5: Pippenger points padded to one 128-byte line each: batch / certificate GPU tests,
# then config 1 (one-call latency, 64 batches resident) A/B against the unpadded build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05pad; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_messages.py tests/test_gpu_fuzz.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in unpad pad; do
    if [ $v = unpad ]; then L=var/unpad/libnarwhal_amd.so; else L=narwhal_amd/libnarwhal_amd.so; fi
    NW_LIB=$L timeout -k 10 300 python -u bench.py --workload batch --steps 20 --no-cpu-baseline > $O/batch_${v}_$r.json 2> $O/batch_${v}_$r.err || { tail -20 $O/batch_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/batch_${v}_$r.json')); print('$v', d['summary']['batch10k'], d['parity'])"
  done
done
