# Round 5: paired doubling (fe_sq2 / fe_mul2 in ge_dbl, -DNW_DBL2=1) A/B against the in-tree
# strict kernel, then the new batch/strict irregular-key fuzz test.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 300 python -u tools/strict_variants.py --reps 3 --steps 4 narwhal_amd/libnarwhal_amd.so var/dbl2/libnarwhal_amd.so > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -k "irregular_keys_verify_batch" -v --timeout 200 --timeout-method thread > $O/fuzz.log 2>&1 || { tail -40 $O/fuzz.log; exit 1; }
tail -12 $O/fuzz.log
