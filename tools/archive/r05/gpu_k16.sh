# Round 5: the -m gpu suite on the default (16-bit) build after generalizing the key comb
# width (bdigits recoding, an extra j * 2^128 A table when W does not divide 128).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k16; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
