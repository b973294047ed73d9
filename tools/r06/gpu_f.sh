# Round 6, check of the tree with the new defaults (negated-2dT ladder additions and the signed
# LDS read in k_verify_strict; config 1's inputs in host-mapped VRAM; the 51-bit host path):
# the full -m gpu suite, smoke, the default bench line (the profile set: gpu_g.sh).
set -o pipefail
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r06f}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
NW_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); s=d['summary']; print(len(open('$O/bench.json').read()), d['value'], d['parity'], d['roofline']['frac'], d['cpu_baseline'], s['batch10k'], s['cert_stream_Mcerts_s'], s['cert_cpu_certs_s'], s['sha512']['GB_s'], s['service'])"
