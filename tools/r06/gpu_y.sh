# Round 6: the asyncio service leg's parity FAIL in r06x (N = 50, 10^4/s, 20,000 certificates):
# the same load with every mismatch listed, hedge on / off x small-job done flags on / off.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u tools/r06/svc_py_check.py 10000 20000 $HEDGE > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  cut -c1-1200 $O/$tag.json
}
HEDGE=0.001 run hedge_done NW_SMALL_DONE=1
HEDGE=0 run nohedge_done NW_SMALL_DONE=1
HEDGE=0.001 run hedge_event NW_SMALL_DONE=0
HEDGE=0 run nohedge_event NW_SMALL_DONE=0
HEDGE=0.001 run hedge_done2 NW_SMALL_DONE=1
