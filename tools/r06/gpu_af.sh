# Round 6: config 1's one call, the input gate revisited: no gate (default) / gate with
# 1,024-vote chunks / 2,560 / one chunk (the launch queued before any vote is written),
# alternating, three rounds, 300 calls each (tools/r06/c1_ab.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06af; mkdir -p $O
for i in 1 2 3; do
  for cfg in def g1024 g2560 g10000; do
    case $cfg in
      def) E="NW_X=0";;
      g*) E="NW_BATCH_GATE=1 NW_GATE_CHUNK=${cfg#g}";;
    esac
    env $E timeout -k 10 120 python -u tools/r06/c1_ab.py 300 >> $O/c1.jsonl 2> $O/c1_$cfg_$i.err || { tail -5 $O/c1_$cfg_$i.err; exit 1; }
    tail -1 $O/c1.jsonl
  done
done
