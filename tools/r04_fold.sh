#!/bin/bash
# Fold the round-4 profile passes (gpurun_out/prof_r04_<name>, tools/gpu_r04_prof.sh)
# into profiles/r04_<name>_{kernel_stats.csv,pmc.json}, keyed to the bench lines'
# configuration keys (bench.py cfg_key) and ticks per timed launch.
cd "$(dirname "$0")/.."
X="ex_game P=2 cd=7 W=8 d=2 S=65536"
B="brawler P=2 cd=7 W=8 d=2 S=65536"
Q="p2p ex_game P=2 W=8 d=2 rd=2 lag=1,4 S=65536"
QB="p2p brawler P=2 W=8 d=2 rd=2 lag=1,4 S=65536"
Q4="p2p ex_game P=4 W=8 d=2 rd=2 lag=1,4 S=65536"
f() {  # f <name> <config key> <ticks per launch>
  [ -d gpurun_out/prof_r04_$1 ] || { echo "skip $1"; return 0; }
  python3 tools/pmc_summary.py gpurun_out/prof_r04_$1 r04_$1 "$2" "$3" > /dev/null && echo "r04_$1 <- $2 (tpl $3)"
}
f driver "$X tpl=20" 20
f synctest "$X" 50
f synctest1 "$X tpl=1" 1
f p2p "$Q" 50
f p2p1 "$Q tpl=1" 1
f p2p_sparse "$Q sparse" 50
f c4 "$Q4 fanout" 50
f c4_k8 "$Q4 fanout8" 50
f wire "$Q wire tpl=1" 1
f wire_replay "$Q wire-replay" 50
f brawler "$B" 50
f brawler1 "$B tpl=1" 1
f brawler_p2p "$QB" 50
f brawler_p2p_sparse "$QB sparse" 50
f brawler_fan "$QB fanout tpl=20" 1  # (one call of 20 ticks: a P2P and a fan-out launch per tick)
