#!/bin/bash
# Round 4 profile set (GPU box), in parts (one gpurun call each): every bench line's
# rocprofv3 kernel stats + PMC passes (tools/prof_round.sh).  PART=1|2|3|4.
# Back here: tools/r04_fold.sh folds them into profiles/r04_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TAG=r04
p() { NAME=$1 EXTRA=$2 STEPS=$3 WARMUP=$4 bash tools/prof_round.sh; }
case "${PART:-1}" in
1)
  p driver "--ticks-per-launch 20" 20 20 &&
  p synctest "" 400 50 &&
  p synctest1 "--ticks-per-launch 1" 100 50 ;;
4)
  p p2p "--session p2p" 400 50 &&
  p p2p1 "--session p2p --ticks-per-launch 1" 200 50 &&
  p p2p_sparse "--session p2p --sparse-saving" 400 50 ;;
2)
  p c4 "--session p2p --num-players 4 --fanout" 100 50 &&
  p c4_k8 "--session p2p --num-players 4 --fanout --fanout-k 8" 100 50 &&
  p wire "--session p2p --wire" 200 16 &&
  p wire_replay "--session p2p --wire-replay" 400 50 ;;
3)
  p brawler "--game brawler" 100 50 &&
  p brawler1 "--game brawler --ticks-per-launch 1" 32 8 &&
  p brawler_p2p "--game brawler --session p2p" 100 50 &&
  p brawler_p2p_sparse "--game brawler --session p2p --sparse-saving" 100 50 &&
  p brawler_fan "--game brawler --session p2p --fanout" 20 10 ;;
esac
