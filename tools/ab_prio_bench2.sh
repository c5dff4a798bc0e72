#!/bin/bash
# Bench A/B of the wave-priority turns on the C4 fan-out and the brawler (variants prod / noprio)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  echo "## c4"; VARS="prod noprio" EXTRA="--session p2p --num-players 4 --fanout --steps 100 --warmup 50" bash tools/varrun.sh || exit 1
  echo "## c4_k8"; VARS="prod noprio" EXTRA="--session p2p --num-players 4 --fanout --fanout-k 8 --steps 100 --warmup 50" bash tools/varrun.sh || exit 1
  echo "## brawler"; VARS="prod noprio" EXTRA="--game brawler --steps 100 --warmup 32" bash tools/varrun.sh || exit 1
  echo "## brawler_p2p"; VARS="prod noprio" EXTRA="--game brawler --session p2p --steps 100 --warmup 50" bash tools/varrun.sh || exit 1
  echo "## p2p1"; VARS="prod noprio" EXTRA="--session p2p --ticks-per-launch 1 --steps 400" bash tools/varrun.sh || exit 1
done
