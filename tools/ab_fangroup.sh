#!/bin/bash
# A/B: fan-out chain group of 4 (prod) or 3 (g3), and 3 with a 3-waves-per-SIMD VGPR cap (g3w3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  echo "## c4"; VARS="prod g3 g3w3" EXTRA="--session p2p --num-players 4 --fanout --steps 100 --warmup 50" bash tools/varrun.sh || exit 1
  echo "## c4_k8"; VARS="prod g3 g3w3" EXTRA="--session p2p --num-players 4 --fanout --fanout-k 8 --steps 100 --warmup 50" bash tools/varrun.sh || exit 1
done
