#!/bin/bash
# A/B of the priority rotation at 131,072 sessions per GPU (4 waves per SIMD: config 5's share)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  echo "## synctest 131k"; VARS="prod par2 noprio" EXTRA="--sessions-per-gpu 131072 --steps 400" bash tools/varrun.sh || exit 1
  echo "## p2p 131k"; VARS="prod par2 noprio" EXTRA="--sessions-per-gpu 131072 --session p2p --steps 400" bash tools/varrun.sh || exit 1
  echo "## synctest 65k"; VARS="prod par2" EXTRA="--steps 400" bash tools/varrun.sh || exit 1
done
