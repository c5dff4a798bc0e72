#!/bin/bash
# A/B: the LDS input ring (RB_SHORT_HBM_RING=0 variant) against the HBM ring in short launches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  echo "## p2p1"; VARS="prod ldsring" EXTRA="--session p2p --ticks-per-launch 1 --steps 400" bash tools/varrun.sh || exit 1
  echo "## p2p tpl2"; VARS="prod ldsring" EXTRA="--session p2p --ticks-per-launch 2 --steps 400" bash tools/varrun.sh || exit 1
  echo "## p2p tpl8"; VARS="prod ldsring" EXTRA="--session p2p --ticks-per-launch 8 --steps 400" bash tools/varrun.sh || exit 1
  echo "## p2p tpl50"; VARS="prod" EXTRA="--session p2p --steps 400" bash tools/varrun.sh || exit 1
  echo "## wire"; VARS="prod ldsring" EXTRA="--session p2p --wire --steps 200" bash tools/varrun.sh || exit 1
done
