#!/bin/bash
# Short P2P launches (2-16 ticks): HBM cells + HBM input ring (prod), LDS cells from 2 ticks (ldsc2),
# HBM cells + LDS input ring (ldsring)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for tpl in 2 4 8 16; do
    echo "## tpl $tpl"; VARS="prod ldsc2 ldsring" EXTRA="--session p2p --ticks-per-launch $tpl --steps 400" bash tools/varrun.sh || exit 1
  done
done
