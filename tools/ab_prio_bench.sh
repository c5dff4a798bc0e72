#!/bin/bash
# Bench A/B of the wave-priority turns (tools/mkvar.sh variants prod / noprio / p2pprio / p2pprio12)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  echo "## synctest"; VARS="prod noprio" EXTRA="--steps 400" bash tools/varrun.sh || exit 1
  echo "## driver"; VARS="prod noprio" EXTRA="--gpus 1 --steps 20 --warmup 5" bash tools/varrun.sh || exit 1
  echo "## p2p"; VARS="prod p2pprio p2pprio12" EXTRA="--session p2p --steps 400" bash tools/varrun.sh || exit 1
  echo "## p2p_sparse"; VARS="prod p2pprio" EXTRA="--session p2p --sparse-saving --steps 400" bash tools/varrun.sh || exit 1
  echo "## wire_replay"; VARS="prod p2pprio" EXTRA="--session p2p --wire-replay --steps 400" bash tools/varrun.sh || exit 1
done
