#!/bin/bash
# Round profile set (GPU box): every bench line's kernel stats + PMC passes, and the
# WRITE_SIZE calibration of the brawler's store pattern.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -k 10 60 ./tools/build/calib_write > gpurun_out/calib/plain.log 2>&1 || exit $?
cat gpurun_out/calib/plain.log
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d "$PWD/gpurun_out/calib/pmc" -o run --output-format csv -- ./tools/build/calib_write \
  > gpurun_out/calib/pmc.log 2>&1 || exit $?
NAME=synctest EXTRA="" bash tools/prof_round.sh || exit $?
NAME=brawler EXTRA="--game brawler" bash tools/prof_round.sh || exit $?
NAME=p2p EXTRA="--session p2p" bash tools/prof_round.sh || exit $?
NAME=c4 EXTRA="--session p2p --num-players 4 --fanout" STEPS=100 WARMUP=16 bash tools/prof_round.sh || exit $?
NAME=wire EXTRA="--session p2p --wire" STEPS=200 WARMUP=16 bash tools/prof_round.sh || exit $?
