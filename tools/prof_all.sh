#!/bin/bash
# Round profile set (GPU box): every bench line's kernel stats + PMC passes, the driver's exact
# command under --kernel-trace --stats, and the WRITE_SIZE calibration of the brawler's store
# pattern.  Stops at the first failure.  TAG=r03 bash tools/prof_all.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
export TAG
mkdir -p gpurun_out/calib gpurun_out/prof_${TAG}_driver
if [ -x ./tools/build/calib_write ]; then
  timeout -k 10 60 ./tools/build/calib_write > gpurun_out/calib/plain.log 2>&1 || exit $?
fi
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_driver/stats" -o run --output-format csv -- \
  python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${TAG}_driver/stats.log 2>&1 || exit $?
NAME=synctest EXTRA="" bash tools/prof_round.sh || exit $?
NAME=brawler EXTRA="--game brawler" STEPS=100 bash tools/prof_round.sh || exit $?
NAME=brawler1 EXTRA="--game brawler --ticks-per-launch 1 --realtime-ticks 0" STEPS=32 WARMUP=8 bash tools/prof_round.sh || exit $?
NAME=p2p EXTRA="--session p2p" bash tools/prof_round.sh || exit $?
NAME=p2p_sparse EXTRA="--session p2p --sparse-saving" bash tools/prof_round.sh || exit $?
NAME=c4 EXTRA="--session p2p --num-players 4 --fanout" STEPS=100 WARMUP=16 bash tools/prof_round.sh || exit $?
NAME=wire EXTRA="--session p2p --wire" STEPS=200 WARMUP=16 bash tools/prof_round.sh || exit $?
NAME=wire_replay EXTRA="--session p2p --wire-replay" STEPS=400 WARMUP=50 bash tools/prof_round.sh || exit $?
