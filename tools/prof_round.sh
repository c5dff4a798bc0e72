#!/bin/bash
# rocprofv3 evidence for one bench configuration (run on the GPU box through gpurun):
#   1. --kernel-trace --stats of the bench command (per-kernel average duration)
#   2. separate --pmc passes: FETCH_SIZE, WRITE_SIZE, SQ issue counters + GRBM clock,
#      L2 hit/miss (one pass per block budget, MI355X_MICROARCH.md §rocprofv3 PMC slots)
# then tools/pmc_summary.py (run here, after gpurun merges gpurun_out/) folds
# them into profiles/<tag>_<name>_*.
# usage: TAG=r02 NAME=synctest EXTRA="" WARMUP=50 bash tools/prof_round.sh
# WARMUP 50 = one warm-up launch of exactly --ticks-per-launch steady ticks (the
# start-up ticks run before it), so every steady launch in the trace covers the
# same number of ticks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
NAME=${NAME:-synctest}
OUT=gpurun_out/prof_${TAG}_${NAME}
mkdir -p "$OUT"
export TMPDIR=/tmp
EXTRA=${EXTRA:-}
WARMUP=${WARMUP:-50}
STEPS=${STEPS:-400}
BENCH="bench.py --steps $STEPS --warmup $WARMUP --ticks-per-launch 50 --realtime-ticks 0 --no-cpu-baseline $EXTRA"
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "=== $NAME/$name ($(date +%T))"
  timeout -s KILL "$t" rocprofv3 "$@" -d "$PWD/$OUT/$name" -o run --output-format csv -- python3 -u $BENCH \
    > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 1 "$OUT/$name.log" | cut -c1-300
  echo "=== $NAME/$name rc=$rc"
  return $rc
}
run stats 300 --kernel-trace --stats &&
run pmc_fetch 180 --pmc FETCH_SIZE &&
run pmc_write 180 --pmc WRITE_SIZE &&
run pmc_sq 180 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE &&
run pmc_l2 180 --pmc TCC_HIT_sum TCC_MISS_sum
# back in the container: python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_${NAME} ${TAG}_${NAME} <config_key> <ticks_per_launch>
