#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box through gpurun):
#   1. --kernel-trace --stats of the bench command (per-kernel average duration)
#   2. separate --pmc passes: FETCH_SIZE, WRITE_SIZE, SQ occupancy/issue counters,
#      L2 hit/miss (one pass per block budget, MI355X_MICROARCH.md §rocprofv3 PMC slots)
# then tools/pmc_summary.py (run here, after gpurun merges gpurun_out/) folds
# them into profiles/<tag>_*.
# --warmup 58 = 8 start-up ticks + one 50-tick steady launch, so every
# steady_kernel launch in the trace covers exactly --ticks-per-launch ticks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
EXTRA=${EXTRA:-}
BENCH="bench.py --steps 400 --warmup 58 --ticks-per-launch 50 --no-cpu-baseline $EXTRA"
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -s KILL "$t" rocprofv3 "$@" -d "$PWD/$OUT/$name" -o run --output-format csv -- python3 -u $BENCH \
    > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$OUT/$name.log"
  echo "=== $name rc=$rc"
  return $rc
}
run stats 300 --kernel-trace --stats &&
run pmc_fetch 180 --pmc FETCH_SIZE &&
run pmc_write 180 --pmc WRITE_SIZE &&
run pmc_sq 180 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR &&
run pmc_l2 180 --pmc TCC_HIT_sum TCC_MISS_sum
# back in the container: python3 tools/pmc_summary.py gpurun_out/prof_$TAG $TAG
