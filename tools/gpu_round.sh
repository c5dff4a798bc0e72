#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout/fault (exit codes
# other than 0 = ok and 1 = test failures) ends the script immediately.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r02}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 25 "$OUT/$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || true
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || true
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
  step bench_driver 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 || true  # the driver's exact command
  step bench 600 python -u bench.py --steps 400 --warmup 32 || true
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_$TAG" -o run --output-format csv -- python3 -u bench.py --steps 200 --warmup 32 --no-cpu-baseline || true
  find "$OUT/prof_$TAG" -name '*stats*' | head
fi
