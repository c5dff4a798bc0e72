#!/bin/bash
# C4 (BASELINE config 4) kernel split: rocprofv3 --kernel-trace --stats of the fan-out bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r03}_${NAME:-c4}
mkdir -p "$OUT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/stats" -o run --output-format csv -- \
  python3 -u bench.py --session p2p --num-players 4 --fanout --steps ${STEPS:-50} --warmup 16 --no-cpu-baseline ${EXTRA:-} \
  > "$OUT/stats.log" 2>&1
rc=$?
find "$OUT/stats" -name '*kernel_stats.csv' -exec head -6 {} \;
exit $rc
