#!/bin/bash
# Round 5 bench lines at the north-star scale, each a fresh process:
#   NAME "args"  -> gpurun_out/r05_line_NAME.json (+ .err)
# usage (GPU box): LINES="p2p131k p2p1_1m" bash tools/r05_lines.sh   (default: all)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
declare -A A
A[drv]="--gpus 1 --steps 20 --warmup 5"
A[sync131k]="--sessions-per-gpu 131072 --steps 200 --realtime-ticks 64"
A[sync1m]="--sessions-per-gpu 1048576 --steps 20 --warmup 5 --realtime-ticks 32"
A[p2p]="--session p2p --steps 400 --warmup 50"
A[p2p131k]="--session p2p --sessions-per-gpu 131072 --steps 400 --warmup 50"
A[p2p1]="--session p2p --ticks-per-launch 1 --steps 100 --warmup 20"
A[p2p1_131k]="--session p2p --ticks-per-launch 1 --sessions-per-gpu 131072 --steps 100 --warmup 20"
A[p2p1_1m]="--session p2p --ticks-per-launch 1 --sessions-per-gpu 1048576 --steps 50 --warmup 10"
A[p2p1m]="--session p2p --sessions-per-gpu 1048576 --steps 100 --warmup 50"
for n in ${LINES:-drv sync131k sync1m p2p p2p131k p2p1 p2p1_131k p2p1_1m}; do
  timeout -k 10 ${TMO:-240} python3 -u bench.py ${A[$n]} ${EXTRA:---no-cpu-baseline} > gpurun_out/r05_line_$n.json \
    2> gpurun_out/r05_line_$n.err || { echo "$n failed"; tail -3 gpurun_out/r05_line_$n.err; exit 1; }
  python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.load(open(f"gpurun_out/r05_line_{n}.json"))
r = d["roofline"]
rt = d.get("realtime") or {}
print(f"{n:10s} value {d['value']:.4e}  wall/step {d['ms_per_step'] * 1e3:8.2f} us  kernel/launch {r['kernel_avg_us']:8.1f} us "
      f"({r['ticks_per_launch']:.0f} ticks)  frac {r['frac']:.3f}"
      + (f"  realtime: wall {rt['wall_us_per_tick']:.1f} kernel {rt['kernel_us_per_tick']:.1f} us/tick" if rt else ""))
PY
done
