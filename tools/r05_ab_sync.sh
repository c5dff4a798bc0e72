#!/bin/bash
# Interleaved A/B of library variants on the SyncTest bench: the driver's command (events off in the
# timed region) and 400 ticks in 50-tick launches (kernel time per launch from the launches' events).
# usage: VARS="cur pcold" bash tools/r05_ab_sync.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
lib() { [ "$1" = cur ] && echo "$PWD/ggrs_amd/libggrs_amd.so" || echo "$PWD/ggrs_amd/var/lib_$1.so"; }
for rep in 1 2 3; do
  for v in ${VARS:-cur}; do
    GGRS_AMD_LIB=$(lib $v) GGRS_BENCH_EVENTS=off timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 \
      --no-cpu-baseline --realtime-ticks 0 > gpurun_out/abs_$v.json 2> gpurun_out/abs_$v.err || exit $?
    GGRS_AMD_LIB=$(lib $v) timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --realtime-ticks 0 $EXTRA \
      > gpurun_out/abs50_$v.json 2> gpurun_out/abs50_$v.err || exit $?
    python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/abs_{v}.json")); e = json.load(open(f"gpurun_out/abs50_{v}.json"))
print(f"{v:8s} driver wall {d['ms_per_step'] * 20e3:6.1f} us ({d['value']:.4e})  50-tick kernel {e['roofline']['kernel_avg_us']:6.1f} us ({e['value']:.4e})")
PY
  done
done
