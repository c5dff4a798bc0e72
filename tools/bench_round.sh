#!/bin/bash
# The round's bench lines (GPU box): the driver's exact command, then every
# configuration with its CPU baseline.  One JSON line per run in
# gpurun_out/bench_<TAG>_<name>.jsonl; stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04}
mkdir -p gpurun_out
b() {  # b <name> <timeout> <bench args...>
  local name=$1 t=$2; shift 2
  if [ -n "${ONLY:-}" ] && [[ " $ONLY " != *" $name "* ]]; then return 0; fi  # ONLY="a b": just those lines
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" python3 -u bench.py "$@" > "gpurun_out/bench_${TAG}_$name.log" 2>&1
  local rc=$?
  grep '^{' "gpurun_out/bench_${TAG}_$name.log" > "gpurun_out/bench_${TAG}_$name.jsonl"
  python3 - "gpurun_out/bench_${TAG}_$name.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]; c = d.get("cpu_baseline") or {}
    print(f"  value {d['value']:.4g} {d['unit']}  ms/step {d['ms_per_step']:.4f}  kernel_us {r.get('kernel_avg_us', 0):.1f}"
          f"  frac {r['frac']:.3f}  cpu {c.get('value', 0):.3g} ({c.get('cores', '-')} threads)")
PY
  echo "=== $name rc=$rc"
  return $rc
}
b driver 300 --gpus 1 --steps 20 --warmup 5 &&
b synctest 300 --steps 400 --warmup 32 &&
b brawler 600 --game brawler --steps 100 --warmup 32 &&
b brawler_tpl1 600 --game brawler --ticks-per-launch 1 --steps 32 --warmup 8 &&
b p2p 600 --session p2p --steps 400 --warmup 32 &&
b p2p_tpl1 600 --session p2p --ticks-per-launch 1 --steps 400 --warmup 32 &&
b p2p_sparse 600 --session p2p --sparse-saving --steps 400 --warmup 32 &&
b brawler_p2p 600 --game brawler --session p2p --steps 100 --warmup 32 &&
b brawler_p2p_sparse 600 --game brawler --session p2p --sparse-saving --steps 100 --warmup 32 &&
b c4 600 --session p2p --num-players 4 --fanout --steps 100 --warmup 16 &&
b c4_k8 600 --session p2p --num-players 4 --fanout --fanout-k 8 --steps 100 --warmup 16 &&
b brawler_fan 600 --game brawler --session p2p --fanout --steps 20 --warmup 10 &&
b wire 600 --session p2p --wire --steps 200 --warmup 32 &&
b wire_replay 600 --session p2p --wire-replay --steps 400 --warmup 32
