#!/bin/bash
# Round 4: scheduler A/B (variant libraries, tools/mkvar.sh): max-ILP scheduling, occupancy hint
# <= 2 waves per SIMD for the steady kernel, latency-weighted metric; interleaved, 2 reps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_sched
mkdir -p $O
ab() {  # name, args
  local name=$1; shift
  for rep in 1 2; do
    for lib in prod ilp wpe2 bias0; do
      L=""; [ $lib != prod ] && L=$PWD/ggrs_amd/var/lib_$lib.so
      GGRS_AMD_LIB=$L timeout -k 10 200 python3 -u bench.py "$@" --no-cpu-baseline > $O/${name}_$lib.log 2>&1 || return $?
      python3 -c "
import json
for l in open('$O/${name}_$lib.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']
        print('%-8s %-6s'%('$name','$lib'), 'value %.4e'%d['value'], 'kernel_us %.2f'%r['kernel_avg_us'], 'tpl %.0f'%r['ticks_per_launch'])"
    done
  done
}
ab sync --steps 400 --warmup 50 --ticks-per-launch 50 --realtime-ticks 0 || exit $?
ab p2p --session p2p --steps 200 --warmup 50 --ticks-per-launch 50 || exit $?
ab live --session p2p --steps 200 --warmup 16 --ticks-per-launch 1 || exit $?
ab driver --gpus 1 --steps 20 --warmup 5 || exit $?
