#!/bin/bash
# Round 4: workgroups per CU for the steady kernel (RB_LDS_PAD reserves dynamic LDS per workgroup,
# so at most floor(160 KiB / pad) workgroups share a CU): 0 (occupancy-limited: up to 4 per CU),
# 56 KiB (2 per CU: 512 workgroups over 256 CUs exactly), 41 KiB (3 per CU); interleaved, 2 reps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_pad
mkdir -p $O
ab() {  # name, args
  local name=$1; shift
  for rep in 1 2; do
    for pad in 0 57344 41984; do
      RB_LDS_PAD=$pad timeout -k 10 200 python3 -u bench.py "$@" --no-cpu-baseline > $O/${name}_$pad.log 2>&1 || return $?
      python3 -c "
import json
for l in open('$O/${name}_$pad.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; rt=d.get('realtime') or {}
        print('%-8s pad %-6s'%('$name','$pad'), 'value %.4e'%d['value'], 'kernel_us %.2f'%r['kernel_avg_us'], 'tpl %.0f'%r['ticks_per_launch'], 'rt', rt.get('kernel_us_per_tick'))"
    done
  done
}
ab sync --steps 400 --warmup 50 --ticks-per-launch 50 --realtime-ticks 32 || exit $?
ab driver --gpus 1 --steps 20 --warmup 5 || exit $?
