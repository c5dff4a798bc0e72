#!/bin/bash
# A/B of the P2P bench line: lock-step ticks (RB_P2P_SYNC_TICKS=1) vs
# lane-asynchronous ticks (p2p.hpp kAsync), interleaved on one box.
# EXTRA="--lag-max 8" etc. are passed to bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in sync async; do
    sync=0; [ "$v" = sync ] && sync=1
    RB_P2P_SYNC_TICKS=$sync timeout -k 10 200 python3 -u bench.py --session p2p ${EXTRA:-} --steps 400 --warmup 32 --no-cpu-baseline \
      > gpurun_out/abp_$v.log 2>&1 || exit $?
    python3 -c "
import json
for l in open('gpurun_out/abp_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$v', 'value %.3e'%d['value'], 'kernel_us %.1f'%r['kernel_avg_us'], 'frac %.3f'%r['frac'])"
  done
done
