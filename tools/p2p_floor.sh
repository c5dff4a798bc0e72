#!/bin/bash
# P2P bench variants: where the P2P tick time goes (no-rollback floor vs lagged network)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lag in "0,0" "1,1" "1,4"; do
  timeout -k 10 300 python3 -u bench.py --session p2p --lag $lag --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/p2p_lag_${lag/,/_}.log 2>&1 || exit $?
  python3 -c "
import json
for l in open('gpurun_out/p2p_lag_${lag/,/_}.log'):
    if l.startswith('{'):
        d=json.loads(l); c=d['config']; r=d['roofline']
        print('lag $lag', 'value %.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'kernel_us %.1f'%r['kernel_avg_us'], 'adv/st %.3f'%c['advance_frames_per_session_tick'], 'rb/st %.3f'%c['rollbacks_per_session_tick'])"
done
