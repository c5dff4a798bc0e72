#!/bin/bash
# Fan-out parity tests, then the C4 bench line (GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_p2p.py -k "${K:-fanout or disconnect}" 2>&1 | tail -5
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
for a in ${ARGS:-"--fanout"}; do
  timeout -k 10 200 python -u bench.py --session p2p --num-players 4 ${a//,/ } --steps 100 --warmup 16 --no-cpu-baseline > gpurun_out/c4.json || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/c4.json')); r=d['roofline']; c=d['config']
print('$a', 'value %.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'us/tick %.2f' % (r['kernel_avg_us']/r['ticks_per_launch']), 'sel %.3f' % c['speculative']['select_fraction'], 'branch/s %.3e' % c['speculative']['branch_frames_per_s'])"
done
