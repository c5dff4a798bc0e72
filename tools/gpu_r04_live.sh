#!/bin/bash
# Round 4: one-tick P2P launches (p2p_kernel kLive) — parity tests, then A/B bench lines
# (RB_P2P_LIVE=0: the round-3 one-tick kernel) for the plain and the packet-fed live tick.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r04_live
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_p2p.py tests/test_wire.py \
  > $O/pytest.log 2>&1
rc=$?
tail -n 3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  for mode in plain wire; do
    extra=""; [ $mode = wire ] && extra="--wire"
    RB_P2P_LIVE=$v timeout -k 10 300 python3 -u bench.py --session p2p --ticks-per-launch 1 --steps 200 --warmup 16 \
      --no-cpu-baseline $extra > $O/bench_${mode}_live$v.log 2>&1 || exit $?
    python3 -c "
import json
for l in open('$O/bench_${mode}_live$v.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']
        print('$mode live=$v', 'value %.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'kernel_us %.2f'%r['kernel_avg_us'])"
  done
done
