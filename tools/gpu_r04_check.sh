#!/bin/bash
# Round 4: the whole GPU suite, then the driver's command and the P2P lines it changed
# (kernel-owned timing events; fan-out candidates from the move-to-front list).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_check
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?
tail -n 3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
line() {  # name, args
  local name=$1; shift
  timeout -k 10 300 python3 -u bench.py "$@" > $O/$name.log 2>&1 || return $?
  python3 -c "
import json
for l in open('$O/$name.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; c=d['config']
        x=(c.get('speculative') or {})
        print('%-10s'%'$name', 'value %.4e'%d['value'], 'ms/step %.5f'%d['ms_per_step'], 'kernel_us %.2f'%r['kernel_avg_us'],
              'tpl %.0f'%r['ticks_per_launch'], 'frac %.3f'%r['frac'], 'sel %.3f'%x.get('select_fraction', 0),
              'rt', (d.get('realtime') or {}).get('kernel_us_per_tick'), (d.get('realtime') or {}).get('wall_us_per_tick'))"
}
for rep in 1 2 3; do
  line driver$rep --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
line p2p_live --session p2p --ticks-per-launch 1 --steps 200 --warmup 16 --no-cpu-baseline || exit $?
line wire_live --session p2p --wire --steps 200 --warmup 16 --no-cpu-baseline || exit $?
line c4_k16 --session p2p --num-players 4 --fanout --steps 100 --warmup 50 --no-cpu-baseline || exit $?
line c4_k8 --session p2p --num-players 4 --fanout --fanout-k 8 --steps 100 --warmup 50 --no-cpu-baseline || exit $?
