#!/bin/bash
# Round 4: fan-out parity tests, then the C4 lines (K = 16 alphabet, K = 8 move-to-front candidates)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_c4
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_p2p.py \
  tests/test_p2p_fullsize.py > $O/pytest.log 2>&1
rc=$?
tail -n 2 $O/pytest.log
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
              'tpl %.0f'%r['ticks_per_launch'], 'frac %.3f'%r['frac'], 'sel %.3f'%x.get('select_fraction', 0))"
}
for rep in 1 2; do
  line c4_k16 --session p2p --num-players 4 --fanout --steps 100 --warmup 50 --no-cpu-baseline || exit $?
  line c4_k8 --session p2p --num-players 4 --fanout --fanout-k 8 --steps 100 --warmup 50 --no-cpu-baseline || exit $?
done
line brawler_fan --session p2p --game brawler --num-players 2 --fanout --fanout-k 16 --steps 20 --warmup 10 --no-cpu-baseline || exit $?
