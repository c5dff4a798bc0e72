#!/bin/bash
# Round 4: where the one-tick P2P launch's time goes (p2p_kernel kLive attribution builds,
# tools/mkvar.sh -DRB_P2P_EXP=...): launch floor, state in/out, + input window, full tick.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_attr
mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --session p2p --ticks-per-launch 1 --steps 200 --warmup 16 \
    --no-cpu-baseline $EXTRA > $O/$name.log 2>&1 || return $?
  python3 -c "
import json
for l in open('$O/$name.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']
        print('%-10s'%'$name', 'value %.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'kernel_us %.2f'%r['kernel_avg_us'])"
}
for rep in 1 2; do
  run live1 RB_P2P_LIVE=1 || exit $?
  run live0 RB_P2P_LIVE=0 || exit $?
  for v in exp32 exp8 exp16 exp1; do
    run $v GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_$v.so || exit $?
  done
done
