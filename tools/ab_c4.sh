#!/bin/bash
# A/B of the C4 (speculative fan-out) bench line, interleaved: the generic
# fanout_kernel (RB_FANOUT_GENERIC=1) vs fanout_indep_kernel (the default for ex_game).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in generic indep; do
    gen=0; [ "$v" = generic ] && gen=1
    RB_FANOUT_GENERIC=$gen timeout -k 10 200 python3 -u bench.py --session p2p --num-players 4 --fanout --steps 100 --warmup 16 \
      --no-cpu-baseline > gpurun_out/abc4_$v.log 2>&1 || exit $?
    python3 -c "
import json
for l in open('gpurun_out/abc4_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$v', 'value %.3e'%d['value'], 'kernel_us %.1f'%r['kernel_avg_us'], 'ms/step %.4f'%d['ms_per_step'])"
  done
done
