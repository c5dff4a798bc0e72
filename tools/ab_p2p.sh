#!/bin/bash
# A/B of P2P bench lines across library builds: VARS="r1 cur" (cur = the in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARS:-r1 cur}; do
  lib=$PWD/ggrs_amd/var/lib_$v.so; [ "$v" = cur ] && lib=$PWD/ggrs_amd/libggrs_amd.so
  for rep in 1 2; do
    GGRS_AMD_LIB=$lib timeout -k 10 200 python3 -u bench.py --session p2p ${EXTRA:-} --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit $?
    python3 -c "
import json
for l in open('gpurun_out/ab_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$v', 'value %.3e'%d['value'], 'kernel_us %.1f'%r['kernel_avg_us'])"
  done
done
