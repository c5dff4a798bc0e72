#!/bin/bash
# A/B of one bench line across library builds, interleaved on one box:
# VARS="base cur" EXTRA="<bench args>" (cur = the in-tree build; others ggrs_amd/var/lib_<v>.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${VARS:-cur}; do
    lib=$PWD/ggrs_amd/var/lib_$v.so; [ "$v" = cur ] && lib=$PWD/ggrs_amd/libggrs_amd.so
    GGRS_AMD_LIB=$lib timeout -k 10 200 python3 -u bench.py ${EXTRA:-} --no-cpu-baseline > gpurun_out/ablib_$v.log 2>&1 || exit $?
    python3 -c "
import json
for l in open('gpurun_out/ablib_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$v', 'value %.3e'%d['value'], 'kernel_us %.1f'%r['kernel_avg_us'], 'ms/step %.4f'%d['ms_per_step'])"
  done
done
