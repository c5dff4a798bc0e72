#!/bin/bash
# A/B of the SyncTest bench line across library builds, interleaved on one box:
# VARS="old cur" (cur = the in-tree build; others ggrs_amd/var/lib_<v>.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in ${VARS:-old cur}; do
    lib=$PWD/ggrs_amd/var/lib_$v.so; [ "$v" = cur ] && lib=$PWD/ggrs_amd/libggrs_amd.so
    GGRS_AMD_LIB=$lib timeout -k 10 120 python3 -u bench.py --steps 400 --warmup 32 --no-cpu-baseline ${EXTRA:-} \
      > gpurun_out/abs_$v.log 2>&1 || exit $?
    python3 -c "
import json
for l in open('gpurun_out/abs_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', '%.4g'%d['value'], '%.1f'%d['roofline']['kernel_avg_us'])"
  done
done
