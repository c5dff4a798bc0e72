#!/bin/bash
# Interleaved A/B of C4 (BASELINE config 4) on variant libraries (tools/mkvar.sh, ALLP=1): VARS="a b" REPS="1 2"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in ${REPS:-1 2}; do
  for v in ${VARS:-fin0 fin1}; do
    GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_$v.so timeout -k 10 200 python3 -u bench.py --session p2p --num-players 4 --fanout \
      --steps 100 --warmup 16 --no-cpu-baseline ${EXTRA:-} > gpurun_out/abc4_$v.log 2>&1 || { echo "FAILED $v"; tail -5 gpurun_out/abc4_$v.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/abc4_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$v', 'value %.4e'%d['value'], 'us/tick %.2f'%(r['kernel_avg_us']/r['ticks_per_launch']), 'ms/step %.4f'%d['ms_per_step'])"
  done
done
