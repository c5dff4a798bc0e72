#!/bin/bash
# Instruction mix of the P2P kernel, lock-step (RB_P2P_SYNC_TICKS=1) vs
# lane-asynchronous ticks, at the lags in LAGS (default "0,0 1,4").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lag in ${LAGS:-0,0 1,4}; do
  for v in 1 0; do
    export RB_P2P_SYNC_TICKS=$v
    out=gpurun_out/mix_l${lag/,/_}_s$v; rm -rf $out
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d "$PWD/$out" -o run --output-format csv -- python3 -u bench.py --session p2p --lag $lag --steps 100 --warmup 0 --ticks-per-launch 50 --no-cpu-baseline > "$out.log" 2>&1 || exit 1
    python3 tools/pmc_mix.py "$out" "lag$lag-sync$v" 50 || exit 1
    timeout -k 10 100 python3 -u bench.py --session p2p --lag $lag --steps 400 --warmup 32 --no-cpu-baseline > gpurun_out/b_l${lag/,/_}_s$v.log 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/b_l${lag/,/_}_s$v.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('lag $lag sync $v', 'value %.3e'%d['value'], 'kernel_us %.1f'%r['kernel_avg_us'])"
  done
done
