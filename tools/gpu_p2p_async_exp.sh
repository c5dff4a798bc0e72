#!/bin/bash
# Lane-asynchronous P2P ticks, experiment run (GPU box): loop iterations per wave
# (tools/p2p_iters.py on a `tools/mkvar.sh p2pexp4 -DRB_P2P_EXP=4` build) at three
# lags, then the instruction mix of lock-step vs asynchronous ticks.
export TMPDIR=/tmp
GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_p2pexp4.so timeout -k 10 120 python -u tools/p2p_iters.py > gpurun_out/iters.log 2>&1 && 
LAG=0,0 GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_p2pexp4.so timeout -k 10 120 python -u tools/p2p_iters.py >> gpurun_out/iters.log 2>&1 &&
LAG=1,8 GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_p2pexp4.so timeout -k 10 120 python -u tools/p2p_iters.py >> gpurun_out/iters.log 2>&1; cat gpurun_out/iters.log
for v in 1 0; do
  export RB_P2P_SYNC_TICKS=$v
  out=gpurun_out/mixs_$v; rm -rf $out
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d "$PWD/$out" -o run --output-format csv -- python3 -u bench.py --session p2p --steps 100 --warmup 0 --ticks-per-launch 50 --no-cpu-baseline > "$out.log" 2>&1 || exit 1
  python3 tools/pmc_mix.py "$out" "sync$v" 50
done
