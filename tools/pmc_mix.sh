#!/bin/bash
# Instruction mix of the P2P kernel per library build: one rocprofv3 --pmc pass
# (8 SQ counters) per VARS entry over a short bench run, summarised per wave
# and tick by tools/pmc_mix.py.  usage: VARS="cur none" EXTRA="--lag 0,0" bash tools/pmc_mix.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARS:-cur}; do
  lib=$PWD/ggrs_amd/var/lib_$v.so; [ "$v" = cur ] && lib=$PWD/ggrs_amd/libggrs_amd.so
  out=gpurun_out/mix_$v
  rm -rf "$out"
  GGRS_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d "$PWD/$out" -o run --output-format csv -- \
    python3 -u bench.py --session p2p ${EXTRA:-} --steps 100 --warmup 0 --ticks-per-launch 50 --no-cpu-baseline \
    > "$out.log" 2>&1 || exit $?
  python3 tools/pmc_mix.py "$out" "$v" 50 || exit $?
done
