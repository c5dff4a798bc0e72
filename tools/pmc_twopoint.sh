#!/bin/bash
# What saturates steady_kernel: the SyncTest bench at SIZES sessions (default
# 65,536 = 2 waves per SIMD and 131,072 = 4), 50-tick launches, one rocprofv3 --pmc pass per counter
# group (MI355X_MICROARCH.md: at most 8 SQ counters per pass, GRBM separate).  Folded by
# tools/pmc_twopoint.py into profiles/<TAG>_twopoint.json.
# usage (GPU box): TAG=r05 SIZES="65536 131072" bash tools/pmc_twopoint.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r05}
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
P3="SQ_ACTIVE_INST_VALU2 SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
P4="SQC_ICACHE_MISSES SQC_ICACHE_HITS TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for S in ${SIZES:-65536 131072}; do
  i=0
  for grp in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i + 1))
    out=gpurun_out/pmc2_${TAG}_${S}_p$i
    rm -rf "$out"
    echo "=== S=$S pass $i ($(date +%T))"
    timeout -s KILL 90 rocprofv3 --pmc $grp -d "$PWD/$out" -o run --output-format csv -- \
      python3 -u bench.py --steps 100 --warmup 50 --ticks-per-launch 50 --realtime-ticks 0 --no-cpu-baseline \
      --sessions-per-gpu "$S" > "$out.log" 2>&1
    rc=$?
    tail -n 2 "$out.log" | cut -c1-200
    echo "=== rc=$rc"
    [ $rc -ne 0 ] && [ $i -lt 3 ] && exit $rc
  done
done
exit 0
