#!/bin/bash
# Round 4: new parity tests (packet-fed ticks vs the oracle, bad packets, in-range device math),
# then rocprofv3 kernel trace + SQ counters of the one-tick P2P launch, kLive (RB_P2P_LIVE=1)
# against the round-3 kernel (RB_P2P_LIVE=0), and the empty-launch floor (lib_exp32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04_livepmc
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_wire.py tests/test_p2p.py \
  tests/test_gpu_parity.py::test_device_inrange_sincos_and_rotation_step_every_float tests/test_p2p_fullsize.py \
  > $O/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -25
[ $rc -ne 0 ] && exit $rc
B="bench.py --session p2p --ticks-per-launch 1 --steps 100 --warmup 16 --no-cpu-baseline"
for v in 1 0; do
  RB_P2P_LIVE=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $PWD/$O/stats_live$v -o run --output-format csv \
    -- python3 -u $B > $O/stats_live$v.log 2>&1 || exit $?
  RB_P2P_LIVE=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $PWD/$O/sq_live$v -o run --output-format csv \
    -- python3 -u $B > $O/sq_live$v.log 2>&1 || exit $?
done
GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_exp32.so timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $PWD/$O/stats_exp32 \
  -o run --output-format csv -- python3 -u $B > $O/stats_exp32.log 2>&1 || exit $?
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; grep p2p_kernel "$f" | cut -c1-220; done
# A/B: the product library against one built with -fno-slp-vectorize (no packed-f32 VALU)
ab() {  # name, args
  local name=$1; shift
  for rep in 1 2; do
    for lib in prod noslp; do
      L=""; [ $lib = noslp ] && L=$PWD/ggrs_amd/var/lib_noslp.so
      GGRS_AMD_LIB=$L timeout -k 10 200 python3 -u bench.py "$@" --no-cpu-baseline > $O/ab_${name}_$lib.log 2>&1 || return $?
      python3 -c "
import json
for l in open('$O/ab_${name}_$lib.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']
        print('%-8s %-6s'%('$name','$lib'), 'value %.4e'%d['value'], 'kernel_us %.2f'%r['kernel_avg_us'], 'tpl %.0f'%r['ticks_per_launch'])"
    done
  done
}
ab sync --steps 400 --warmup 50 --ticks-per-launch 50 --realtime-ticks 0 || exit $?
ab p2p --session p2p --steps 200 --warmup 50 --ticks-per-launch 50 || exit $?
ab live --session p2p --steps 200 --warmup 16 --ticks-per-launch 1 || exit $?
