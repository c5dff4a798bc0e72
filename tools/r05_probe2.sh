#!/bin/bash
# Round 5: VALU issue costs per instruction class at 1/2/4 waves per SIMD (dual issue), and the
# per-wave clocks of the driver's 20-tick launch (ticks 13-33) and of later 20/50-tick launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 tools/build/ubench_valu > gpurun_out/r05_ubench.log 2>&1 || exit $?
cat gpurun_out/r05_ubench.log
GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_wclk.so W0=13 TPL=20 timeout -k 10 120 python3 -u tools/wave_clock.py \
  > gpurun_out/r05_wclk20.log 2>&1 || exit $?
cat gpurun_out/r05_wclk20.log
GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_wclk.so W0=32 TPL=50 timeout -k 10 120 python3 -u tools/wave_clock.py \
  > gpurun_out/r05_wclk50.log 2>&1 || exit $?
cat gpurun_out/r05_wclk50.log
