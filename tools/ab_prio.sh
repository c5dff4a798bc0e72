#!/bin/bash
# A/B of the steady kernel's wave-priority turns (RB_STEADY_PRIO builds with RB_WAVE_CLOCK, tools/mkvar.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in ${VARS:-wclk prio8 prio9 prio10}; do
    echo "== $v"
    GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_$v.so timeout -k 10 120 python3 -u tools/wave_clock.py 2>&1 | grep -E "^launch|slot|SIMD pairs" | cut -c1-200 || exit 1
  done
done
