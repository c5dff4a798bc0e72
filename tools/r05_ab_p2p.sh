#!/bin/bash
# Interleaved A/B of library variants on the fused P2P bench (lag 1-4, 50-tick launches) at SIZES
# sessions.  usage: VARS="cur q q4" SIZES="65536 131072" bash tools/r05_ab_p2p.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
lib() { [ "$1" = cur ] && echo "$PWD/ggrs_amd/libggrs_amd.so" || echo "$PWD/ggrs_amd/var/lib_$1.so"; }
for rep in 1 2; do
  for S in ${SIZES:-65536 131072}; do
    for v in ${VARS:-cur}; do
      GGRS_AMD_LIB=$(lib $v) timeout -k 10 120 python3 -u bench.py --session p2p --sessions-per-gpu $S --steps 200 \
        --warmup 50 --no-cpu-baseline $EXTRA > gpurun_out/abp_$v.json 2> gpurun_out/abp_$v.err || exit $?
      python3 -c "import json;d=json.load(open('gpurun_out/abp_$v.json'));r=d['roofline'];print('$v S=$S', 'us/tick %.2f' % (r['kernel_avg_us']/r['ticks_per_launch']), 'value %.4e' % d['value'], 'adv/tick %.3f' % d['config']['advance_frames_per_session_tick'])"
    done
  done
done
