#!/bin/bash
# Round 5: the per-player fan-out's parity tests, then the C4 line in both fan-out forms (and the
# one-player form on the library before per-player speculation, A/B), each a fresh process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_p2p.py \
  tests/test_p2p_fullsize.py tests/test_fanout_adaptive.py > gpurun_out/r05_c4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05_c4_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in one per; do
    lib=$PWD/ggrs_amd/libggrs_amd.so; [ $v = base ] && lib=$PWD/ggrs_amd/var/lib_base.so
    mode=single; [ $v = per ] && mode=per-player
    GGRS_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --session p2p --num-players 4 --fanout --fanout-mode $mode \
      --steps 100 --warmup 16 --no-cpu-baseline > gpurun_out/r05_c4_$v.json 2> gpurun_out/r05_c4_$v.err || { tail -3 gpurun_out/r05_c4_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r05_c4_$v.json'));c=d['config']['speculative'];r=d['roofline'];print('$v', 'us/tick %.2f' % (r['kernel_avg_us']/r['ticks_per_launch']), 'wall us/tick %.2f' % (d['ms_per_step']*1e3), 'selects %.3f' % c['select_fraction'], 'adv/tick %.3f' % d['config']['advance_frames_per_session_tick'])"
  done
done
