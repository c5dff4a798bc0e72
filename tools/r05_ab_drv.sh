#!/bin/bash
# A/B of library variants on the driver's exact command (events off in the timed region), interleaved,
# plus the variants' wave clocks on the driver's launch shape.  usage: VARS="cur prog" bash tools/r05_ab_drv.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
lib() { [ "$1" = cur ] && echo "$PWD/ggrs_amd/libggrs_amd.so" || echo "$PWD/ggrs_amd/var/lib_$1.so"; }
for rep in 1 2 3; do
  for v in ${VARS:-cur prog}; do
    GGRS_AMD_LIB=$(lib $v) GGRS_BENCH_EVENTS=off timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 \
      --no-cpu-baseline --realtime-ticks 0 > gpurun_out/abd_$v.json 2> gpurun_out/abd_$v.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/abd_$v.json'));print('$v wall us', round(d['ms_per_step']*20e3,1), 'replay kernel', round(d['roofline']['kernel_avg_us'],1), 'value %.4e' % d['value'])"
  done
done
for v in ${WCLK:-}; do
  echo "== wave clock $v"
  GGRS_AMD_LIB=$(lib $v) W0=13 TPL=20 timeout -k 10 120 python3 -u tools/wave_clock.py 2>&1 | grep -E "^launch|slot|pairs" | cut -c1-260 || exit 1
done
