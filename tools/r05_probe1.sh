#!/bin/bash
# Round 5, first GPU call: the driver command's wall time outside the kernel (tools/sync_probe.py,
# the driver command with and without the kernels' own events in the timed region), then the
# two-point PMC profile of steady_kernel (tools/pmc_twopoint.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 180 python3 -u tools/sync_probe.py > gpurun_out/r05_sync_probe.log 2>&1 || exit $?
cat gpurun_out/r05_sync_probe.log
for v in launch off launch off; do
  GGRS_BENCH_EVENTS=$v GGRS_BENCH_TRACE=1 timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 \
    --no-cpu-baseline --realtime-ticks 0 > gpurun_out/r05_drv_$v.json 2> gpurun_out/r05_drv_$v.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r05_drv_$v.json'));print('events=$v wall us', round(d['ms_per_step']*20e3,1), 'kernel', round(d['roofline']['kernel_avg_us'],1), 'value %.4e' % d['value'])"
  grep trace gpurun_out/r05_drv_$v.err
done
ROC_ACTIVE_WAIT_TIMEOUT=1000 GGRS_BENCH_TRACE=1 timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 \
  --no-cpu-baseline --realtime-ticks 0 > gpurun_out/r05_drv_spin.json 2> gpurun_out/r05_drv_spin.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r05_drv_spin.json'));print('spin wall us', round(d['ms_per_step']*20e3,1), 'kernel', round(d['roofline']['kernel_avg_us'],1), 'value %.4e' % d['value'])"
grep trace gpurun_out/r05_drv_spin.err
TAG=r05 bash tools/pmc_twopoint.sh
