#!/bin/bash
# The driver's bench command, three times plain and twice traced (GGRS_BENCH_TRACE: host call time, first
# synchronize, GPU marker-to-marker time), each a fresh process (GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --realtime-ticks 0 > gpurun_out/drv_$i.json 2> gpurun_out/drv_$i.err || exit 1; python -c "import json;d=json.load(open('gpurun_out/drv_$i.json'));print('plain us', d['ms_per_step']*20e3, 'kernel', d['roofline']['kernel_avg_us'], 'value %.3e' % d['value'])"; done
for i in 1 2; do GGRS_BENCH_TRACE=1 timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --realtime-ticks 0 > gpurun_out/drvt_$i.json 2> gpurun_out/drvt_$i.err || exit 1; grep trace gpurun_out/drvt_$i.err; done
