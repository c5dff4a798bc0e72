cd "${GRAFT_REPO_ROOT}"
VARS="c0 c1 c2 c3" LINES="c4" REPS="1" bash tools/ab_r03.sh || exit 1
for cd in 7 12; do
  W=$((cd + 1)); [ $cd -eq 12 ] && W=16
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 16 --check-distance $cd --max-prediction $W --no-cpu-baseline --realtime-ticks 0 > gpurun_out/cd$cd.json || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/cd$cd.json')); r=d['roofline']
print('cd $cd W $W', 'value %.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'kernel_us %.1f' % r['kernel_avg_us'], 'tpl', r['ticks_per_launch'], 'launches', r['launches_timed'])"
done
