#!/bin/bash
# Interleaved A/B of variant libraries (tools/mkvar.sh) on one GPU box:
# VARS="base cur cur:RB_STEADY_PIPE=0" LINES="sync p2p" bash tools/ab_r03.sh  (lib[:ENV=val])
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in ${REPS:-1 2}; do
  for line in ${LINES:-sync}; do
    case $line in
      sync) args="--steps 400 --warmup 32 --realtime-ticks 0" ;;
      p2p) args="--session p2p --steps 400 --warmup 32" ;;
      c4) args="--session p2p --num-players 4 --fanout --steps 100 --warmup 16" ;;
      wire) args="--session p2p --wire --steps 200 --warmup 32" ;;
      p2p1) args="--session p2p --ticks-per-launch 1 --steps 200 --warmup 32" ;;
      c4k8) args="--session p2p --num-players 4 --fanout --fanout-k 8 --steps 100 --warmup 16" ;;
      brawler1) args="--game brawler --ticks-per-launch 1 --steps 32 --warmup 8 --realtime-ticks 0" ;;
    esac
    for v in ${VARS:-base cur}; do
      lib=${v%%:*}; envs=""; [ "$lib" != "$v" ] && envs=${v#*:}   # "cur:RB_STEADY_PIPE=0" = lib cur + env
      env $envs GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_$lib.so timeout -k 10 200 python3 -u bench.py $args --no-cpu-baseline \
        > gpurun_out/ab_${line}_$v.log 2>&1 || { echo "FAILED $line $v"; tail -5 gpurun_out/ab_${line}_$v.log; exit 1; }
      python3 -c "
import json
for l in open('gpurun_out/ab_${line}_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$line', '$v', 'value %.4e'%d['value'], 'kernel_us %.1f'%r['kernel_avg_us'], 'tpl %.1f'%r['ticks_per_launch'], 'ms/step %.4f'%d['ms_per_step'])"
    done
  done
done
