#!/bin/bash
# Round 4 re-measure after the priority turns: GPU suite, every profile pass, every bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests \
  > gpurun_out/r04_pytest_gpu.log 2>&1
rc=$?
tail -n 2 gpurun_out/r04_pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
PART=1 bash tools/gpu_r04_prof.sh > gpurun_out/prof_final.log 2>&1 &&
PART=4 bash tools/gpu_r04_prof.sh >> gpurun_out/prof_final.log 2>&1 &&
PART=2 bash tools/gpu_r04_prof.sh >> gpurun_out/prof_final.log 2>&1 &&
PART=3 bash tools/gpu_r04_prof.sh >> gpurun_out/prof_final.log 2>&1 || { echo "profiles failed"; exit 1; }
echo "profiles ok"
TAG=r04 bash tools/bench_round.sh
