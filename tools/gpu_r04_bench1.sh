#!/bin/bash
# Round 4 measurement pass, part 1: the GPU test suite, then the first bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests \
  > gpurun_out/r04_pytest_gpu.log 2>&1
rc=$?
tail -n 3 gpurun_out/r04_pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
ONLY="driver synctest brawler brawler_tpl1 p2p p2p_tpl1 p2p_sparse" TAG=r04 bash tools/bench_round.sh
