#!/bin/bash
# P2P parity tests (incl. disconnects, fan-out, wire) then the P2P bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_p2p.py tests/test_wire.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/p2p_disc.log 2>&1; rc=$?
tail -30 gpurun_out/p2p_disc.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --session p2p --steps 400 --warmup 50 --no-cpu-baseline > gpurun_out/bench_p2p.log 2>&1; rc=$?
tail -1 gpurun_out/bench_p2p.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --session p2p --num-players 4 --fanout --steps 100 --warmup 16 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c4.log; exit $rc
