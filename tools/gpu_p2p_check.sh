set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_p2p.py tests/test_wire.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/p2p_disc.log 2>&1; rc=$?
tail -30 gpurun_out/p2p_disc.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --session p2p --steps 400 --warmup 32 --no-cpu-baseline > gpurun_out/bench_p2p.log 2>&1; rc=$?
tail -3 gpurun_out/bench_p2p.log; exit $rc
