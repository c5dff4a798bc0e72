cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
TAG=r03
b() { local name=$1; shift; timeout -k 10 300 python3 -u bench.py "$@" > gpurun_out/bench_${TAG}_$name.log 2>&1 || { tail -3 gpurun_out/bench_${TAG}_$name.log; exit 1; }; grep '^{' gpurun_out/bench_${TAG}_$name.log > gpurun_out/bench_${TAG}_$name.jsonl; }
b wire --session p2p --wire --steps 200 --warmup 32 &&
b wire_replay --session p2p --wire-replay --steps 400 --warmup 32 &&
NAME=wire EXTRA="--session p2p --wire" STEPS=200 WARMUP=16 TAG=r03 bash tools/prof_round.sh > gpurun_out/pw.log 2>&1 &&
NAME=wire_replay EXTRA="--session p2p --wire-replay" STEPS=400 WARMUP=50 TAG=r03 bash tools/prof_round.sh > gpurun_out/pwr.log 2>&1 && echo done
