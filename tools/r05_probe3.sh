cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 60 tools/build/ubench_mix
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $PWD/gpurun_out/p1m_$c -o run --output-format csv -- python3 -u bench.py --session p2p --ticks-per-launch 1 --sessions-per-gpu 1048576 --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/p1m_$c.log 2>&1 || exit 1
done
