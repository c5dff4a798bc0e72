#!/bin/bash
# Round 3: GPU tests + the driver's bench command + host-overhead probe (GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
step() {  # step <name> <timeout> <cmd...>; stops the script on a crash / timeout
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  tail -n ${TAILN:-6} "gpurun_out/${TAG}_$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-pytest driver ho}; do
  case $s in
    pytest) step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    driver) step driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    ho) step ho 300 python -u tools/host_overhead.py ;;
    synctest) step synctest 300 python -u bench.py --steps 400 --warmup 32 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
