#!/bin/bash
# A/B: the first tick's packet heads loaded with the state (prod) or in the poll (base)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wire.py \
  tests/test_p2p_fullsize.py -k "packet or wire" > gpurun_out/wirehead_pytest.log 2>&1 || { tail -30 gpurun_out/wirehead_pytest.log; exit 1; }
tail -1 gpurun_out/wirehead_pytest.log
for rep in 1 2; do
  echo "## wire"; VARS="prod base" EXTRA="--session p2p --wire --steps 200" bash tools/varrun.sh || exit 1
  echo "## wire_replay"; VARS="prod base" EXTRA="--session p2p --wire-replay --steps 400" bash tools/varrun.sh || exit 1
done
