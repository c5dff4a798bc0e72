"""ex_game SyncTest steady kernel: one lane per player (the default) vs one
lane per session (with_lane_per_session), interleaved in one process, the
bench workload (65,536 sessions, cd 7, delay 2), per-launch kernel time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ggrs_amd as G  # noqa: E402

S = int(os.environ.get("S", 65536))
T, W0, TPL = 32 + 400, 32, 50
inputs = torch.from_numpy(G.synth_inputs(S, 2, T)).cuda()
for rep in range(2):
    for lps in (False, True):
        s = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_check_distance(7).with_input_delay(2)
             .with_checked_mismatches(False).with_lane_per_session(lps).start_synctest_session())
        s.run_ticks(inputs[:W0])
        s.synchronize()
        s.profile_enable(1)
        s.profile_take()
        for c in range(W0, T, TPL):
            s.run_ticks(inputs[c:min(T, c + TPL)])
        s.synchronize()
        ms, n = s.profile_take()
        print(f"lane_per_session={lps}: {ms / n * 1e3:.1f} us per {TPL}-tick launch", flush=True)
        s.close()
