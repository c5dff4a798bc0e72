"""Steady-kernel time attribution (experiment only): time rb_run_ticks with
parts of the fused tick disabled through rb_config.reserved[0] knobs:
1 trivial advance, 2 no snapshot stores, 4 no checksums, 32 | mask<<8:
inputs ANDed with mask."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ggrs_amd as G  # noqa: E402

S = int(os.environ.get("S", 65536))
GAME = G.Game.BRAWLER if os.environ.get("GAME") == "brawler" else G.Game.EX_GAME
T, W0 = 32 + 200, 32
inputs = torch.from_numpy(G.synth_inputs(S, 2, T)).cuda()
cases = [(0, "base"), (1, "trivial_advance"), (2, "no_snap_store"), (4, "no_checksum"),
         (6, "no_store_no_cs"), (32 | (0xF3F3 << 8), "no_thrust(no sincos)"), (32 | (0xFCFC << 8), "no_rotation"),
         (32, "no_input_at_all"), (1 | 2 | 4, "loop_only")]
for flags, name in cases:
    s = (G.SessionBuilder(GAME, num_sessions=S).with_check_distance(7).with_input_delay(2)
         .with_checked_mismatches(False).with_debug_flags(flags).start_synctest_session())
    s.run_ticks(inputs[:W0])
    s.synchronize()
    s.profile_enable(1)
    s.profile_take()
    t0 = time.perf_counter()
    for c in range(W0, T, 50):
        s.run_ticks(inputs[c:min(T, c + 50)])
    s.synchronize()
    el = time.perf_counter() - t0
    ms, n = s.profile_take()
    print(f"{name:24s}: kernel {ms / n * 1e3:7.3f} us/tick   wall {el / (T - W0) * 1e6:7.3f} us/tick", flush=True)
    s.close()
