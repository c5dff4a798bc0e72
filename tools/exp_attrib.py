"""Kernel time attribution: time the tick kernel with parts disabled (debug knobs)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import ggrs_amd as G

S = int(os.environ.get("S", 65536)); T = 96; W0 = 32
inputs = torch.from_numpy(G.synth_inputs(S, 2, T)).cuda()
for flags, name in [(0, "base"), (1, "no_advance"), (2, "no_snap_store"), (4, "no_checksum"), (6, "no_store_no_cs"), (7, "nothing"), (8, "launch_only")]:
    for block, lps in ((256, False), (128, False), (256, True)):
        s = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_check_distance(7).with_input_delay(2)
             .with_checked_mismatches(False).with_debug_flags(flags).with_block_size(block)
             .with_lane_per_session(lps).start_synctest_session())
        s.run_ticks(inputs[:W0]); s.synchronize()
        s.profile_enable(1); s.profile_take()
        t0 = time.perf_counter(); s.run_ticks(inputs[W0:]); s.synchronize(); el = time.perf_counter() - t0
        ms, n = s.profile_take()
        print(f"{name:16s} block {block:3d} {'lps' if lps else 'lpp'}: kernel {ms / n * 1e3:7.2f} us   step {el / (T - W0) * 1e6:7.2f} us", flush=True)
        s.close()
