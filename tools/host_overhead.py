"""Where the driver's 20-step wall time goes: host call vs kernel vs sync (GPU box)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import ggrs_amd as G
S, P, cd, steps = 65536, 2, 7, 20
T = 8 + 5 + steps * 12
inputs = G.synth_inputs(S, P, T)
dev = torch.device("cuda", 0)
d = torch.from_numpy(inputs).to(dev)
stream = torch.cuda.Stream(device=dev)
sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S, device=0).with_num_players(P).with_check_distance(cd)
        .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
sess.set_stream(stream)
with torch.cuda.stream(stream):
    for t in range(13):
        sess.run_ticks(d[t:t + 1])
    torch.cuda.synchronize()
    t = 13
    for rep in range(10):
        x = d[t:t + steps]
        sess.profile_enable(True); sess.profile_take()
        t0 = time.perf_counter()
        sess.run_ticks(x)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ms, n = sess.profile_take()
        print(f"call {1e6*(t1-t0):7.1f} us  wall {1e6*(t2-t0):7.1f} us  kernel {1e3*ms:7.1f} us")
        t += steps
