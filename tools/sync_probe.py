"""Where the driver command's wall time outside the kernel goes (GPU box).

One rb_run_ticks call of STEPS fused ticks per rep, in bench.py's timed-region
shape (synchronize, call, synchronize), with the closing wait done several ways:
  device  torch.cuda.synchronize() (hipDeviceSynchronize; what bench.py uses)
  stream  stream.synchronize() then torch.cuda.synchronize()
  event   an event recorded after the call, event.synchronize(), then torch.cuda.synchronize()
and the launch with (EV=1) or without (EV=0) the kernel's own profiling events.
Also times an empty torch kernel + synchronize (the floor of any launch + wait).
Prints one line per (mode, ev): median / min wall per call and the kernel time."""
import ctypes
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ggrs_amd as G  # noqa: E402

S = int(os.environ.get("S", "65536"))
P, cd, steps = 2, 7, int(os.environ.get("STEPS", "20"))
reps = int(os.environ.get("REPS", "12"))
modes = os.environ.get("MODES", "device,stream,event").split(",")
evs = [int(x) for x in os.environ.get("EVS", "1,0").split(",")]
T = 13 + steps * reps * len(modes) * len(evs) + 8
dev = torch.device("cuda", 0)
d = torch.from_numpy(G.synth_inputs(S, P, T)).to(dev)
stream = torch.cuda.Stream(device=dev)
sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S, device=0).with_num_players(P).with_check_distance(cd)
        .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
sess.set_stream(stream)
with torch.cuda.stream(stream):
    sess.profile_enable(True)
    sess.run_ticks(d[0:8])
    sess.run_ticks(d[8:13])
    torch.cuda.synchronize()
    sess.profile_take()
    t = 13
    x = torch.zeros(1, device=dev)
    fl = []
    for r in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        fl.append(time.perf_counter() - t0)
    print(f"floor: empty torch kernel + synchronize: median {1e6 * statistics.median(fl):.1f} us, "
          f"min {1e6 * min(fl):.1f} us", flush=True)
    for ev in evs:
        sess.profile_enable(bool(ev))
        sess.profile_take()
        for mode in modes:
            walls, calls, kers = [], [], []
            done_ev = torch.cuda.Event()
            done_ev.record()
            for r in range(reps):
                call, check = sess.prepare_ticks(d[t:t + steps])
                t += steps
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                st = call()
                t1 = time.perf_counter()
                if mode == "stream":
                    stream.synchronize()
                elif mode == "event":
                    done_ev.record()
                    done_ev.synchronize()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                if st:
                    check(st)
                ms, n = sess.profile_take()
                walls.append(t2 - t0)
                calls.append(t1 - t0)
                if n:
                    kers.append(ms * 1e3 / n)
            k = f"kernel median {statistics.median(kers):.1f} us" if kers else "kernel (no events)"
            print(f"ev={ev} sync={mode:6s}: wall median {1e6 * statistics.median(walls):.1f} us, min "
                  f"{1e6 * min(walls):.1f}, call median {1e6 * statistics.median(calls):.1f} us, {k}", flush=True)
sess.close()
