"""Which live kernel timer agrees with rocprofv3 (GPU box; VERDICT r05 "next" 1).

The SyncTest steady kernel at 65,536 sessions, launched REPS times at each launch length
(1, 20 and 50 ticks) under each timer, in this fixed order (so a rocprofv3 --kernel-trace of
the same command can be matched dispatch by dispatch):
  own1   the launch's own events (hipExtLaunchKernel), one launch at a time
  ownbb  the launch's own events, REPS launches queued back to back
  mark1  a torch event pair on the stream around each launch, one at a time
  markbb one torch event pair around REPS back-to-back launches (per-launch average)
  clock  the kernel's own first-wave start / last-wave end on the 100 MHz constant clock
         (rb_launch_clock_arm / rb_launch_clock_read; in-kernel, so rocprofv3 cannot perturb it), one at a time
Prints one JSON line per (length, timer): per-launch microseconds (median, mean, list).
    python3 tools/timer_check.py > gpurun_out/tc.jsonl
    rocprofv3 --kernel-trace -d gpurun_out/tc_prof -o run --output-format csv -- python3 tools/timer_check.py
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ggrs_amd as G  # noqa: E402

S = int(os.environ.get("S", "65536"))
REPS = int(os.environ.get("REPS", "6"))
LENS = [int(x) for x in os.environ.get("LENS", "1,20,50").split(",")]
TIMERS = os.environ.get("TIMERS", "own1,ownbb,mark1,markbb,clock").split(",")
P, cd = 2, 7
T = 13 + sum(LENS) * REPS * len(TIMERS) + 8
dev = torch.device("cuda", 0)
d = torch.from_numpy(G.synth_inputs(S, P, T)).to(dev)
stream = torch.cuda.Stream(device=dev)
sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S, device=0).with_num_players(P).with_check_distance(cd)
        .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
sess.set_stream(stream)
with torch.cuda.stream(stream):
    sess.run_ticks(d[0:13])
    torch.cuda.synchronize()
    t = 13
    for L in LENS:
        for tm in TIMERS:
            calls = []
            for _ in range(REPS):
                calls.append(sess.prepare_ticks(d[t:t + L])[0])
                t += L
            us = []
            sess.profile_enable(tm in ("own1", "ownbb"))
            sess.profile_take()
            if tm in ("own1", "mark1", "clock"):
                for c in calls:
                    if tm == "mark1":
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                    if tm == "clock":
                        sess.launch_clock_arm(1)
                    assert c() == 0
                    if tm == "mark1":
                        e1.record()
                    torch.cuda.synchronize()
                    if tm == "own1":
                        ms, n = sess.profile_take()  # (ms, ticks covered): one launch
                        us.append(ms * 1e3)
                    elif tm == "mark1":
                        us.append(e0.elapsed_time(e1) * 1e3)
                    else:
                        us += sess.launch_clock_read(1)
            else:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for c in calls:
                    assert c() == 0
                e1.record()
                torch.cuda.synchronize()
                if tm == "ownbb":
                    ms, n = sess.profile_take()
                    us = [ms * 1e3 / REPS]
                else:
                    us = [e0.elapsed_time(e1) * 1e3 / REPS]
            sess.profile_enable(False)
            print(json.dumps({"len": L, "timer": tm, "reps": REPS, "median_us": statistics.median(us),
                              "mean_us": statistics.mean(us), "us": us}), flush=True)
sess.close()
