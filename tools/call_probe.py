"""Host time of one rb_run_ticks call, rep by rep, in bench.py's timed-region
shape (synchronize, call, synchronize), to separate first-call costs from the
steady per-call cost (GPU box).  MODE=direct calls the C ABI straight from
ctypes (no Python wrapper)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import ggrs_amd as G

S, P, cd, steps = 65536, 2, 7, 20
reps = int(os.environ.get("REPS", "8"))
mode = os.environ.get("MODE", "wrapper")
GC = os.environ.get("GC", "1") == "1"  # GC=0: gc.collect() then gc.disable() before the reps
ZERO = os.environ.get("ZERO", "0") == "1"  # ZERO=1: a zero-tick run_ticks right before each rep
T = 13 + steps * reps
dev = torch.device("cuda", 0)
d = torch.from_numpy(G.synth_inputs(S, P, T)).to(dev)
stream = torch.cuda.Stream(device=dev)
sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S, device=0).with_num_players(P).with_check_distance(cd)
        .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
sess.set_stream(stream)
lib = G._lib.load()
with torch.cuda.stream(stream):
    sess.profile_enable(True)
    sess.run_ticks(d[0:8])
    sess.run_ticks(d[8:13])
    torch.cuda.synchronize()
    sess.profile_take()
    t = 13
    if not GC:
        import gc
        gc.collect()
        gc.disable()
    for r in range(reps):
        x = d[t:t + steps]
        ptr, done = ctypes.c_void_p(x.data_ptr()), ctypes.c_int32()
        torch.cuda.synchronize()
        if ZERO:
            sess.run_ticks(d[t:t])
        t0 = time.perf_counter()
        if mode == "direct":
            lib.rb_run_ticks(sess._h, steps, ptr, P * S, 1, ctypes.byref(done))
        else:
            sess.run_ticks(x)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ms, n = sess.profile_take()
        print(f"rep {r}: call {1e6 * (t1 - t0):6.1f} us  wall {1e6 * (t2 - t0):6.1f} us  kernel {1e3 * ms:6.1f} us",
              flush=True)
        t += steps
sess.close()
