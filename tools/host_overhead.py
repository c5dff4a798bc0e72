"""Where the driver's 20-step wall time goes (GPU box): the run_ticks call on
the host, the wall time to the end of a synchronize, and the kernel time from
HIP events; with and without the profiling events, with device vs stream
synchronize, and the floor of one trivial launch + synchronize.

SPIN=early|late|0 (default 0): hipSetDeviceFlags(hipDeviceScheduleSpin) before
the first GPU call, after it, or not at all (HIP's default wait blocks on an
interrupt once a short active wait has passed)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch

SPIN = os.environ.get("SPIN", "0")


def set_spin():
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded (same soname)
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
    print(f"hipSetDeviceFlags(spin) -> {rc}", flush=True)


if SPIN == "early":
    set_spin()
import ggrs_amd as G
S, P, cd, steps = 65536, 2, 7, int(os.environ.get("STEPS", "20"))
reps = 12
T = 8 + 5 + steps * (7 * reps + 2) + 200
inputs = G.synth_inputs(S, P, T)
dev = torch.device("cuda", 0)
d = torch.from_numpy(inputs).to(dev)
if SPIN == "late":
    set_spin()
stream = torch.cuda.Stream(device=dev)
sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S, device=0).with_num_players(P).with_check_distance(cd)
        .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
sess.set_stream(stream)
lib = G._lib.load()
t = 13


def rows(label, prof, sync, direct=False, double=False):
    global t
    out = []
    for rep in range(reps):
        x = d[t:t + steps]
        sess.profile_enable(prof)
        sess.profile_take()
        torch.cuda.synchronize()
        if direct:
            ptr = ctypes.c_void_p(x.data_ptr())
            done = ctypes.c_int32()
            stride = P * S
        t0 = time.perf_counter()
        if direct:
            lib.rb_run_ticks(sess._h, steps, ptr, stride, 1, ctypes.byref(done))
        else:
            sess.run_ticks(x)
        t1 = time.perf_counter()
        sync()
        if double:
            sync()
        t2 = time.perf_counter()
        ms, n = sess.profile_take()
        out.append((1e6 * (t1 - t0), 1e6 * (t2 - t0), 1e3 * ms))
        t += steps
    a = np.array(out[2:])
    med = np.median(a, 0)
    print(f"{label:40s} call {med[0]:7.1f} us  wall {med[1]:7.1f} us  kernel {med[2]:7.1f} us  "
          f"(min wall {a[:, 1].min():.1f})", flush=True)


with torch.cuda.stream(stream):
    sess.run_ticks(d[0:13])
    torch.cuda.synchronize()
    rows("prof on, device sync x2 (bench.py)", True, torch.cuda.synchronize, double=True)
    rows("prof on, device sync", True, torch.cuda.synchronize)
    rows("prof off, device sync", False, torch.cuda.synchronize)
    rows("prof on, stream sync", True, stream.synchronize)
    rows("prof off, stream sync", False, stream.synchronize)
    rows("prof on, direct rb_run_ticks, dev sync", True, torch.cuda.synchronize, direct=True)
    rows("prof off, direct rb_run_ticks, dev sync", False, torch.cuda.synchronize, direct=True)
    # floor: one trivial kernel + synchronize on the same stream
    z = torch.zeros(64, device=dev)
    w = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        z.add_(1)
        torch.cuda.synchronize()
        w.append(1e6 * (time.perf_counter() - t0))
    print(f"{'trivial torch launch + sync':40s} wall {np.median(w[2:]):7.1f} us", flush=True)
    w = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        w.append(1e6 * (time.perf_counter() - t0))
    print(f"{'idle synchronize':40s} wall {np.median(w[2:]):7.1f} us", flush=True)
    # per-tick launches (live play: one tick of inputs per call)
    sess.profile_enable(True)
    sess.profile_take()
    torch.cuda.synchronize()
    n1 = 64
    t0 = time.perf_counter()
    for k in range(n1):
        sess.run_ticks(d[t + k:t + k + 1])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ms, n = sess.profile_take()
    t += n1
    print(f"{'one tick per call':40s} call {1e6*(t1-t0)/n1:7.1f} us/tick  wall {1e6*(t2-t0)/n1:7.1f} us/tick  "
          f"kernel {1e3*ms/max(1,n):7.1f} us/tick", flush=True)
    # one tick per call, synchronised every tick (a 60 Hz loop waits for its tick)
    sess.profile_enable(False)
    w = []
    for k in range(n1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sess.run_ticks(d[t + k:t + k + 1])
        torch.cuda.synchronize()
        w.append(1e6 * (time.perf_counter() - t0))
    print(f"{'one tick per call + sync (latency)':40s} wall {np.median(w[2:]):7.1f} us", flush=True)
sess.close()
