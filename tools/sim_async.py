"""Iteration-cost model of the lane-asynchronous P2P kernel (p2p.hpp kAsync) against
batched tick openings (VERDICT r03 "batch tick openings per wave").

A wave holds 32 sessions; per session and tick, a rollback happens with the
bench's measured probability (0.084 per session-tick at lag 1-4) and resimulates
1.64 frames on average (adv/session-tick 1.138).  Every loop iteration costs the
code paths some lane of the wave takes in it: the tick opening O (any lane opens
a tick), one AdvanceFrame F (always), the tick close C (any lane closes one).
'async' opens a lane's next tick as soon as it closed the last one (the product);
'batch k' lets a ready lane wait until k lanes are ready or no lane is mid-rollback.
The async iteration count matches the measured one (65 per 50 ticks,
tools/p2p_iters.py); every batching threshold costs more under every cost split
tried, so openings are not batched."""
import numpy as np

rng = np.random.default_rng(1)
T, N, TRIALS = 50, 32, 200
P_RB, MEAN_DEPTH = 0.084, 1.64


def depths():
    rb = rng.random((T, N)) < P_RB
    return np.where(rb, np.clip(rng.poisson(MEAN_DEPTH - 1, (T, N)) + 1, 1, 4), 0)


def sim(policy, O, C, F, thr=None):
    tot = iters = 0
    for _ in range(TRIALS):
        d = depths()
        t = np.zeros(N, int)
        rem = np.full(N, -1)  # -1: between ticks; >= 0: frames before the tick's new frame
        cost = it = 0
        while (t < T).any() or (rem >= 0).any():
            idle, busy = (rem < 0) & (t < T), rem >= 0
            if policy == "async":
                opening = idle
            else:
                opening = idle if (idle.sum() >= thr or not busy.any()) else np.zeros(N, bool)
            rem = np.where(opening, d[np.minimum(t, T - 1), np.arange(N)], rem)
            active = rem >= 0
            if not active.any():
                break
            closing = active & (rem == 0)
            cost += O * opening.any() + F + C * closing.any()
            rem = np.where(active, rem - 1, rem)
            t = np.where(closing, t + 1, t)
            it += 1
        tot += cost
        iters += it
    return tot / TRIALS, iters / TRIALS


if __name__ == "__main__":
    for O, C, F in [(1, 1, 1), (2, 1, 1), (1.5, 0.7, 1)]:
        print("O,C,F =", O, C, F)
        for pol, thr in [("async", None), ("batch", 8), ("batch", 16), ("batch", 24), ("batch", 28)]:
            c, i = sim(pol, O, C, F, thr)
            print(f"  {pol:6s} {str(thr):5s} cost {c:7.1f}  iterations per {T} ticks {i:6.1f}")
