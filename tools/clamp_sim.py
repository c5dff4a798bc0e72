"""Is ex_game's speed clamp a per-player regime that regrouping sessions could exploit?

Replays the bench's synthetic inputs (ggrs_amd.synth, the seed bench.py uses) through ex_game's
advance (ex_game.rs:259-321, numpy f32; statistics only, not the bit-exact path) for 16,384
sessions x 2 players x 1,600 frames, and prints: the clamp rate per lane-frame, the share of
wave-frames (32 sessions x 2 players) in which some lane clamps (the branch the whole wave runs),
per-player clamp fractions, whether clamping in one 400-frame window predicts the next, and the
wave-frame share after regrouping sessions by their clamp count in the previous window (once, and
every 20/50/100 frames).  DESIGN.md section 4.2 quotes its output.
    python3 tools/clamp_sim.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ggrs_amd.synth import synth_inputs  # noqa: E402

S, P, T = 16384, 2, 1600
f32 = np.float32


def main():
    inp = synth_inputs(S, P, T)  # [T, P, S]
    rot = np.zeros((P, S), f32)
    for i in range(P):
        rot[i] = f32((i / P * 2 * np.pi + np.pi) % (2 * np.pi))
    vx = np.zeros((P, S), f32)
    vy = np.zeros((P, S), f32)
    x = np.full((P, S), 300, f32)
    y = np.full((P, S), 400, f32)
    cl = np.zeros((T, P, S), bool)
    for t in range(T):
        a = inp[t].astype(np.int32)
        vx, vy = vx * f32(0.98), vy * f32(0.98)
        up, dn, lf, rt = (a & 1) != 0, (a & 2) != 0, (a & 4) != 0, (a & 8) != 0
        th = np.where(up & ~dn, 1, np.where(~up & dn, -1, 0)).astype(f32)
        vx = vx + th * f32(0.25) * np.cos(rot).astype(f32)
        vy = vy + th * f32(0.25) * np.sin(rot).astype(f32)
        step = f32(2.5 / 60)
        rot = np.where(lf & ~rt, (rot - step) % f32(2 * np.pi),
                       np.where(~lf & rt, (rot + step) % f32(2 * np.pi), rot)).astype(f32)
        m = np.sqrt(vx * vx + vy * vy)
        k = m > 7
        cl[t] = k
        safe = np.where(k, m, f32(1))
        vx = np.where(k, vx * 7 / safe, vx)
        vy = np.where(k, vy * 7 / safe, vy)
        x = np.clip(x + vx, 0, 600)
        y = np.clip(y + vy, 0, 800)

    def wave_any(c):
        n = c.shape[0]
        return c.reshape(n, P, S // 32, 32).any(axis=(1, 3))

    print("clamp rate per lane-frame", cl.mean())
    print("wave-frames with some lane clamping", wave_any(cl).mean())
    print("per-player clamp fraction quantiles 0.5/0.9/0.99/0.999", np.quantile(cl.mean(0), [0.5, 0.9, 0.99, 0.999]))
    a, b = cl[400:800].any(0), cl[800:1200].any(0)
    print("P(clamp in window 2 | clamp in window 1)", (a & b).sum() / max(1, a.sum()), " P(clamp in window 2)", b.mean())
    order = np.argsort(cl[400:800].any(1).sum(0), kind="stable")
    print("regrouped once by the previous window:", wave_any(cl[800:1200][:, :, order]).mean(),
          " unsorted:", wave_any(cl[800:1200]).mean())
    for win in (20, 50, 100):
        tot = n = 0
        for t0 in range(400, 1200, win):
            o = np.argsort(cl[t0 - win:t0].sum((0, 1)), kind="stable")
            w = wave_any(cl[t0:t0 + win][:, :, o])
            tot, n = tot + w.sum(), n + w.size
        print(f"regrouped every {win} frames:", tot / n)


if __name__ == "__main__":
    main()
