"""Per-wave timing of the SyncTest steady kernel (A/B build with -DRB_WAVE_CLOCK=1, e.g.
tools/mkvar.sh wclk -DRB_WAVE_CLOCK=1; run with GGRS_AMD_LIB=ggrs_amd/var/lib_wclk.so).
Every wave records its start and end (s_memrealtime, 100 MHz), its XCC and HW_ID, and how many
ticks it ran in the general form; this prints how the launch's span splits into start skew,
wave lifetimes and the tail, by XCC and by SIMD slot."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ggrs_amd as G  # noqa: E402
from ggrs_amd import _lib  # noqa: E402

S = int(os.environ.get("S", 65536))
TPL = int(os.environ.get("TPL", 50))
W0 = int(os.environ.get("W0", 32))
T = W0 + 3 * TPL
inputs = torch.from_numpy(G.synth_inputs(S, 2, T)).cuda()
s = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_check_distance(7).with_input_delay(2)
     .with_checked_mismatches(False).start_synctest_session())
s.run_ticks(inputs[:W0])
lib = _lib.load()
buf = np.zeros(4 * 8192, dtype=np.uint64)
for c in range(W0, T, TPL):
    s.run_ticks(inputs[c:c + TPL])
    s.synchronize()
    assert lib.rb_debug_wave_clock(buf.ctypes.data_as(ctypes.c_void_p), 8192) == 0
    nw = (S * 2 + 63) // 64
    r = buf.reshape(-1, 4)[:nw].astype(np.int64)
    st, en, hw, gen = r[:, 0], r[:, 1], r[:, 2], r[:, 3] & 0xFF
    t0 = st.min()
    life = (en - st) / 100.0  # us
    extra = r[:, 3]
    clamp = extra >> 40
    print(f"  block waves {np.unique((extra >> 16) & 0xFF)}; frames with a clamp per wave mean {clamp.mean():.0f} of "
          f"{8 * TPL}, min/max {clamp.min()}/{clamp.max()}; lifetime corr {np.corrcoef(clamp, life)[0, 1]:.2f}")
    span = (en.max() - t0) / 100.0
    xcc = (hw >> 32) & 0xF
    hid = hw & 0xFFFFFFFF
    simd, cu, sh, se = (hid >> 4) & 3, (hid >> 8) & 0xF, (hid >> 12) & 1, (hid >> 13) & 7
    print(f"launch of {TPL} ticks: span {span:.1f} us; start skew p50/p90/max {np.percentile((st - t0) / 100, 50):.1f}/"
          f"{np.percentile((st - t0) / 100, 90):.1f}/{(st.max() - t0) / 100:.1f} us; lifetime min/p10/p50/p90/max "
          + "/".join(f"{v:.1f}" for v in np.percentile(life, [0, 10, 50, 90, 100])) + " us; "
          f"end p10/p50/max {np.percentile((en - t0) / 100, 10):.1f}/{np.percentile((en - t0) / 100, 50):.1f}/{span:.1f}")
    print("  mean lifetime by XCC: " + " ".join(f"{x}:{life[xcc == x].mean():.1f}" for x in range(8) if (xcc == x).any()))
    print(f"  general-form ticks per wave: mean {gen.mean():.2f}, max {gen.max()}; lifetime corr {np.corrcoef(gen, life)[0, 1]:.2f}"
          if gen.std() > 0 else "  no general-form ticks")
    slot = hid & 0xF
    BS = int(os.environ.get("BLOCK_WAVES", 4))
    blk = np.arange(nw) // BS
    wib = np.arange(nw) % BS
    print(f"  waves on SIMD (wave in block % 4): {(simd == wib % 4).mean():.2f} of waves")
    print("  lifetime by HW wave slot: " + " ".join(f"{w}:{life[slot == w].mean():.1f}(n={int((slot == w).sum())})"
                                                     for w in range(16) if (slot == w).any()))
    print("  lifetime by block index < or >= 256: %.1f / %.1f" % (life[blk < 256].mean(), life[blk >= 256].mean()))
    h, e = np.histogram(life, bins=12)
    print("  histogram: " + " ".join(f"{e[i]:.0f}:{h[i]}" for i in range(len(h))))
    # the two waves sharing a SIMD: same XCC/SE/SH/CU/SIMD
    sk = ((((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd)
    order = np.lexsort((st, sk))
    pairs = [(order[i], order[i + 1]) for i in range(0, len(order) - 1) if sk[order[i]] == sk[order[i + 1]]]
    if pairs:
        a = np.array([life[i] for i, _ in pairs]); b = np.array([life[j] for _, j in pairs])
        sa = np.array([slot[i] for i, _ in pairs]); sb = np.array([slot[j] for _, j in pairs])
        ba = np.array([blk[i] for i, _ in pairs]); bb = np.array([blk[j] for _, j in pairs])
        print(f"  {len(pairs)} SIMD pairs: first-started wave lifetime {a.mean():.1f}, second {b.mean():.1f}; "
              f"first shorter in {(a < b).mean():.2f}; slots (first,second) e.g. {list(zip(sa[:6], sb[:6]))}; "
              f"blocks e.g. {list(zip(ba[:6], bb[:6]))}; |shorter-longer| mean {np.abs(a - b).mean():.1f}")
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    cus = {}
    for k, l, sd in zip(key, life, simd):
        cus.setdefault(k, []).append(l)
    per_cu = np.array([np.mean(v) for v in cus.values()])
    cnt = np.array([len(v) for v in cus.values()])
    print(f"  {len(cus)} CUs used; waves per CU min/max {cnt.min()}/{cnt.max()}; CU mean lifetime min/p50/max "
          f"{per_cu.min():.1f}/{np.median(per_cu):.1f}/{per_cu.max():.1f} us", flush=True)
s.close()
