"""Phase clocks of one-tick P2P launches (A/B build with -DRB_P2P_PHASE=1, e.g.
tools/mkvar.sh phase -DRB_P2P_PHASE=1; run with GGRS_AMD_LIB=ggrs_amd/var/lib_phase.so):
per wave, the constant clock at entry, state loads in, poll + threshold done, rollback +
saves done, the tick's frame done, end; prints each phase's p50/p90/max and the launch span."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ggrs_amd as G  # noqa: E402
from ggrs_amd import _lib  # noqa: E402
from ggrs_amd.p2p import PlayerType, synth_network  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
T, W0 = 96, 48
inputs, upto, rin = synth_network(S, 2, T, 0b1, 2, 1, 4)
di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
b = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(2).with_max_prediction_window(8)
     .with_input_delay(2).with_remote_input_delay(2))
b.add_player(PlayerType.Local, 0)
b.add_player(PlayerType.Remote, 1)
sess = b.start_p2p_session()
lib = _lib.load()
buf = np.zeros(8 * 4096, dtype=np.uint64)
names = ["state loads", "poll+threshold", "rollback+saves", "tick frame", "epilogue"]
acc = {n: [] for n in names}
spans = []
for t in range(T):
    sess.run_ticks(di[t:t + 1], du[t:t + 1], dr)
    if t < W0:
        continue
    torch.cuda.synchronize()
    assert lib.rb_debug_p2p_phase(buf.ctypes.data_as(ctypes.c_void_p), 4096) == 0
    r = buf.reshape(-1, 8)[:2048].astype(np.int64)
    ok = (r[:, :6] > 0).all(axis=1)
    r = r[ok]
    t0 = r[:, 0].min()
    spans.append((r[:, 5].max() - t0) / 100.0)
    for i, n in enumerate(names):
        acc[n].append((r[:, i + 1] - r[:, i]) / 100.0)
    if t == T - 1:
        print(f"waves recorded {ok.sum()}; entry skew p50/max {np.percentile((r[:, 0] - t0) / 100, 50):.2f}/"
              f"{(r[:, 0].max() - t0) / 100:.2f} us; loads per wave p50 {np.percentile(r[:, 7] >> 32, 50)}")
print(f"span (first entry to last end) p50 {np.percentile(spans, 50):.2f} us over {len(spans)} launches")
for n in names:
    a = np.concatenate(acc[n])
    print(f"  {n:16s} p50 {np.percentile(a, 50):6.2f}  p90 {np.percentile(a, 90):6.2f}  max {a.max():6.2f} us")
end = np.concatenate([[0]])
