"""Experiment (RB_P2P_EXP=4 builds only, tools/mkvar.sh): loop iterations per
wave and launch of the lane-asynchronous P2P kernel, next to the AdvanceFrames
the sessions executed, for the bench's P2P workload.  The build reports the
summed per-wave iteration maxima through the unexpected-path counter."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ggrs_amd as G  # noqa: E402
from ggrs_amd.p2p import PlayerType, synth_network  # noqa: E402

S, P, W, T, TPL = 65536, 2, 8, 432, 50
lo, hi = (int(x) for x in os.environ.get("LAG", "1,4").split(","))
inputs, upto, rin = synth_network(S, P, T, 1, 2, lo, hi, seed=0x67677273, first_session=0)
di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
b = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
     .with_input_delay(2).with_remote_input_delay(2))
for h in range(P):
    b.add_player(PlayerType.Local if h == 0 else PlayerType.Remote, h)
s = b.start_p2p_session()
for t in range(0, 32, 16):
    s.run_ticks(di[t:t + 16], du[t:t + 16], dr)
torch.cuda.synchronize()
a0, c0 = s.totals(), s.counters()
launches = 0
for t in range(32, T, TPL):
    s.run_ticks(di[t:t + TPL], du[t:t + TPL], dr)
    launches += 1
torch.cuda.synchronize()
a1, c1 = s.totals(), s.counters()
waves = S * 2 // 64
it = (c1[1] - c0[1]) / waves / launches
adv = (a1[0] - a0[0]) / S / (T - 32)
print(f"lag {lo},{hi}: {it:.1f} iterations per wave-launch of {TPL} ticks; {adv:.3f} AdvanceFrames per session-tick")
