"""Peer-reported disconnects: update_player_disconnects (p2p_session.rs:707-742)
over the peers' connect-status reports (UdpProtocol::peer_connect_status,
protocol.rs:627-636), disconnect_player_at_frame (:555-581) and the
resimulation from the reported frame.

GGRS 0.9.4 restated as written: disconnect_player_at_frame marks the player
disconnected and schedules the rollback but does not move the player's
last_frame to the reported frame (GGPO's DisconnectPlayerQueue does), so a
peer reporting an earlier frame than we hold keeps re-triggering the rollback
every tick until load_frame's window assert fires (sync_layer.rs:141-145).
The device batch must reproduce that too, tick for tick.
"""
import numpy as np
import pytest

import ggrs_amd as G
from ggrs_amd._lib import RB_PANIC
from ggrs_amd.p2p import PlayerType, synth_network
from oracle import oracle as O
from test_p2p import compare_queues

P, W, D, RD = 3, 8, 1, 2
MASK = 0b001  # handle 0 local; handles 1, 2 remote (each its own endpoint)


def drive(orc, inputs, upto, rin, t):
    for h in range(P):
        if not (MASK >> h) & 1:
            orc.deliver(h, upto[t, h], rin[:, h, :])
    orc.add_local_input(0, inputs[t, 0])
    return orc.advance()


def reports(S, upto, t):
    """Connect-status reports (endpoint, last_frames [P, S], disconnected [P, S]) given before tick t
    (they reach update_player_disconnects after tick t's poll, like the reports riding on that
    poll's input messages):
    sessions 0..7: endpoint 2 reports player 1 disconnected at the frame we hold (no re-trigger);
    8..15: at 2 frames before it (GGRS re-triggers the disconnect every tick -> a panic);
    16..23: endpoint 1 reports the LOCAL player 0 disconnected (disconnect_player_at_frame: no-op);
    24..: plain connected reports."""
    held = upto[t]  # frames delivered through tick t's poll, per remote handle
    out = []
    for e in (1, 2):
        last = np.full((P, S), -1, np.int32)
        disc = np.zeros((P, S), np.uint8)
        for i in range(P):
            last[i] = np.maximum(held[i] if i != 0 else t - 1 + D, -1)
        if e == 2:
            disc[1, 0:8] = 1
            disc[1, 8:16] = 1
            last[1, 8:16] = held[1, 8:16] - 2
        if e == 1:
            disc[0, 16:24] = 1
        out.append((e, last, disc))
    return out


def test_oracle_peer_reported_disconnects():
    S, T, t_rep = 32, 60, 25
    inputs, upto, rin = synth_network(S, P, T, MASK, RD, 1, 3)
    orc = O.OracleP2P(O.EX_GAME, P, W, D, MASK, S, remote_delay=RD)
    panicked_at = np.full(S, -1)
    held = upto[t_rep, 1]
    frame = np.where(np.arange(S) < 8, held, held - 2)[:16]  # the reported frame F
    for t in range(T):
        if t == t_rep:
            for e, last, disc in reports(S, upto, t):
                orc.receive_peer_connect_status(e, last, disc)
            cur = orc.frames()[0][:16]  # each session's current frame (PredictionThreshold ticks lag)
        st, lf, _, _ = drive(orc, inputs, upto, rin, t)
        panicked_at[(st == O.KIND_PANIC) & (panicked_at < 0)] = t
        if t == t_rep:
            st_rep = st.copy()
            # disconnect_player_at_frame(1, F): disconnect_frame = F + 1 when current > F.  F + 1 ==
            # current loads the current frame, which load_frame's assert refuses (sync_layer.rs:141-145),
            # unless another player's misprediction rolls back further in the same tick.
            pan = st[:16] == O.KIND_PANIC
            assert (frame[pan] == cur[pan] - 1).all()
            back = (frame < cur) & ~pan
            assert ((lf[:16][back] >= 0) & (lf[:16][back] <= frame[back] + 1)).all()
            at_cur = (frame == cur - 1) & ~pan
            assert (lf[:16][at_cur] <= frame[at_cur]).all()
    ok = st_rep[:8] != O.KIND_PANIC
    assert ok.any() and (panicked_at[:8][ok] == -1).all()  # reported at the frame we hold: once
    assert (panicked_at[8:16] >= t_rep).all()  # re-triggered every tick until an assert fires
    assert (panicked_at[16:] == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_gpu_peer_reported_disconnects_match_oracle_every_tick(gpu_available, sparse):
    import torch
    S, T, t_rep = 64, 60, 25
    inputs, upto, rin = synth_network(S, P, T, MASK, RD, 1, 3)
    b = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
         .with_input_delay(D).with_remote_input_delay(RD).with_sparse_saving_mode(sparse)
         .with_peer_connect_status(True))
    for h in range(P):
        b.add_player(PlayerType.Local if (MASK >> h) & 1 else PlayerType.Remote, h)
    sess = b.start_p2p_session()
    orc = O.OracleP2P(O.EX_GAME, P, W, D, MASK, S, sparse_saving=sparse, remote_delay=RD)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    alive = np.ones(S, bool)
    for t in range(T):
        if t == t_rep:
            for e, last, disc in reports(S, upto, t):
                orc.receive_peer_connect_status(e, last, disc)
                sess.receive_peer_connect_status(e, torch.from_numpy(last).cuda(), torch.from_numpy(disc).cuda())
        sess.run_ticks(di[t:t + 1], du[t:t + 1], dr)
        ost, olf, ona, ons = drive(orc, inputs, upto, rin, t)
        st, lf, na, ns = sess.status()
        np.testing.assert_array_equal(st, np.where(ost == O.KIND_PANIC, RB_PANIC, ost), err_msg=f"status, tick {t}")
        alive &= ost != O.KIND_PANIC
        np.testing.assert_array_equal(lf[alive], olf[alive], err_msg=f"load frame, tick {t}")
        np.testing.assert_array_equal(na[alive], ona[alive], err_msg=f"AdvanceFrames, tick {t}")
        np.testing.assert_array_equal(ns[alive], ons[alive], err_msg=f"SaveGameStates, tick {t}")
        compare_queues(sess, orc, t, alive)
        if t % 5 == 4:
            np.testing.assert_array_equal(sess.read_live()[alive], orc.read_live()[0][alive], err_msg=f"live, tick {t}")
            c, k = sess.frames()
            oc, ok = orc.frames()
            np.testing.assert_array_equal(c[alive], oc[alive])
            np.testing.assert_array_equal(k[alive], ok[alive])
    assert alive[16:].all() and alive[:8].any() and not alive[8:16].any()
    sess.close()
