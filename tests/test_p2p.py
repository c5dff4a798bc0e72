"""P2PSession rollback: the network-free oracle restatement
(oracle/ggrs_oracle.hpp P2PSession) and, on the GPU, the device batch
(ggrs_amd/csrc/p2p.hpp) against it.

Pinning: the reference's own P2P test (tests/test_p2p_session.rs:97-145, two
peers exchanging inputs: game frame == i + 1 after every advance) is restated
with two oracle sessions delivering to each other.  Beyond that the oracle is
a restatement (parity unpinned numerically, as for SyncTest), checked here by
a property every correct rollback must have: the cells of confirmed frames
equal those of a run in which every remote input arrived before it was needed.
"""
import numpy as np
import pytest

import ggrs_amd as G
from ggrs_amd._lib import RB_PANIC
from ggrs_amd.p2p import PlayerType, synth_network
from oracle import oracle as O

ORC_GAME = {G.Game.EX_GAME: O.EX_GAME, G.Game.STUB: O.STUB, G.Game.STUB_ENUM: O.STUB_ENUM, G.Game.BRAWLER: O.BRAWLER}


def drive_oracle(orc, local_mask, inputs, upto, remote_in, T, t0=0, disc=None):
    """Ticks [t0, T) of the oracle batch; returns per-tick (status, load, nadv, nsave).
    disc: {tick: [(handle, session mask)]} disconnect_player calls before that tick."""
    out = []
    P = inputs.shape[1]
    for t in range(t0, T):
        for h, m in (disc or {}).get(t, []):
            assert orc.disconnect_player(h, m) == 0
        for h in range(P):
            if not (local_mask >> h) & 1:
                assert orc.deliver(h, upto[t, h], remote_in[:, h, :]) == 0, orc.last_panic()
        for h in range(P):
            if (local_mask >> h) & 1:
                assert orc.add_local_input(h, inputs[t, h]) == 0
        out.append(orc.advance())
    return out


# ---------------------------------------------------------------------------- oracle (CPU)
def test_oracle_two_peers_advance_like_reference_test():
    # tests/test_p2p_session.rs:97-145: sess1 (local 0, remote 1) and sess2
    # (remote 0, local 1) exchange StubInput{inp: i}; after each advance both
    # games are at frame i + 1.  Inputs sent by one peer reach the other before
    # its next advance (the poll_remote_clients of the next iteration).
    s1 = O.OracleP2P(O.STUB, 2, 8, 0, 0b01, 1)
    s2 = O.OracleP2P(O.STUB, 2, 8, 0, 0b10, 1)
    sent1, sent2 = [], []  # inputs each peer added, by frame
    for i in range(10):
        if sent2:
            s1.deliver(1, [len(sent2) - 1], np.array(sent2, np.uint32)[:, None])
        if sent1:
            s2.deliver(0, [len(sent1) - 1], np.array(sent1, np.uint32)[:, None])
        s1.add_local_input(0, [i])
        st, _, _, _ = s1.advance()
        assert st[0] == 0
        sent1.append(i)
        s2.add_local_input(1, [i])
        st, _, _, _ = s2.advance()
        assert st[0] == 0
        sent2.append(i)
        img1, fr1 = s1.read_live()
        img2, fr2 = s2.read_live()
        assert int(np.frombuffer(img1[0, :4].tobytes(), np.int32)[0]) == i + 1
        assert int(np.frombuffer(img2[0, :4].tobytes(), np.int32)[0]) == i + 1


@pytest.mark.parametrize("game", [G.Game.STUB, G.Game.EX_GAME])
@pytest.mark.parametrize("sparse", [False, True])
def test_oracle_rollback_reaches_the_confirmed_truth(game, sparse):
    S, P, W, T, mask = 16, 2, 8, 120, 0b01
    dt = np.uint32 if game == G.Game.STUB else np.uint8
    inputs, upto, rin = synth_network(S, P, T, mask, remote_delay=1, min_lag=1, max_lag=5, dtype=dt,
                                      mask=0x3 if game == G.Game.STUB else 0x0F)
    lag = O.OracleP2P(ORC_GAME[game], P, W, 2, mask, S, sparse_saving=sparse, remote_delay=1)
    res = drive_oracle(lag, mask, inputs, upto, rin, T)
    assert all((r[0] == 0).all() for r in res), "no PredictionThreshold / panic expected"
    loads = np.array([r[1] for r in res])
    assert (loads != G.NULL_FRAME).sum() > S, "the schedule must cause rollbacks"
    # ground truth: every remote input delivered before the first advance
    truth = O.OracleP2P(ORC_GAME[game], P, W, 2, mask, S, sparse_saving=False, remote_delay=1)
    full = np.full((T, P, S), T, np.int32)
    seen = {}  # (session, frame) -> (image, checksum) of every cell the truth run saved
    for t in range(T):
        r = drive_oracle(truth, mask, inputs, full, rin, t + 1, t0=t)[0]
        assert (r[1] == G.NULL_FRAME).all(), "no rollback with everything delivered"
        ttags, timgs, tcs = truth.read_cells()
        for w in range(W):
            for s in range(S):
                if ttags[w, s] >= 0:
                    seen[(s, int(ttags[w, s]))] = (timgs[w, s].copy(), tcs[w, s].copy())
    cur, conf = lag.frames()
    tags, imgs, cs = lag.read_cells()
    checked = 0
    for s in range(S):
        for w in range(W):
            f = int(tags[w, s])
            if f < 0 or f > conf[s]:
                continue
            timg, tc = seen[(s, f)]
            np.testing.assert_array_equal(imgs[w, s], timg, err_msg=f"session {s} frame {f}")
            assert (cs[w, s] == tc).all()
            checked += 1
    assert checked >= S


def test_oracle_prediction_threshold_drops_the_requests():
    # A peer that stops sending: after max_prediction frames advance_frame
    # returns PredictionThreshold and the game no longer moves.
    S, P, W, T, mask = 4, 2, 4, 12, 0b01
    inputs, upto, rin = synth_network(S, P, T, mask, remote_delay=0, min_lag=1, max_lag=1)
    upto[:] = np.where(np.arange(T)[:, None, None] < 3, upto, upto[2])  # deliveries stop after tick 2
    orc = O.OracleP2P(O.EX_GAME, P, W, 0, mask, S)
    res = drive_oracle(orc, mask, inputs, upto, rin, T)
    st = np.array([r[0] for r in res])
    assert (st[-1] == 1).all() and (st[0] == 0).all()
    cur, _ = orc.frames()
    assert (cur < T).all()


INVALID_REQUEST = 2  # ggrs_oracle.hpp ErrorKind::InvalidRequest


def test_oracle_disconnect_player_errors_like_reference_test():
    # tests/test_p2p_session.rs:45-63 (the spectator handle is not part of the batch)
    orc = O.OracleP2P(O.STUB, 2, 8, 0, 0b01, 3)
    assert orc.disconnect_player(5) == INVALID_REQUEST  # invalid handle
    assert orc.disconnect_player(0) == INVALID_REQUEST  # local players cannot be disconnected
    assert orc.disconnect_player(1) == 0
    assert orc.disconnect_player(1) == INVALID_REQUEST  # already disconnected


def test_oracle_disconnect_at_the_current_frame_asserts_like_reference():
    # disconnect_player_at_frame sets disconnect_frame = last_frame + 1 whenever
    # current_frame > last_frame (p2p_session.rs:576-580).  With last_frame =
    # current_frame - 1 that is the current frame itself, and adjust_gamestate's
    # load_frame asserts frame_to_load < current_frame (sync_layer.rs:141-145).
    # One frame older, the session rolls back one frame and goes on.
    S, P, mask = 2, 2, 0b01
    orc = O.OracleP2P(O.EX_GAME, P, 8, 0, mask, S)
    by_frame = np.zeros((16, S), np.uint8)
    for t in range(4):
        orc.deliver(1, [t, t - 1], by_frame)  # after tick 3: session 0 holds frame 3, session 1 frame 2
        orc.add_local_input(0, [1, 1])
        assert (orc.advance()[0] == 0).all()
    assert orc.disconnect_player(1) == 0
    orc.add_local_input(0, [1, 1])
    st, lf, na, _ = orc.advance()
    assert st[0] == O.KIND_PANIC
    assert st[1] == 0 and lf[1] == 3 and na[1] == 2  # load frame 3, resimulate it, advance frame 4


def disconnect_schedule(upto, t0, h):
    """The last frame each session had received from handle h when it is
    disconnected before tick t0, and a delivery schedule that hands exactly
    those frames over before the first tick."""
    last = upto[t0 - 1, h].copy() if t0 > 0 else np.full(upto.shape[2], -1, np.int32)
    full = upto.copy()
    full[:, h, :] = last[None, :]
    return last, full


@pytest.mark.parametrize("game", [G.Game.STUB, G.Game.EX_GAME])
@pytest.mark.parametrize("sparse", [False, True])
def test_oracle_disconnect_resimulates_to_the_disconnected_truth(game, sparse):
    # After disconnect_player(h) every frame past h's last input is advanced with
    # (zeroed, Disconnected), including the frames already simulated on a
    # prediction (disconnect_frame = last_frame + 1, p2p_session.rs:576-580).
    # So the late-delivery run must end with the same cells and state as a run
    # in which h's inputs up to its last frame all arrived before tick 0.
    S, P, W, T, mask, h, t0 = 24, 3, 8, 90, 0b001, 2, 40
    dt = np.uint32 if game == G.Game.STUB else np.uint8
    inputs, upto, rin = synth_network(S, P, T, mask, remote_delay=1, min_lag=1, max_lag=5, dtype=dt,
                                      mask=0x3 if game == G.Game.STUB else 0x0F)
    last, full_h = disconnect_schedule(upto, t0, h)
    lag = O.OracleP2P(ORC_GAME[game], P, W, 1, mask, S, sparse_saving=sparse, remote_delay=1)
    res = drive_oracle(lag, mask, inputs, upto, rin, T, disc={t0: [(h, None)]})
    assert all((r[0] == 0).all() for r in res)
    loads = np.array([r[1] for r in res])
    assert (loads[t0] != G.NULL_FRAME).any(), "the disconnect must roll sessions back"
    # the truth run still receives the other remote (handle 1) late: compare only
    # after both runs have confirmed everything they saved
    truth = O.OracleP2P(ORC_GAME[game], P, W, 1, mask, S, sparse_saving=sparse, remote_delay=1)
    drive_oracle(truth, mask, inputs, full_h, rin, T, disc={t0: [(h, None)]})
    np.testing.assert_array_equal(lag.read_live()[0], truth.read_live()[0])
    a, b = lag.read_cells(), truth.read_cells()
    if not sparse:  # sparse saving picks its cells by the confirmed frame, which depends on delivery timing
        np.testing.assert_array_equal(a[0], b[0])
    same = (a[0] == b[0]) & (a[0] >= 0)
    assert same.sum() >= S
    for x, y in zip(a[1:], b[1:]):
        np.testing.assert_array_equal(x[same], y[same])


# ---------------------------------------------------------------------------- device vs oracle
def gpu_pair(game, S, P, W, d, rd, mask, sparse, lane_per_session=False, fanout=False, candidates=16,
             per_player=False):
    b = (G.SessionBuilder(game, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
         .with_input_delay(d).with_sparse_saving_mode(sparse).with_remote_input_delay(rd)
         .with_lane_per_session(lane_per_session).with_speculative_fanout(fanout, candidates, per_player=per_player))
    for h in range(P):
        b.add_player(PlayerType.Local if (mask >> h) & 1 else PlayerType.Remote, h)
    sess = b.start_p2p_session()
    orc = O.OracleP2P(ORC_GAME[game], P, W, d, mask, S, sparse_saving=sparse, remote_delay=rd)
    return sess, orc


def compare_state(sess, orc, tick, alive=None):
    """Cells, live state and frames of the device batch == the oracle's
    (sessions where `alive` is true; a panicked session is dead)."""
    tags, imgs, cs = sess.read_cells()
    otags, oimgs, ocs = orc.read_cells()
    a = np.ones(tags.shape[1], bool) if alive is None else alive
    np.testing.assert_array_equal(tags[:, a], otags[:, a], err_msg=f"cell frames, tick {tick}")
    valid = (otags >= 0) & a[None, :]
    np.testing.assert_array_equal(imgs[valid], oimgs[valid], err_msg=f"cell images, tick {tick}")
    np.testing.assert_array_equal(cs[valid], ocs[valid], err_msg=f"cell checksums, tick {tick}")
    np.testing.assert_array_equal(sess.read_live()[a], orc.read_live()[0][a], err_msg=f"live state, tick {tick}")
    c, k = sess.frames()
    oc, ok = orc.frames()
    np.testing.assert_array_equal(c[a], oc[a])
    np.testing.assert_array_equal(k[a], ok[a])
    compare_queues(sess, orc, tick, a)


def compare_queues(sess, orc, tick, alive):
    """Every InputQueue's bookkeeping (last added / tail / length / last requested / prediction /
    first incorrect frame) and ConnectionStatus == the oracle's."""
    dq, oq = sess.read_queues(), orc.queues()
    # inputs[tail].frame before a queue's first add: NULL in the reference, 0 on the device (the
    # frame its first add puts there); nothing reads it before then
    dq[:, :, 1] = np.where(dq[:, :, 0] < 0, oq[:, :, 1], dq[:, :, 1])
    np.testing.assert_array_equal(dq[alive], oq[alive], err_msg=f"input queues, tick {tick}")


CASES = [  # game, P, W, d, rd, local_mask, sparse, lag range
    (G.Game.EX_GAME, 2, 8, 0, 0, 0b01, False, (1, 4)),
    (G.Game.EX_GAME, 2, 8, 2, 2, 0b01, False, (0, 6)),
    (G.Game.EX_GAME, 2, 8, 2, 1, 0b10, True, (1, 5)),
    (G.Game.EX_GAME, 4, 8, 1, 1, 0b0001, False, (1, 5)),
    (G.Game.EX_GAME, 3, 7, 0, 2, 0b010, True, (0, 4)),
    (G.Game.STUB, 2, 8, 1, 0, 0b01, False, (1, 5)),
    (G.Game.STUB, 2, 6, 0, 1, 0b10, True, (1, 4)),
    (G.Game.EX_GAME, 2, 4, 0, 0, 0b01, False, (1, 6)),  # lags past the window: PredictionThreshold
    # stubs_enum.rs: the game compares (input, InputStatus) tuples, so Predicted vs Confirmed matters
    (G.Game.STUB_ENUM, 2, 8, 1, 1, 0b01, False, (1, 4)),
    (G.Game.STUB_ENUM, 2, 6, 0, 2, 0b10, True, (0, 5)),
    # W > 8: the snapshot ring stays in HBM (the LDS ring holds at most 8 cells)
    (G.Game.EX_GAME, 2, 12, 1, 1, 0b01, False, (1, 9)),
    # the brawler: one wave per session, 8 KiB cells (too big for the LDS ring: HBM cells)
    (G.Game.BRAWLER, 2, 8, 1, 1, 0b01, False, (1, 4)),
    (G.Game.BRAWLER, 2, 6, 0, 2, 0b10, True, (0, 5)),
    (G.Game.EX_GAME, 3, 10, 0, 2, 0b001, True, (1, 7)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0].name}-P{c[1]}-W{c[2]}-d{c[3]}-rd{c[4]}-m{c[5]}-sp{int(c[6])}"
                                             for c in CASES])
def test_gpu_p2p_matches_oracle_every_tick(gpu_available, case):
    import torch
    game, P, W, d, rd, mask, sparse, (lo, hi) = case
    S, T = 70, 90
    dt = np.uint32 if game == G.Game.STUB else np.uint8
    imask = {G.Game.STUB: 0x3, G.Game.STUB_ENUM: 0x1}.get(game, 0x0F)
    inputs, upto, rin = synth_network(S, P, T, mask, rd, lo, hi, dtype=dt, mask=imask)
    sess, orc = gpu_pair(game, S, P, W, d, rd, mask, sparse)
    di = torch.from_numpy(inputs).cuda()
    du = torch.from_numpy(upto).cuda()
    dr = torch.from_numpy(rin).cuda()
    saw_rollback = saw_threshold = False
    for t in range(T):
        sess.run_ticks(di[t:t + 1], du[t:t + 1], dr)
        ost, olf, ona, ons = drive_oracle(orc, mask, inputs, upto, rin, t + 1, t0=t)[0]
        st, lf, na, ns = sess.status()
        np.testing.assert_array_equal(st, ost, err_msg=f"status, tick {t}")
        np.testing.assert_array_equal(lf, olf, err_msg=f"LoadGameState frame, tick {t}")
        np.testing.assert_array_equal(na, ona, err_msg=f"AdvanceFrame count, tick {t}")
        np.testing.assert_array_equal(ns, ons, err_msg=f"SaveGameState count, tick {t}")
        saw_rollback |= bool((lf != G.NULL_FRAME).any())
        saw_threshold |= bool((st == 1).any())
        if t % 10 == 9 or t == T - 1:
            compare_state(sess, orc, t)
    assert saw_rollback
    if W == 4:
        assert saw_threshold
    assert sess.counters()[2] == 0


@pytest.mark.gpu
def test_gpu_p2p_fused_launch_equals_per_tick(gpu_available):
    # One launch of T ticks == T launches of one tick (state in registers across ticks).
    import torch
    game, P, W, d, rd, mask = G.Game.EX_GAME, 2, 8, 2, 1, 0b01
    S, T = 200, 64
    inputs, upto, rin = synth_network(S, P, T, mask, rd, 1, 5)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    a, _ = gpu_pair(game, S, P, W, d, rd, mask, False)
    b, orc = gpu_pair(game, S, P, W, d, rd, mask, False)
    for t in range(T):
        a.run_ticks(di[t:t + 1], du[t:t + 1], dr)
    b.run_ticks(di[:T // 2], du[:T // 2], dr)
    b.run_ticks(di[T // 2:], du[T // 2:], dr)
    drive_oracle(orc, mask, inputs, upto, rin, T)
    np.testing.assert_array_equal(a.read_live(), b.read_live())
    compare_state(b, orc, T - 1)
    for x, y in zip(a.read_cells(), b.read_cells()):
        np.testing.assert_array_equal(x, y)


FUSED_CASES = [  # game, P, W, d, rd, local_mask, lag range, ticks per launch, sparse saving
    (G.Game.EX_GAME, 2, 8, 2, 2, 0b01, (0, 6), 16, False),
    (G.Game.EX_GAME, 4, 8, 1, 1, 0b0001, (1, 5), 24, False),
    (G.Game.EX_GAME, 3, 7, 0, 2, 0b010, (0, 4), 32, False),
    (G.Game.EX_GAME, 2, 4, 0, 0, 0b01, (1, 6), 12, False),  # PredictionThreshold ticks inside the launches
    # sparse saving on the lane-asynchronous kernel (launches of >= 24 ticks): check_last_saved_state's
    # second rollback inside the launch, PredictionThreshold from the dry run
    (G.Game.EX_GAME, 2, 8, 2, 1, 0b10, (1, 5), 32, True),
    (G.Game.EX_GAME, 3, 7, 0, 2, 0b010, (0, 4), 48, True),
    (G.Game.EX_GAME, 2, 4, 0, 0, 0b01, (1, 6), 24, True),
    # launches of 4-23 ticks: HBM cells, the input ring in LDS (p2p.hpp kLdsQMinTicks)
    (G.Game.EX_GAME, 2, 8, 2, 1, 0b10, (1, 5), 8, True),
    (G.Game.EX_GAME, 3, 7, 0, 2, 0b010, (0, 4), 5, False),
    (G.Game.BRAWLER, 2, 8, 2, 2, 0b01, (1, 4), 10, False),  # the brawler: HBM cells, LDS input ring
]


@pytest.mark.gpu
@pytest.mark.parametrize("sync_ticks", [False, True], ids=["async", "lockstep"])
@pytest.mark.parametrize("case", FUSED_CASES, ids=[f"P{c[1]}-W{c[2]}-d{c[3]}-rd{c[4]}-m{c[5]}-tpl{c[7]}-sp{int(c[8])}"
                                                   for c in FUSED_CASES])
def test_gpu_p2p_fused_launches_match_oracle(gpu_available, monkeypatch, case, sync_ticks):
    # Multi-tick launches with sessions of different lags, so that inside a launch
    # sessions sit at different ticks (p2p.hpp kAsync: one AdvanceFrame per session
    # per iteration) — and the lock-step kernel (RB_P2P_SYNC_TICKS=1): after every
    # launch the last tick's request counts and every cell, state and queue equal
    # the oracle's.
    import torch
    monkeypatch.setenv("RB_P2P_SYNC_TICKS", "1" if sync_ticks else "0")
    game, P, W, d, rd, mask, (lo, hi), tpl, sparse = case
    S, T = 300, 96
    inputs, upto, rin = synth_network(S, P, T, mask, rd, lo, hi)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    sess, orc = gpu_pair(game, S, P, W, d, rd, mask, sparse)
    for t0 in range(0, T, tpl):
        t1 = min(T, t0 + tpl)
        sess.run_ticks(di[t0:t1], du[t0:t1], dr)
        ost, olf, ona, ons = drive_oracle(orc, mask, inputs, upto, rin, t1, t0=t0)[-1]
        st, lf, na, ns = sess.status()
        np.testing.assert_array_equal(st, ost, err_msg=f"status, tick {t1 - 1}")
        np.testing.assert_array_equal(lf, olf, err_msg=f"LoadGameState frame, tick {t1 - 1}")
        np.testing.assert_array_equal(na, ona, err_msg=f"AdvanceFrame count, tick {t1 - 1}")
        np.testing.assert_array_equal(ns, ons, err_msg=f"SaveGameState count, tick {t1 - 1}")
        compare_state(sess, orc, t1 - 1)
    assert sess.counters()[2] == 0
    assert sess.totals()[2] > 0  # rollbacks (LoadGameStates) executed inside the fused launches


FANOUT_CASES = [  # P, W, d, rd, local_mask, lag range (BASELINE config 4 = P 4, W 8)
    (4, 8, 1, 1, 0b0001, (1, 5)),
    (2, 8, 2, 2, 0b01, (0, 6)),
    (3, 7, 0, 0, 0b010, (1, 4)),
    (4, 4, 0, 0, 0b0001, (1, 6)),  # PredictionThreshold hits too
]


@pytest.mark.gpu
@pytest.mark.parametrize("generic", [False, True], ids=["indep", "generic"])
@pytest.mark.parametrize("case", FANOUT_CASES, ids=[f"P{c[0]}-W{c[1]}-d{c[2]}-rd{c[3]}-m{c[4]}" for c in FANOUT_CASES])
def test_gpu_speculative_fanout_matches_rollback(gpu_available, monkeypatch, case, generic):
    # With the fan-out, matching mispredictions are served by a branch select:
    # statuses, logical request counts, cells and states must stay identical to
    # the reference's rollback (the oracle) on every tick, and selects must
    # actually happen.  ex_game's players move independently, so p2p_kernel
    # runs the fan-out itself (p2p.hpp inlane_fan: the speculated player's
    # branches only); RB_FANOUT_GENERIC=1 makes the batch run the generic
    # fanout_kernel (16 branches x every player) as a launch of its own instead.
    import torch
    monkeypatch.setenv("RB_FANOUT_GENERIC", "1" if generic else "0")
    P, W, d, rd, mask, (lo, hi) = case
    S, T = 96, 80
    inputs, upto, rin = synth_network(S, P, T, mask, rd, lo, hi)
    sess, orc = gpu_pair(G.Game.EX_GAME, S, P, W, d, rd, mask, False, fanout=True)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    for t in range(T):
        sess.run_ticks(di[t:t + 1], du[t:t + 1], dr)
        ost, olf, ona, ons = drive_oracle(orc, mask, inputs, upto, rin, t + 1, t0=t)[0]
        st, lf, na, ns = sess.status()
        np.testing.assert_array_equal(st, ost, err_msg=f"status, tick {t}")
        np.testing.assert_array_equal(lf, olf, err_msg=f"rollback frame, tick {t}")
        np.testing.assert_array_equal(na, ona, err_msg=f"AdvanceFrame count, tick {t}")
        np.testing.assert_array_equal(ns, ons, err_msg=f"SaveGameState count, tick {t}")
        if t % 8 == 7 or t == T - 1:
            compare_state(sess, orc, t)
    adv, saves, loads, selects, branch_frames = sess.totals()
    assert selects > 0, "no misprediction was served by a branch select"
    assert branch_frames > 0
    # no panic, and no lane (the padding lane of P = 3 included) ever took the
    # out-of-range math path: a selected branch never hands a lane garbage
    assert sess.counters()[2] == 0 and sess.counters()[1] == 0


FANOUT_K_CASES = [  # game, P, W, d, rd, local_mask, lag, K, input mask
    (G.Game.EX_GAME, 4, 8, 1, 1, 0b0001, (1, 5), 6, 0x0F),   # K < the 16-value alphabet: the most likely 6
    (G.Game.EX_GAME, 2, 8, 2, 2, 0b01, (0, 6), 2, 0x0F),     # K = 2: the prediction and the input before it
    (G.Game.BRAWLER, 2, 8, 1, 1, 0b01, (1, 5), 16, 0x07),    # the brawler: a wave per branch, 8-bit inputs
    (G.Game.BRAWLER, 3, 6, 0, 1, 0b010, (1, 4), 8, 0x1F),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", FANOUT_K_CASES, ids=[f"{c[0].name}-P{c[1]}-K{c[7]}-m{c[8]:x}" for c in FANOUT_K_CASES])
def test_gpu_fanout_top_k_candidates_match_rollback(gpu_available, case):
    # The fan-out with K most-likely candidates (include/ggrs_amd.h RB_P2P_FLAG_FANOUT): every
    # select must stay observably identical to the reference's rollback (the oracle) on every tick,
    # for ex_game with K below its alphabet and for the brawler (one wave per branch, 8-bit inputs,
    # candidates = the most recently confirmed distinct inputs).
    import torch
    game, P, W, d, rd, mask, (lo, hi), K, imask = case
    S, T = (48, 60) if game == G.Game.BRAWLER else (96, 80)
    inputs, upto, rin = synth_network(S, P, T, mask, rd, lo, hi, mask=imask)
    sess, orc = gpu_pair(game, S, P, W, d, rd, mask, False, fanout=True, candidates=K)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    for t in range(T):
        sess.run_ticks(di[t:t + 1], du[t:t + 1], dr)
        ost, olf, ona, ons = drive_oracle(orc, mask, inputs, upto, rin, t + 1, t0=t)[0]
        st, lf, na, ns = sess.status()
        np.testing.assert_array_equal(st, ost, err_msg=f"status, tick {t}")
        np.testing.assert_array_equal(lf, olf, err_msg=f"rollback frame, tick {t}")
        np.testing.assert_array_equal(na, ona, err_msg=f"AdvanceFrame count, tick {t}")
        np.testing.assert_array_equal(ns, ons, err_msg=f"SaveGameState count, tick {t}")
        if t % 10 == 9 or t == T - 1:
            compare_state(sess, orc, t)
    adv, saves, loads, selects, branch_frames = sess.totals()
    assert selects > 0, "no misprediction was served by a branch select"
    assert branch_frames > 0
    assert sess.counters()[2] == 0 and sess.counters()[1] == 0


FANOUT_FUSED_CASES = [  # P, W, d, rd, local_mask, lag range, K, ticks per launch
    (4, 8, 1, 1, 0b0001, (1, 5), 16, 24),  # config 4's shape; >= 24 ticks: the LDS snapshot ring
    (4, 8, 1, 1, 0b0001, (1, 5), 6, 7),    # K < 16 (recently confirmed values), HBM cells
    (2, 8, 2, 2, 0b01, (0, 6), 16, 32),    # 8 branches per lane
    (3, 7, 0, 0, 0b010, (1, 4), 16, 30),   # the padding lane of a 4-lane group runs branches too
    (4, 4, 0, 0, 0b0001, (1, 6), 16, 24),  # PredictionThreshold ticks inside the launches
    (3, 8, 1, 1, 0b001, (1, 5), 5, 40),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", FANOUT_FUSED_CASES, ids=[f"P{c[0]}-W{c[1]}-K{c[6]}-tpl{c[7]}" for c in FANOUT_FUSED_CASES])
def test_gpu_fanout_fused_launches_match_oracle(gpu_available, case):
    # The in-kernel fan-out lets one launch hold many ticks (p2p.hpp inlane_fan): the fan-out of
    # tick t and the select of tick t + 1 run inside the same launch, across launch boundaries
    # through spec_meta.  After every launch the last tick's request counts and every cell,
    # state and queue equal the reference's rollback (the oracle), and selects happen.
    import torch
    P, W, d, rd, mask, (lo, hi), K, tpl = case
    S, T = 150, 96
    inputs, upto, rin = synth_network(S, P, T, mask, rd, lo, hi)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    sess, orc = gpu_pair(G.Game.EX_GAME, S, P, W, d, rd, mask, False, fanout=True, candidates=K)
    for t0 in range(0, T, tpl):
        t1 = min(T, t0 + tpl)
        sess.run_ticks(di[t0:t1], du[t0:t1], dr)
        ost, olf, ona, ons = drive_oracle(orc, mask, inputs, upto, rin, t1, t0=t0)[-1]
        st, lf, na, ns = sess.status()
        np.testing.assert_array_equal(st, ost, err_msg=f"status, tick {t1 - 1}")
        np.testing.assert_array_equal(lf, olf, err_msg=f"rollback frame, tick {t1 - 1}")
        np.testing.assert_array_equal(na, ona, err_msg=f"AdvanceFrame count, tick {t1 - 1}")
        np.testing.assert_array_equal(ns, ons, err_msg=f"SaveGameState count, tick {t1 - 1}")
        compare_state(sess, orc, t1 - 1)
    adv, saves, loads, selects, branch_frames = sess.totals()
    assert selects > 0, "no misprediction was served by a branch select"
    assert branch_frames > 0
    assert sess.counters()[2] == 0 and sess.counters()[1] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("tpl", [1, 24], ids=["tick", "fused"])
@pytest.mark.parametrize("case", FANOUT_CASES, ids=[f"P{c[0]}-W{c[1]}-d{c[2]}-rd{c[3]}-m{c[4]}" for c in FANOUT_CASES])
def test_gpu_per_player_fanout_matches_rollback(gpu_available, case, tpl):
    # Per-player speculation (RB_P2P_FLAG_FANOUT_PER_PLAYER): every remote player's input classes are
    # presimulated from the oldest first unconfirmed frame, so rollbacks in which several players
    # mispredicted become selects too.  One-tick launches (HBM cells) and 24-tick launches (the LDS
    # snapshot ring): statuses, request counts, cells, states and queues equal the reference's
    # rollback (the oracle) after every launch, and more rollbacks become selects than with the
    # one-player fan-out on the same inputs.
    import torch
    P, W, d, rd, mask, (lo, hi) = case
    S, T = 96, 96
    inputs, upto, rin = synth_network(S, P, T, mask, rd, lo, hi)
    sess, orc = gpu_pair(G.Game.EX_GAME, S, P, W, d, rd, mask, False, fanout=True, per_player=True)
    one, _ = gpu_pair(G.Game.EX_GAME, S, P, W, d, rd, mask, False, fanout=True)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    for t0 in range(0, T, tpl):
        t1 = min(T, t0 + tpl)
        sess.run_ticks(di[t0:t1], du[t0:t1], dr)
        one.run_ticks(di[t0:t1], du[t0:t1], dr)
        ost, olf, ona, ons = drive_oracle(orc, mask, inputs, upto, rin, t1, t0=t0)[-1]
        st, lf, na, ns = sess.status()
        np.testing.assert_array_equal(st, ost, err_msg=f"status, tick {t1 - 1}")
        np.testing.assert_array_equal(lf, olf, err_msg=f"rollback frame, tick {t1 - 1}")
        np.testing.assert_array_equal(na, ona, err_msg=f"AdvanceFrame count, tick {t1 - 1}")
        np.testing.assert_array_equal(ns, ons, err_msg=f"SaveGameState count, tick {t1 - 1}")
        if tpl > 1 or t1 % 8 == 0 or t1 == T:
            compare_state(sess, orc, t1 - 1)
    adv, saves, loads, selects, branch_frames = sess.totals()
    assert selects > 0 and branch_frames > 0
    assert sess.counters()[2] == 0 and sess.counters()[1] == 0
    if P > 2:  # several remote players: the per-player form selects where the one-player form cannot
        assert selects > one.totals()[3], (selects, one.totals()[3])
    assert loads + selects == one.totals()[2] + one.totals()[3]


@pytest.mark.gpu
def test_gpu_per_player_fanout_needs_the_whole_alphabet(gpu_available):
    with pytest.raises(G.InvalidRequest):  # K = 8 < ex_game's 16 inputs: candidates from a list
        gpu_pair(G.Game.EX_GAME, 64, 4, 8, 1, 1, 0b0001, False, fanout=True, candidates=8, per_player=True)
    with pytest.raises(G.InvalidRequest):  # the brawler's players interact
        gpu_pair(G.Game.BRAWLER, 64, 2, 8, 1, 1, 0b01, False, fanout=True, per_player=True)


@pytest.mark.gpu
def test_gpu_speculative_fanout_state_after_many_ticks(gpu_available):
    # Long run, fused call of many ticks: final cells and state equal the plain P2P batch.
    import torch
    P, W, d, rd, mask = 4, 8, 1, 1, 0b0001
    S, T = 256, 160
    inputs, upto, rin = synth_network(S, P, T, mask, rd, 1, 5)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    spec, _ = gpu_pair(G.Game.EX_GAME, S, P, W, d, rd, mask, False, fanout=True)
    plain, _ = gpu_pair(G.Game.EX_GAME, S, P, W, d, rd, mask, False)
    spec.run_ticks(di, du, dr)
    plain.run_ticks(di, du, dr)
    np.testing.assert_array_equal(spec.read_live(), plain.read_live())
    for x, y in zip(spec.read_cells(), plain.read_cells()):
        np.testing.assert_array_equal(x, y)
    ts, tp = spec.totals(), plain.totals()
    assert ts[3] > 0 and ts[2] + ts[3] == tp[2], (ts, tp)  # every rollback is a load or a select


DISC_CASES = [  # game, P, W, d, rd, local_mask, sparse, fanout, lag range
    (G.Game.EX_GAME, 2, 8, 2, 1, 0b01, False, False, (1, 5)),
    (G.Game.EX_GAME, 3, 7, 0, 2, 0b010, True, False, (0, 4)),
    (G.Game.EX_GAME, 4, 8, 1, 1, 0b0001, False, True, (1, 5)),
    (G.Game.STUB, 2, 8, 1, 0, 0b10, False, False, (1, 5)),
    (G.Game.EX_GAME, 2, 4, 0, 0, 0b01, False, False, (1, 6)),  # PredictionThreshold around the disconnect
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", DISC_CASES, ids=[f"{c[0].name}-P{c[1]}-W{c[2]}-m{c[5]}-sp{int(c[6])}-fo{int(c[7])}"
                                                  for c in DISC_CASES])
def test_gpu_p2p_disconnect_matches_oracle_every_tick(gpu_available, case):
    # disconnect_player between ticks, for half of the sessions at one tick and
    # the rest later: statuses, request counts, cells and states equal the
    # oracle's on every tick; the batch raises InvalidRequest like the reference.
    import torch
    game, P, W, d, rd, mask, sparse, fanout, (lo, hi) = case
    S, T = 70, 80
    dt = np.uint32 if game == G.Game.STUB else np.uint8
    inputs, upto, rin = synth_network(S, P, T, mask, rd, lo, hi, dtype=dt, mask=0x3 if game == G.Game.STUB else 0x0F)
    sess, orc = gpu_pair(game, S, P, W, d, rd, mask, sparse, fanout=fanout)
    remotes = [h for h in range(P) if not (mask >> h) & 1]
    local = [h for h in range(P) if (mask >> h) & 1][0]
    h = remotes[-1]
    half = np.arange(S) % 2 == 0
    disc = {30: [(h, half)], 47: [(h, ~half)]}
    if len(remotes) > 1:
        disc[55] = [(remotes[0], np.arange(S) % 3 == 0)]
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    saw_rollback_at_disconnect = False
    # A disconnect whose last frame is current_frame - 1 sets disconnect_frame =
    # current_frame, and the reference's load_frame asserts (sync_layer.rs:141-145);
    # so does loading a cell whose SaveGameState was dropped with a
    # PredictionThreshold error (:148).  Both implementations panic on exactly
    # those sessions; after that a session is dead and no longer compared.
    alive = np.ones(S, bool)
    for t in range(T):
        for hh, m in disc.get(t, []):
            sess.disconnect_player(hh, m)
        ost, olf, ona, ons = drive_oracle(orc, mask, inputs, upto, rin, t + 1, t0=t, disc=disc)[0]
        sess.run_ticks(di[t:t + 1], du[t:t + 1], dr)
        st, lf, na, ns = sess.status()
        st = np.where(st == RB_PANIC, O.KIND_PANIC, st)
        np.testing.assert_array_equal(st[alive], ost[alive], err_msg=f"status, tick {t}")
        alive &= ost != O.KIND_PANIC
        np.testing.assert_array_equal(lf[alive], olf[alive], err_msg=f"LoadGameState frame, tick {t}")
        np.testing.assert_array_equal(na[alive], ona[alive], err_msg=f"AdvanceFrame count, tick {t}")
        np.testing.assert_array_equal(ns[alive], ons[alive], err_msg=f"SaveGameState count, tick {t}")
        if t in disc:
            saw_rollback_at_disconnect |= bool((lf[alive] != G.NULL_FRAME).any())
        if t % 10 == 9 or t in disc or t == T - 1:
            compare_state(sess, orc, t, alive)
    assert saw_rollback_at_disconnect
    assert alive.sum() >= S // 4
    if W >= 8:
        assert alive.all() and sess.counters()[2] == 0
    with pytest.raises(G.InvalidRequest, match="already disconnected"):
        sess.disconnect_player(h, half)
    with pytest.raises(G.InvalidRequest, match="Local Player"):
        sess.disconnect_player(local)
    with pytest.raises(G.InvalidRequest, match="Invalid Player Handle"):
        sess.disconnect_player(P)


@pytest.mark.gpu
@pytest.mark.parametrize("sync_ticks", [False, True], ids=["async", "lockstep"])
@pytest.mark.parametrize("P,mask", [(2, 0b01), (4, 0b0001)])
def test_gpu_p2p_disconnects_between_fused_launches(gpu_available, monkeypatch, P, mask, sync_ticks):
    # disconnect_player between multi-tick launches (the disconnect's rollback and
    # the (zeroed, Disconnected) inputs then run inside fused launches where the
    # sessions sit at different ticks, p2p.hpp kAsync): after every launch the last
    # tick's request counts and every cell, state and queue equal the oracle's.
    import torch
    monkeypatch.setenv("RB_P2P_SYNC_TICKS", "1" if sync_ticks else "0")
    W, d, rd, (lo, hi) = 8, 1, 1, (1, 5)
    S, T, tpl = 150, 80, 26  # launches of >= 24 ticks run the lane-asynchronous kernel, shorter ones lock-step
    inputs, upto, rin = synth_network(S, P, T, mask, rd, lo, hi)
    sess, orc = gpu_pair(G.Game.EX_GAME, S, P, W, d, rd, mask, False)
    remotes = [h for h in range(P) if not (mask >> h) & 1]
    half = np.arange(S) % 2 == 0
    disc = {30: [(remotes[-1], half)], 47: [(remotes[-1], ~half)]}
    if len(remotes) > 1:
        disc[55] = [(remotes[0], np.arange(S) % 3 == 0)]
    cuts = sorted(set(list(range(0, T, tpl)) + list(disc) + [T]))
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    for t0, t1 in zip(cuts[:-1], cuts[1:]):
        for hh, m in disc.get(t0, []):
            sess.disconnect_player(hh, m)
        ost, olf, ona, ons = drive_oracle(orc, mask, inputs, upto, rin, t1, t0=t0, disc=disc)[-1]
        sess.run_ticks(di[t0:t1], du[t0:t1], dr)
        st, lf, na, ns = sess.status()
        np.testing.assert_array_equal(st, ost, err_msg=f"status, tick {t1 - 1}")
        np.testing.assert_array_equal(lf, olf, err_msg=f"LoadGameState frame, tick {t1 - 1}")
        np.testing.assert_array_equal(na, ona, err_msg=f"AdvanceFrame count, tick {t1 - 1}")
        np.testing.assert_array_equal(ns, ons, err_msg=f"SaveGameState count, tick {t1 - 1}")
        compare_state(sess, orc, t1 - 1)
    assert sess.counters()[2] == 0


@pytest.mark.gpu
def test_gpu_p2p_long_disconnect_takes_the_absolute_rows(gpu_available):
    """The bookkeeping rows hold frames as 16-bit deltas from the current frame (p2p.hpp q_pack).  A
    player disconnected for more than 32,767 frames keeps its last added, connection and tail frames,
    so its rows take the escape bit and the absolute rows.  Statuses, request counts, queues, cells and
    states equal the oracle's before and after the crossing, through fused lane-asynchronous, kQ and
    one-tick launches."""
    import torch
    P, W, d, rd, mask = 2, 8, 1, 1, 0b01
    S, T = 70, 32900
    inputs, upto, rin = synth_network(S, P, T, mask, rd, 1, 5)
    sess, orc = gpu_pair(G.Game.EX_GAME, S, P, W, d, rd, mask, False)
    half = np.arange(S) % 2 == 0
    disc = {30: half, 40: ~half}
    r1 = np.ascontiguousarray(rin[:64, 1, :])  # the remote frames delivered before the disconnects
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    cuts = [0, 30] + list(range(31, 42)) + list(range(100, 32750, 50)) + list(range(32750, 32830)) + \
        list(range(32830, 32878, 8)) + [T]  # one-tick launches across the crossing (cur - 32,767 ~ 32,800)
    ot = 0
    for t0, t1 in zip(cuts[:-1], cuts[1:]):
        if t0 in disc:
            sess.disconnect_player(1, disc[t0])
            assert orc.disconnect_player(1, disc[t0]) == 0
        sess.run_ticks(di[t0:t1], du[t0:t1], dr)
        for t in range(ot, t1):
            if t <= 40:  # (a disconnected player's deliveries are ignored, p2p_session.rs:852)
                assert orc.deliver(1, upto[t, 1], r1) == 0
            assert orc.add_local_input(0, inputs[t, 0]) == 0
            res = orc.advance()
        ot = t1
        if t1 in (30, 41, 32750, 32790, 32800, 32810, 32830, T):
            st, lf, na, ns = sess.status()
            for a, b, what in zip((st, lf, na, ns), res, ("status", "LoadGameState frame", "AdvanceFrames", "saves")):
                np.testing.assert_array_equal(a, b, err_msg=f"{what}, tick {t1 - 1}")
            compare_state(sess, orc, t1 - 1)
    assert (sess.frames()[0] - sess.read_queues()[:, 1, 0] > 32767).all()  # every session's player 1 escaped
    assert sess.counters()[2] == 0


@pytest.mark.gpu
def test_gpu_disconnect_at_the_current_frame_asserts_like_reference(gpu_available):
    # The device side of test_oracle_disconnect_at_the_current_frame_asserts_like_reference.
    import torch
    S, P, mask, T = 2, 2, 0b01, 5
    sess, orc = gpu_pair(G.Game.EX_GAME, S, P, 8, 0, 0, mask, False)
    inputs = np.ones((T, P, S), np.uint8)
    upto = np.zeros((T, P, S), np.int32)
    for t in range(T):
        upto[t, 1] = [t, t - 1]
    rin = np.zeros((16, P, S), np.uint8)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    sess.run_ticks(di[:4], du[:4], dr)
    sess.disconnect_player(1)
    sess.run_ticks(di[4:], du[4:], dr)
    st, lf, na, _ = sess.status()
    assert st[0] == RB_PANIC
    assert st[1] == 0 and lf[1] == 3 and na[1] == 2
