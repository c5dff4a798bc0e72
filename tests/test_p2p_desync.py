"""P2P desync detection (row J): ChecksumReports between the two peers of a
session and GGRSEvent::DesyncDetected (p2p_session.rs:873-928,
protocol.rs:27, 710-742), plus the InputQueue length assert
(input_queue.rs:181) and the sticky panic of a batch session.

Peer A holds handle 0 local / handle 1 remote, peer B the reverse, over the
same inputs (synth_network with one seed): A's remote inputs of handle 1 are
B's local inputs and vice versa.  After both peers advanced a tick, each
one's reports are handed to the other (on one node: an all-gather, see
tests/test_distributed.py), which receives them before its next
advance_frame — the order UdpProtocol gives them.

Pinning: the reference's tests hold no desync case; the oracle restates the
four functions line by line and is checked here against the property the
feature exists for (no event while both peers agree on every reported frame,
events on exactly the corrupted sessions once one peer's state is flipped),
the GPU batch against the oracle on every tick.
"""
import numpy as np
import pytest

import ggrs_amd as G
from ggrs_amd._lib import RB_P2P_EVENTS_KEPT, RB_P2P_REPORTS_PER_TAKE, RB_PANIC
from ggrs_amd.p2p import PlayerType, synth_network
from oracle import oracle as O

P, W = 2, 8
MASK_A, MASK_B = 0b01, 0b10
ORC_PANIC = 99


def networks(S, T, d, lag, seed=0x67677273):
    """(inputs, (upto, remote_in) of A, (upto, remote_in) of B); both peers use input delay d."""
    ia, ua, ra = synth_network(S, P, T, MASK_A, d, lag[0], lag[1], seed=seed)
    ib, ub, rb = synth_network(S, P, T, MASK_B, d, lag[0], lag[1], seed=seed)
    assert np.array_equal(ia, ib)
    return ia, (ua, ra), (ub, rb)


def oracle_peer(mask, S, d, interval, sparse=False, game=O.EX_GAME):
    orc = O.OracleP2P(game, P, W, d, mask, S, sparse_saving=sparse, remote_delay=d)
    orc.set_desync_detection(interval)
    return orc


def oracle_tick(orc, mask, inputs, net, t):
    upto, rin = net
    for h in range(P):
        if not (mask >> h) & 1:
            orc.deliver(h, upto[t, h], rin[:, h, :])
    for h in range(P):
        if (mask >> h) & 1:
            orc.add_local_input(h, inputs[t, h])
    return orc.advance()


def exchange_oracle(a, b):
    fa, ca = a.take_checksum_reports(RB_P2P_REPORTS_PER_TAKE)
    fb, cb = b.take_checksum_reports(RB_P2P_REPORTS_PER_TAKE)
    a.receive_checksum_reports(1, fb, cb)
    b.receive_checksum_reports(0, fa, ca)
    return (fa, ca), (fb, cb)


# ---------------------------------------------------------------------------- oracle (CPU)
def test_oracle_peers_report_every_interval_and_agree():
    S, T, d, interval = 48, 120, 2, 10
    inputs, na, nb = networks(S, T, d, (0, 1))
    a, b = oracle_peer(MASK_A, S, d, interval), oracle_peer(MASK_B, S, d, interval)
    for t in range(T):
        assert (oracle_tick(a, MASK_A, inputs, na, t)[0] == 0).all()
        assert (oracle_tick(b, MASK_B, inputs, nb, t)[0] == 0).all()
        (fa, ca), (fb, cb) = exchange_oracle(a, b)
        # check_checksum_send_interval: at current % interval == 0, frame = last_saved - 1 = current - 1,
        # only once that frame is past max_prediction
        want = t - 1 if t % interval == 0 and t - 1 > W else -1
        assert (fa[0] == want).all() and (fb[0] == want).all() and (fa[1:] == -1).all()
        if want >= 0:  # with lag <= 1 every reported frame is confirmed at both peers: the same checksum
            np.testing.assert_array_equal(ca[0], cb[0])
    for orc in (a, b):
        n, *_ = orc.desync_events()
        assert (n == 0).all()


def test_oracle_corrupted_sessions_raise_desync_detected():
    S, T, d, interval = 48, 110, 2, 10
    inputs, na, nb = networks(S, T, d, (0, 1))
    a, b = oracle_peer(MASK_A, S, d, interval), oracle_peer(MASK_B, S, d, interval)
    bad = [5, 17, 40]
    for t in range(T):
        if t == 43:
            for s in bad:
                a.corrupt(s, 4 * P, 0x00100000)  # player 0's rotation (canonical word 4P): the offset persists
        oracle_tick(a, MASK_A, inputs, na, t)
        oracle_tick(b, MASK_B, inputs, nb, t)
        exchange_oracle(a, b)
    for orc, handle in ((a, 1), (b, 0)):
        n, fr, hd, lo, ro = orc.desync_events()
        assert sorted(np.nonzero(n)[0].tolist()) == bad
        for s in bad:
            k = int(min(n[s], RB_P2P_EVENTS_KEPT))
            ev = fr[s, -k:] if n[s] >= RB_P2P_EVENTS_KEPT else fr[s, :k]
            assert (ev >= 49).all() and ((ev + 1) % interval == 0).all()  # reports after the flip
            assert (hd[s, :k] == handle).all() and (lo[s, :k] != ro[s, :k]).all()


# ---------------------------------------------------------------------------- device vs oracle
def gpu_peer(mask, S, d, interval, sparse=False, game=G.Game.EX_GAME):
    b = (G.SessionBuilder(game, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
         .with_input_delay(d).with_remote_input_delay(d).with_sparse_saving_mode(sparse)
         .with_desync_detection_mode(interval))
    for h in range(P):
        b.add_player(PlayerType.Local if (mask >> h) & 1 else PlayerType.Remote, h)
    return b.start_p2p_session()


def dev_reports_as_oracle(rep):
    r = rep.cpu().numpy()
    frames = (r[..., 2] & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    cs = np.stack([r[..., 0].view(np.uint64), r[..., 1].view(np.uint64)], -1)
    return frames, cs


DESYNC_CASES = [  # input delay, lag range, interval, sparse, corrupt tick
    (2, (0, 1), 10, False, 43),
    (2, (1, 4), 5, False, 30),   # lag past 1: predicted frames get reported (the reference's false positives)
    (0, (0, 2), 1, False, 20),   # a report every frame: both histories hit their 32-entry retention
    (1, (1, 3), 4, True, 25),    # sparse saving: frame last_saved - 1 often has no cell -> the reference panics
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", DESYNC_CASES, ids=[f"d{c[0]}-lag{c[1][0]}{c[1][1]}-i{c[2]}-sp{int(c[3])}"
                                                    for c in DESYNC_CASES])
def test_gpu_desync_detection_matches_oracle_every_tick(gpu_available, case):
    import torch
    d, lag, interval, sparse, t_bad = case
    S, T = 96, 90
    inputs, na, nb = networks(S, T, d, lag)
    oa, ob = oracle_peer(MASK_A, S, d, interval, sparse), oracle_peer(MASK_B, S, d, interval, sparse)
    ga, gb = gpu_peer(MASK_A, S, d, interval, sparse), gpu_peer(MASK_B, S, d, interval, sparse)
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    di = dev(inputs)
    ua, ra, ub, rb = dev(na[0]), dev(na[1]), dev(nb[0]), dev(nb[1])
    bad = [3, 50, 95]
    alive = np.ones(S, bool)
    for t in range(T):
        if t == t_bad:
            for s in bad:
                oa.corrupt(s, 4 * P, 0x00100000)  # player 0's rotation: the offset persists
                ga.debug_corrupt(s, 4 * P, 0x00100000)
        ga.run_ticks(di[t:t + 1], ua[t:t + 1], ra)
        gb.run_ticks(di[t:t + 1], ub[t:t + 1], rb)
        for g, o, m, net in ((ga, oa, MASK_A, na), (gb, ob, MASK_B, nb)):
            ost, olf, ona, ons = oracle_tick(o, m, inputs, net, t)
            st, lf, nadv, nsave = g.status()
            np.testing.assert_array_equal(st, np.where(ost == ORC_PANIC, RB_PANIC, ost), err_msg=f"status, tick {t}")
            live = ost != ORC_PANIC
            np.testing.assert_array_equal(lf[live], olf[live], err_msg=f"load frame, tick {t}")
            np.testing.assert_array_equal(nadv[live], ona[live])
            alive &= live
        rep_a, rep_b = ga.take_checksum_reports(), gb.take_checksum_reports()
        (fa, ca), (fb, cb) = exchange_oracle(oa, ob)
        for rep, f, c in ((rep_a, fa, ca), (rep_b, fb, cb)):
            gf, gc = dev_reports_as_oracle(rep)
            np.testing.assert_array_equal(gf[:, alive], f[:, alive], err_msg=f"report frames, tick {t}")
            has = (f >= 0) & alive[None, :]
            np.testing.assert_array_equal(gc[has], c[has], err_msg=f"report checksums, tick {t}")
        ga.receive_checksum_reports(1, rep_b)
        gb.receive_checksum_reports(0, rep_a)
        for g, o in ((ga, oa), (gb, ob)):
            gn, gfr, ghd, glo, gro = g.desync_events()
            on, ofr, ohd, olo, oro = o.desync_events(RB_P2P_EVENTS_KEPT)
            for x, y, what in ((gn, on, "counts"), (gfr, ofr, "frames"), (ghd, ohd, "handles"), (glo, olo, "local"),
                               (gro, oro, "remote")):
                np.testing.assert_array_equal(x[alive], y[alive], err_msg=f"desync events {what}, tick {t}")
    n_a = oa.desync_events()[0]
    if not sparse:
        assert alive.all()
        assert set(np.nonzero(n_a)[0].tolist()) >= set(bad)  # at least the corrupted sessions
        if lag == (0, 1):
            assert sorted(np.nonzero(n_a)[0].tolist()) == bad  # and only them


@pytest.mark.gpu
def test_gpu_input_queue_overflow_panics_and_the_panic_sticks(gpu_available):
    # A remote delivering more than 128 frames past the session's discarded
    # frames trips input_queue.rs:181 (assert!(self.length <= INPUT_QUEUE_LENGTH)).
    # The batch stops exactly those sessions; they report RB_PANIC from then on
    # with frames, cells and state unchanged, the others run on.
    import torch
    S, T, d = 64, 40, 1
    inputs, (upto, rin), _ = networks(S, T, d, (1, 2))
    far = T + 200
    rin = np.concatenate([rin, np.zeros((far - rin.shape[0], P, S), rin.dtype)])
    upto = upto.copy()
    victims = np.zeros(S, bool)
    victims[[2, 9, 33]] = True
    upto[20:, 1, victims] = np.arange(20, T)[:, None] + 150  # 150 frames ahead from tick 20 on
    orc = oracle_peer(MASK_A, S, d, 0)
    g = gpu_peer(MASK_A, S, d, 0)
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    di, du, dr = dev(inputs), dev(upto), dev(rin)
    frozen = None
    for t in range(T):
        g.run_ticks(di[t:t + 1], du[t:t + 1], dr)
        ost = oracle_tick(orc, MASK_A, inputs, (upto, rin), t)[0]
        st = g.status()[0]
        np.testing.assert_array_equal(st, np.where(ost == ORC_PANIC, RB_PANIC, ost), err_msg=f"tick {t}")
        if t < 20:
            assert (st == 0).all()
        else:
            assert (st[victims] == RB_PANIC).all() and (st[~victims] == 0).all()
            snap = (g.frames()[0][victims], g.read_cells()[1][:, victims], g.read_live()[victims])
            if frozen is None:
                frozen = snap
            for x, y in zip(snap, frozen):
                np.testing.assert_array_equal(x, y, err_msg=f"a panicked session changed, tick {t}")
    assert g.counters()[2] == victims.sum()  # each panicked session counted once
    live = ~victims
    np.testing.assert_array_equal(g.read_live()[live], orc.read_live()[0][live])


@pytest.mark.gpu
def test_gpu_queue_overflow_panic_inside_fused_launches(gpu_available):
    # The same overflow, tripped inside launches of 30 ticks (lane-asynchronous
    # ticks, p2p.hpp kAsync): the victims stop at the tick the oracle panics,
    # the other sessions run on and equal the oracle after every launch.
    import torch
    S, T, d, tpl = 64, 60, 1, 30
    inputs, (upto, rin), _ = networks(S, T, d, (1, 2))
    far = T + 200
    rin = np.concatenate([rin, np.zeros((far - rin.shape[0], P, S), rin.dtype)])
    upto = upto.copy()
    victims = np.zeros(S, bool)
    victims[[2, 9, 33]] = True
    upto[20:, 1, victims] = np.arange(20, T)[:, None] + 150
    orc = oracle_peer(MASK_A, S, d, 0)
    g = gpu_peer(MASK_A, S, d, 0)
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    di, du, dr = dev(inputs), dev(upto), dev(rin)
    live = ~victims
    for t0 in range(0, T, tpl):
        g.run_ticks(di[t0:t0 + tpl], du[t0:t0 + tpl], dr)
        for t in range(t0, t0 + tpl):
            ost = oracle_tick(orc, MASK_A, inputs, (upto, rin), t)[0]
        st = g.status()[0]
        np.testing.assert_array_equal(st, np.where(ost == ORC_PANIC, RB_PANIC, ost), err_msg=f"tick {t0 + tpl - 1}")
        assert (st[victims] == RB_PANIC).all() and (st[live] == 0).all()
        np.testing.assert_array_equal(g.frames()[0], orc.frames()[0])
        np.testing.assert_array_equal(g.read_live()[live], orc.read_live()[0][live])
    assert g.counters()[2] == victims.sum()


# ---------------------------------------------------------------------------- RCCL at world size 1
@pytest.mark.gpu
def test_gpu_rccl_world1_report_allgather_and_p2p_exchange(gpu_available):
    # The north-star collective executed on the device with the nccl (= RCCL)
    # backend: SyncTest desync reports (rb_export_checksum_report ->
    # shard.gather_reports, messages.rs:75-79) and the P2P ChecksumReport
    # exchange (rb_p2p_take_checksum_reports -> shard.exchange_checksum_reports
    # -> rb_p2p_receive_checksum_reports, p2p_session.rs:873-928), at world size 1:
    # what comes back is what went in, and the peers fed through the collective
    # raise exactly the oracle's DesyncDetected events.
    import socket

    import torch
    import torch.distributed as dist

    from ggrs_amd import shard
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        # SyncTest reports through the all-gather
        S, T = 300, 20
        inputs = G.synth_inputs(S, P, T)
        sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S, device=0).with_num_players(P)
                .with_check_distance(7).with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
        sess.run_ticks(torch.from_numpy(inputs).to(dev))
        rep = torch.full((S, shard.REPORT_WORDS), 7, dtype=torch.int64, device=dev)
        sess.export_checksum_report(T - 1, rep)
        g = shard.gather_reports(rep)
        assert torch.equal(g, rep)
        orc = O.OracleBatch(O.EX_GAME, P, 8, 7, 2, S)
        for t in range(T):
            for h in range(P):
                orc.add_local_input(h, inputs[t, h])
            orc.advance()
        frames, _, _, cs = orc.read_cells()
        w = int(np.nonzero(frames == T - 1)[0][0])
        r = g.cpu().numpy()
        np.testing.assert_array_equal(r[:, 0].view(np.uint64), cs[w][:, 0])
        assert ((r[:, 2] & 0xFFFFFFFF) == T - 1).all() and ((r[:, 2] >> 32) == -1).all()
        # the compact 4 B report (rb_export_compact_report) through the same collective
        crep = torch.full((S,), 7, dtype=torch.int32, device=dev)
        sess.export_compact_report(T - 1, crep)
        cg = shard.gather_compact(crep)
        assert torch.equal(cg, crep)
        np.testing.assert_array_equal(cg.cpu().numpy(), shard.pack_compact(cs[w][:, 0], T - 1, np.full(S, -1, np.int32)))
        # a corrupted snapshot: the next tick's resimulation mismatches, and the record says so
        sess.debug_corrupt_cell(5, T - 7, 0, 0x100)
        more = G.synth_inputs(S, P, T + 1)[T:T + 1]
        sess.run_ticks(torch.from_numpy(np.ascontiguousarray(more)).to(dev))
        mm = sess.mismatches()
        assert mm[5] != G.NULL_FRAME and (np.delete(mm, 5) == G.NULL_FRAME).all()
        sess.export_compact_report(T, crep)
        c = shard.gather_compact(crep).cpu().numpy().view(np.uint32)
        assert (c >> 31).tolist() == [1 if i == 5 else 0 for i in range(S)]
        assert (c[5] >> 16) & 0x7FFF == T - mm[5]
        sess.close()
        # P2P ChecksumReports through the all-gather, one corrupted session
        S, T, d, interval = 96, 60, 2, 5
        inputs, na, nb = networks(S, T, d, (0, 1))
        oa, ob = oracle_peer(MASK_A, S, d, interval), oracle_peer(MASK_B, S, d, interval)
        ga, gb = gpu_peer(MASK_A, S, d, interval), gpu_peer(MASK_B, S, d, interval)
        tens = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
        di, ua, ra, ub, rb = tens(inputs), tens(na[0]), tens(na[1]), tens(nb[0]), tens(nb[1])
        for t in range(T):
            if t == 23:
                oa.corrupt(40, 4 * P, 0x00100000)
                ga.debug_corrupt(40, 4 * P, 0x00100000)
            ga.run_ticks(di[t:t + 1], ua[t:t + 1], ra)
            gb.run_ticks(di[t:t + 1], ub[t:t + 1], rb)
            oracle_tick(oa, MASK_A, inputs, na, t)
            oracle_tick(ob, MASK_B, inputs, nb, t)
            exchange_oracle(oa, ob)
            rep_a, rep_b = ga.take_checksum_reports(), gb.take_checksum_reports()
            xa, xb = shard.exchange_checksum_reports(rep_a), shard.exchange_checksum_reports(rep_b)
            assert xa.shape == (1,) + tuple(rep_a.shape) and torch.equal(xa[0], rep_a) and torch.equal(xb[0], rep_b)
            ga.receive_checksum_reports(1, xb[0])
            gb.receive_checksum_reports(0, xa[0])
        for g_, o_ in ((ga, oa), (gb, ob)):
            gn, gfr, *_ = g_.desync_events()
            on, ofr, *_ = o_.desync_events(RB_P2P_EVENTS_KEPT)
            np.testing.assert_array_equal(gn, on)
            np.testing.assert_array_equal(gfr, ofr)
        assert set(np.nonzero(ga.desync_events()[0])[0].tolist()) == {40}
        ga.close()
        gb.close()
    finally:
        dist.destroy_process_group()
