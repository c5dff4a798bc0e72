"""P2P at bench size (VERDICT r03 "Parity at bench size"): the exact P2P paths the
bench lines time, at 65,536 sessions — plain rollback (lane-asynchronous ticks
over the LDS snapshot ring, 50 ticks per launch), sparse saving, the C4
speculative fan-out (P = 4, K = 16), packet-fed replay and one-tick launches
(live play) — each checked two ways:

* size-independent properties of the whole batch: no panic; the fan-out's
  cells, states and queues equal a plain rollback batch's on the same inputs
  (every rollback is a load or a select); packet-fed ticks equal directly fed
  ones; one-tick launches equal fused ones;
* a bit-exact sample of 64 sessions spread over every workgroup range
  against the oracle's P2PSession (p2p_session.rs:253-371) after every launch:
  the last tick's status, LoadGameState frame and request counts, every cell's
  frame tag / image / checksum, the live state, the frames and every queue.

Configuration = the bench lines (bench.py --session p2p): ex_game, handle 0
local, max_prediction 8, input delay 2, remote delay 2, lag 1-4, inputs 0x0F.
"""
import numpy as np
import pytest

import ggrs_amd as G
from ggrs_amd.p2p import PlayerType, synth_network
from oracle import oracle as O

pytestmark = pytest.mark.gpu

S_FULL = 65536
S_GPU5 = 131072  # config 5's per-GPU share (1,048,576 sessions over 8 GPUs): four waves per SIMD
W, D, RD, LAG = 8, 2, 2, (1, 4)


def sample_of(S):
    return np.linspace(0, S - 1, 64).astype(np.int64)  # one session in every S / 64


SAMPLE = sample_of(S_FULL)


def batch(P, sparse=False, fanout=False, K=16, S=S_FULL, per_player=False):
    b = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
         .with_input_delay(D).with_remote_input_delay(RD).with_sparse_saving_mode(sparse)
         .with_speculative_fanout(fanout, K, per_player=per_player))
    for h in range(P):
        b.add_player(PlayerType.Local if h == 0 else PlayerType.Remote, h)
    return b.start_p2p_session()


class Sample:
    """The oracle's P2PSession for the sampled sessions, driven tick by tick on the same arrays."""

    def __init__(self, P, inputs, upto, rin, sparse=False, sample=SAMPLE):
        self.P = P
        self.sample = sample
        self.inputs = np.ascontiguousarray(inputs[:, :, sample])
        self.upto = np.ascontiguousarray(upto[:, :, sample])
        self.rin = np.ascontiguousarray(rin[:, :, sample])
        self.orc = O.OracleP2P(O.EX_GAME, P, W, D, 0b1, len(sample), sparse_saving=sparse, remote_delay=RD)
        self.t = 0

    def run_to(self, t1):
        last = None
        for t in range(self.t, t1):
            for h in range(1, self.P):
                assert self.orc.deliver(h, self.upto[t, h], self.rin[:, h, :]) == 0, self.orc.last_panic()
            assert self.orc.add_local_input(0, self.inputs[t, 0]) == 0
            last = self.orc.advance()
        self.t = t1
        return last

    def compare(self, sess, last, tick):
        SAMPLE = self.sample
        ost, olf, ona, ons = last
        st, lf, na, ns = sess.status()
        for name, a, b in (("status", st, ost), ("LoadGameState frame", lf, olf), ("AdvanceFrame count", na, ona),
                           ("SaveGameState count", ns, ons)):
            np.testing.assert_array_equal(a[SAMPLE], b, err_msg=f"{name}, tick {tick}")
        tags, imgs, cs = sess.read_cells()
        otags, oimgs, ocs = self.orc.read_cells()
        np.testing.assert_array_equal(tags[:, SAMPLE], otags, err_msg=f"cell frames, tick {tick}")
        valid = otags >= 0
        np.testing.assert_array_equal(imgs[:, SAMPLE][valid], oimgs[valid], err_msg=f"cell images, tick {tick}")
        np.testing.assert_array_equal(cs[:, SAMPLE][valid], ocs[valid], err_msg=f"cell checksums, tick {tick}")
        np.testing.assert_array_equal(sess.read_live()[SAMPLE], self.orc.read_live()[0], err_msg=f"live, tick {tick}")
        c, k = sess.frames()
        oc, ok = self.orc.frames()
        np.testing.assert_array_equal(c[SAMPLE], oc)
        np.testing.assert_array_equal(k[SAMPLE], ok)
        dq, oq = sess.read_queues()[SAMPLE], self.orc.queues()
        dq[:, :, 1] = np.where(dq[:, :, 0] < 0, oq[:, :, 1], dq[:, :, 1])  # (test_p2p.compare_queues)
        np.testing.assert_array_equal(dq, oq, err_msg=f"input queues, tick {tick}")


def assert_same_batch(a, b, what):
    np.testing.assert_array_equal(a.read_live(), b.read_live(), err_msg=f"{what}: live state")
    for x, y, name in zip(a.read_cells(), b.read_cells(), ("tags", "images", "checksums")):
        np.testing.assert_array_equal(x, y, err_msg=f"{what}: cell {name}")
    np.testing.assert_array_equal(a.read_queues(), b.read_queues(), err_msg=f"{what}: input queues")
    for x, y in zip(a.frames(), b.frames()):
        np.testing.assert_array_equal(x, y, err_msg=f"{what}: frames")


def network(P, T, S=S_FULL):
    import torch
    inputs, upto, rin = synth_network(S, P, T, 0b1, RD, *LAG)
    return (inputs, upto, rin), tuple(torch.from_numpy(a).cuda() for a in (inputs, upto, rin))


@pytest.mark.parametrize("sparse", [False, True], ids=["plain", "sparse"])
def test_gpu_p2p_bench_path_at_full_size(gpu_available, sparse):
    """The bench's P2P line (50-tick launches: lane-asynchronous ticks, LDS snapshot ring), and
    with sparse saving, at 65,536 sessions: oracle sample after every launch, no panic."""
    P, T, tpl = 2, 100, 50
    (inputs, upto, rin), (di, du, dr) = network(P, T)
    sess = batch(P, sparse=sparse)
    smp = Sample(P, inputs, upto, rin, sparse=sparse)
    for t0 in range(0, T, tpl):
        sess.run_ticks(di[t0:t0 + tpl], du[t0:t0 + tpl], dr)
        smp.compare(sess, smp.run_to(t0 + tpl), t0 + tpl - 1)
    assert sess.counters()[2] == 0
    st = sess.status()[0]
    assert ((st == 0) | (st == 1)).all()
    assert sess.totals()[2] > S_FULL, "the lagged schedule must roll sessions back"


@pytest.mark.parametrize("sparse", [False, True], ids=["plain", "sparse"])
def test_gpu_p2p_four_waves_per_simd_at_config5_share(gpu_available, sparse):
    """131,072 sessions (config 5's per-GPU share) put four waves on every SIMD, so 50-tick launches
    keep only the input ring in LDS with the cells in HBM (kernels.hpp launch_p2p_as_m, p2p_kernel kQ,
    128 VGPRs): oracle sample after every launch, and the whole batch equals one run in one-tick
    launches (cells and input ring in HBM)."""
    P, T, tpl = 2, 100, 50
    (inputs, upto, rin), (di, du, dr) = network(P, T, S=S_GPU5)
    sess, live = batch(P, sparse=sparse, S=S_GPU5), batch(P, sparse=sparse, S=S_GPU5)
    smp = Sample(P, inputs, upto, rin, sparse=sparse, sample=sample_of(S_GPU5))
    for t0 in range(0, T, tpl):
        sess.run_ticks(di[t0:t0 + tpl], du[t0:t0 + tpl], dr)
        smp.compare(sess, smp.run_to(t0 + tpl), t0 + tpl - 1)
    for t in range(T):
        live.run_ticks(di[t:t + 1], du[t:t + 1], dr)
    assert_same_batch(sess, live, "50-tick (kQ) vs one-tick launches")
    assert sess.counters()[2] == 0 and sess.totals()[:3] == live.totals()[:3]
    assert sess.totals()[2] > S_GPU5, "the lagged schedule must roll sessions back"


def test_gpu_p2p_one_tick_launches_at_full_size(gpu_available):
    """Live play (one launch per tick, the cells and the input ring in HBM) at 65,536 sessions
    equals the fused 50-tick launches (LDS rings, lane-asynchronous ticks) bit for bit, and the
    oracle sample; so do 8-tick launches (HBM cells, the input ring in LDS)."""
    P, T = 2, 60
    (inputs, upto, rin), (di, du, dr) = network(P, T)
    live, fused = batch(P), batch(P)
    smp = Sample(P, inputs, upto, rin)
    for t in range(T):
        live.run_ticks(di[t:t + 1], du[t:t + 1], dr)
        if t % 20 == 19:
            smp.compare(live, smp.run_to(t + 1), t)
    fused.run_ticks(di[:30], du[:30], dr)
    fused.run_ticks(di[30:], du[30:], dr)
    assert_same_batch(live, fused, "one-tick vs fused launches")
    assert live.counters()[2] == 0 and live.totals()[:3] == fused.totals()[:3]
    mid = batch(P)  # 8-tick launches: HBM cells, the input ring in LDS (p2p.hpp kLdsQMinTicks)
    for t0 in range(0, T, 8):
        mid.run_ticks(di[t0:t0 + 8], du[t0:t0 + 8], dr)
    assert_same_batch(mid, fused, "8-tick vs fused launches")


@pytest.mark.parametrize("per_player", [False, True], ids=["one-player", "per-player"])
def test_gpu_c4_fanout_at_full_size(gpu_available, per_player):
    """BASELINE config 4 as the bench runs it (P = 4, K = 16 candidates, the in-kernel fan-out,
    50-tick launches) at 65,536 sessions, speculating the oldest-unconfirmed remote player or every
    remote player: the oracle sample after every launch; the whole batch equals a plain rollback
    batch on the same inputs, with every rollback a load or a select."""
    P, T, tpl = 4, 100, 50
    (inputs, upto, rin), (di, du, dr) = network(P, T)
    spec, plain = batch(P, fanout=True, per_player=per_player), batch(P)
    smp = Sample(P, inputs, upto, rin)
    for t0 in range(0, T, tpl):
        spec.run_ticks(di[t0:t0 + tpl], du[t0:t0 + tpl], dr)
        smp.compare(spec, smp.run_to(t0 + tpl), t0 + tpl - 1)
    plain.run_ticks(di, du, dr)
    assert_same_batch(spec, plain, "fan-out vs plain rollback")
    ts, tp = spec.totals(), plain.totals()
    assert ts[3] > 0 and ts[2] + ts[3] == tp[2], (ts, tp)  # loads + selects == the plain batch's loads
    assert spec.counters()[2] == 0 and spec.counters()[1] == 0


def test_gpu_packet_replay_at_full_size(gpu_available):
    """The bench's --wire-replay line at 65,536 sessions: every tick's packets (encoded on the
    device, 0-2 re-sent frames) decoded inside 50-tick launches and inside one-tick launches;
    both equal a directly fed batch, the acks equal the delivery schedule, no decode fails."""
    import ctypes

    import torch
    from ggrs_amd import _lib as L
    lib = L.load()
    P, T, stride = 2, 60, 32
    (inputs, upto, rin), (di, du, dr) = network(P, T)
    F = rin.shape[0]
    rng = np.random.default_rng(5)
    pk = torch.zeros((T, P, S_FULL, stride), dtype=torch.uint8, device="cuda")
    ln, st = (torch.zeros((T, P, S_FULL), dtype=torch.int32, device="cuda") for _ in range(2))
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    none = torch.full((S_FULL,), -1, dtype=torch.int32, device="cuda")
    for t in range(T):
        prev = du[t - 1, 1] if t > 0 else none
        redo = torch.from_numpy(rng.integers(0, 3, S_FULL).astype(np.int32)).cuda()
        acked = torch.where(prev < 0, prev, torch.clamp(prev - redo, min=RD - 1))
        acked = torch.where(acked < RD, none, acked).contiguous()
        assert lib.rb_encode_input_packets(0, None, 1, P, S_FULL, 1, p(dr), F, RD, p(acked), p(du[t, 1].contiguous()),
                                           p(pk[t, 1]), stride, p(ln[t, 1]), p(st[t, 1])) == 0
    torch.cuda.synchronize()
    assert int((ln < 0).sum()) == 0
    direct, fused, live = batch(P), batch(P), batch(P)
    direct.run_ticks(di, du, dr)
    acks = torch.full((P, S_FULL), -1, dtype=torch.int32, device="cuda")
    dstat = torch.zeros((P, S_FULL), dtype=torch.int32, device="cuda")
    for t0 in range(0, T, 30):
        fused.run_ticks_packets(di[t0:t0 + 30], pk[t0:t0 + 30], ln[t0:t0 + 30], st[t0:t0 + 30], dstat, acks)
        assert int((dstat < 0).sum()) == 0
    lacks = torch.full((P, S_FULL), -1, dtype=torch.int32, device="cuda")
    for t in range(T):
        live.run_ticks_packets(di[t:t + 1], pk[t:t + 1], ln[t:t + 1], st[t:t + 1], dstat, lacks)
    assert int((dstat < 0).sum()) == 0
    np.testing.assert_array_equal(acks.cpu().numpy()[1], upto[-1, 1])
    np.testing.assert_array_equal(lacks.cpu().numpy()[1], upto[-1, 1])
    assert_same_batch(fused, direct, "packet-fed (30-tick launches) vs direct")
    assert_same_batch(live, direct, "packet-fed (one-tick launches) vs direct")
    smp = Sample(P, inputs, upto, rin)
    smp.compare(live, smp.run_to(T), T - 1)
    assert live.counters()[2] == 0 and fused.counters()[2] == 0
