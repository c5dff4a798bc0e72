"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): frame indices and request streams identical;
integer-state checksums bit-exact; ex_game f32 state within 1e-5 relative.
The engine restates glibc's sinf/cosf exactly (ggrs_amd/csrc/device_math.hpp),
so ex_game is asserted BIT-EXACT here too (state images and fletcher16
checksums), which implies the 1e-5 relative tolerance (asserted as well).
"""
import ctypes

import numpy as np
import pytest

import ggrs_amd as G
from ggrs_amd.synth import synth_inputs
from oracle import oracle as O

pytestmark = pytest.mark.gpu

F32_RTOL = 1e-5  # north_star tolerance for f32 ex_game state

ORC_GAME = {G.Game.EX_GAME: O.EX_GAME, G.Game.STUB: O.STUB, G.Game.STUB_ENUM: O.STUB_ENUM,
            G.Game.STUB_RANDOM_CS: O.STUB_RANDOM_CS, G.Game.BRAWLER: O.BRAWLER}


def make_pair(game, S, P=2, W=8, cd=2, d=0, checked=True, seed=0, lane_per_session=False):
    sess = (G.SessionBuilder(game, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
            .with_check_distance(cd).with_input_delay(d).with_checked_mismatches(checked).with_seed(seed)
            .with_lane_per_session(lane_per_session).start_synctest_session())
    orc = O.OracleBatch(ORC_GAME[game], P, W, cd, d, S, seed)
    return sess, orc


def compare_cells(sess, orc, P, game):
    frames, imgs, valid, cs = orc.read_cells()
    for w, fr in enumerate(frames):
        if fr < 0:
            continue
        gimg, gcs = sess.read_cell(int(fr))
        np.testing.assert_array_equal(gimg, imgs[w], err_msg=f"cell image frame {fr}")
        assert valid[w].all()
        np.testing.assert_array_equal(gcs, cs[w], err_msg=f"cell checksum frame {fr}")
        if game == G.Game.EX_GAME:
            a = G.decode_ex_game(gimg, P)
            b = G.decode_ex_game(imgs[w], P)
            for key in ("positions", "velocities", "rotations"):
                np.testing.assert_allclose(a[key], b[key], rtol=F32_RTOL, atol=0)


def compare_live(sess, orc, game):
    gimg, gdcs, gfr = sess.read_live()
    oimg, odcs, ofr = orc.read_live()
    np.testing.assert_array_equal(gimg, oimg, err_msg="live state")
    if game == G.Game.EX_GAME:
        np.testing.assert_array_equal(gdcs, odcs, err_msg="display checksum (Game::last_checksum)")
        assert (ofr == gfr).all()


def run_parity(game, S, P, W, cd, d, T, inputs, check_every=1, checked=True, lane_per_session=False):
    sess, orc = make_pair(game, S, P, W, cd, d, checked, lane_per_session=lane_per_session)
    for t in range(T):
        for h in range(P):
            sess.add_local_input(h, inputs[t, h])
            orc.add_local_input(h, inputs[t, h])
        reqs = sess.advance_frame()
        kinds, frames = orc.advance()
        assert (kinds == 0).all(), (t, kinds[:4], orc.last_panic())
        assert [(int(r.kind), r.frame) for r in reqs] == orc.trace(0), t
        if t % check_every == 0 or t == T - 1:
            compare_cells(sess, orc, P, game)
            compare_live(sess, orc, game)
    assert (sess.mismatches() == G.NULL_FRAME).all()
    sess.close()


# ---------------------------------------------------------------------------- device math
def test_device_sincosf_bit_exact_with_glibc(gpu_available):
    import ctypes
    from ggrs_amd import _lib as L
    lo = np.float32(-0.1).view(np.uint32)
    hi = np.float32(6.4).view(np.uint32)
    pos = np.arange(0, hi, 37, dtype=np.uint32)  # every 37th float in [0, 6.4]
    neg = np.arange(0x80000000, lo, 37, dtype=np.uint32)  # [-0.1, -0]
    special = np.array([0.0, 2 * np.pi, np.pi, np.pi / 2, np.pi / 4, float.fromhex("0x1.921FB6p-1"), 1e-30, 6.2831855, 119.9],
                       np.float32).view(np.uint32)
    x = np.concatenate([pos, neg, special]).view(np.float32)
    gs = np.empty_like(x)
    gc = np.empty_like(x)
    st = L.load().rb_debug_sincosf(0, x.ctypes.data_as(ctypes.c_void_p), gs.ctypes.data_as(ctypes.c_void_p),
                                   gc.ctypes.data_as(ctypes.c_void_p), x.size)
    assert st == 0
    hs, hc = O.sincosf(x)
    bad_s = np.nonzero(gs.view(np.uint32) != hs.view(np.uint32))[0]
    bad_c = np.nonzero(gc.view(np.uint32) != hc.view(np.uint32))[0]
    assert bad_s.size == 0, (x[bad_s[:5]], gs[bad_s[:5]], hs[bad_s[:5]])
    assert bad_c.size == 0, (x[bad_c[:5]], gc[bad_c[:5]], hc[bad_c[:5]])


def test_device_inrange_sincos_and_rotation_step_every_float(gpu_available):
    """The in-range forms the timed steady kernel and the fan-out run (sincosf_glibc<true>,
    rem_euclid_near<true>, rem_euclid<true>; ex_game.rs:282-296) evaluated ON THE DEVICE for every
    float in [+0, 6.5) (1,087,373,312 values: every rotation an in-range tick can meet), bit for bit
    against this host's glibc sinf / cosf and f32::rem_euclid (fmodf)."""
    import os

    import torch
    from ggrs_amd import _lib as L
    lib = L.load()
    end = 0x40D00000  # bits of 6.5f: [+0, 6.5) is bits [0, end)
    chunk = 1 << 25
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    out = torch.empty(6 * chunk, dtype=torch.float32, device="cuda")  # [6][n] packed per chunk
    host = torch.empty(6 * chunk, dtype=torch.float32, pin_memory=True)
    total = 0
    for first in range(0, end, chunk):
        n = min(chunk, end - first)
        assert lib.rb_debug_exgame_inrange(0, first, n, ctypes.c_void_p(out.data_ptr())) == 0
        host[:6 * n].copy_(out[:6 * n])
        bad, fb = O.check_exgame_inrange(first, host[:6 * n].numpy().reshape(6, n), threads)
        assert bad == 0, (bad, hex(fb), np.uint32(fb).view(np.float32))
        total += n
    assert total == end


def test_device_speed_clamp_bit_exact(gpu_available):
    # ex_game.rs:300-304 evaluated with host IEEE f32 (numpy rounds each op)
    # against the device clamp: the short sqrt/division sequences for the
    # normal range and the full ones outside it.
    import ctypes
    from ggrs_amd import _lib as L
    rng = np.random.default_rng(11)
    n = 1 << 22
    ang = rng.uniform(0, 2 * np.pi, n)
    mag = np.concatenate([rng.uniform(6.9, 7.6, n // 2), np.exp(rng.uniform(np.log(7), np.log(1e30), n // 2))])
    vx = (mag * np.cos(ang)).astype(np.float32)
    vy = (mag * np.sin(ang)).astype(np.float32)
    # edge operands: zeros of either sign, tiny/denormal components, huge, inf, nan
    ex = np.array([0.0, -0.0, 1e-30, -1e-40, 7.0, 7.0000005, 1e19, 3e38, np.inf, -np.inf, np.nan, 4.95, -4.95], np.float32)
    gx, gy = np.meshgrid(ex, ex)
    vx = np.concatenate([vx, gx.ravel(), rng.integers(0, 1 << 32, 1 << 16, dtype=np.uint64).astype(np.uint32).view(np.float32)])
    vy = np.concatenate([vy, gy.ravel(), rng.integers(0, 1 << 32, 1 << 16, dtype=np.uint64).astype(np.uint32).view(np.float32)])
    ox = np.empty_like(vx)
    oy = np.empty_like(vy)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    assert L.load().rb_debug_speed_clamp(0, p(vx), p(vy), p(ox), p(oy), vx.size) == 0
    seven = np.float32(7.0)
    with np.errstate(all="ignore"):
        m = np.sqrt(vx * vx + vy * vy)
        c = m > seven
        hx = np.where(c, (vx * seven) / m, vx).astype(np.float32)
        hy = np.where(c, (vy * seven) / m, vy).astype(np.float32)
    assert c.sum() > n // 2
    for got, want in ((ox, hx), (oy, hy)):
        bad = np.nonzero((got.view(np.uint32) != want.view(np.uint32)) & ~(np.isnan(got) & np.isnan(want)))[0]
        assert bad.size == 0, (vx[bad[:5]], vy[bad[:5]], got[bad[:5]], want[bad[:5]])


# ---------------------------------------------------------------------------- ex_game
@pytest.mark.parametrize("P,W,cd,d", [(2, 8, 7, 2), (2, 8, 2, 0), (2, 8, 0, 0), (2, 8, 1, 0), (1, 8, 3, 1),
                                      (3, 8, 5, 2), (4, 8, 7, 2), (2, 9, 8, 0), (2, 16, 12, 3)])
def test_exgame_parity_every_tick(gpu_available, P, W, cd, d):
    S, T = 200, 70
    inputs = synth_inputs(S, P, T)
    run_parity(G.Game.EX_GAME, S, P, W, cd, d, T, inputs)


def test_lane_per_session_layout_is_an_ab_build_only(gpu_available):
    """RB_FLAG_LANE_PER_SESSION (every player of a session in one lane) measured slower than
    one lane per player (5.35 vs 4.4 us per tick); the product library
    no longer carries it and refuses the flag with the reference's InvalidRequest."""
    with pytest.raises(G.InvalidRequest, match="LANE_PER_SESSION"):
        make_pair(G.Game.EX_GAME, 64, 2, 8, 2, 0, lane_per_session=True)


def test_exgame_parity_long_run_periodic_and_wraparound(gpu_available):
    # > 128 frames wraps the input queue ring; frame 100/200 hit CHECKSUM_PERIOD.
    S, P, T = 130, 2, 260
    inputs = synth_inputs(S, P, T, seed=12345)
    run_parity(G.Game.EX_GAME, S, P, 8, 7, 2, T, inputs, check_every=37)


def test_exgame_unchecked_mode_same_results(gpu_available):
    S, P, T = 96, 2, 40
    inputs = synth_inputs(S, P, T, seed=99)
    run_parity(G.Game.EX_GAME, S, P, 8, 7, 2, T, inputs, check_every=13, checked=False)


def test_exgame_device_and_packed_inputs(gpu_available):
    import torch
    S, P, T = 128, 2, 30
    inputs = synth_inputs(S, P, T, seed=5)
    a, _ = make_pair(G.Game.EX_GAME, S, P, 8, 7, 2)
    b, orc = make_pair(G.Game.EX_GAME, S, P, 8, 7, 2)
    dev = torch.from_numpy(inputs).cuda()  # [T, P, S]
    packed = torch.from_numpy(np.ascontiguousarray(inputs.transpose(0, 2, 1))).cuda()  # [T, S, P]
    for t in range(T):
        for h in range(P):
            a.add_local_input(h, dev[t, h])
            orc.add_local_input(h, inputs[t, h])
        b.add_local_inputs(packed[t])
        a.advance_frame()
        b.advance_frame()
        orc.advance()
    compare_live(a, orc, G.Game.EX_GAME)
    compare_live(b, orc, G.Game.EX_GAME)
    compare_cells(b, orc, P, G.Game.EX_GAME)
    # rb_run_ticks: the same T ticks in one native call, device and host inputs
    c, _ = make_pair(G.Game.EX_GAME, S, P, 8, 7, 2)
    assert c.run_ticks(dev) == T
    compare_live(c, orc, G.Game.EX_GAME)
    compare_cells(c, orc, P, G.Game.EX_GAME)
    d, _ = make_pair(G.Game.EX_GAME, S, P, 8, 7, 2, checked=False)
    assert d.run_ticks(inputs[:10]) == 10 and d.run_ticks(inputs[10:]) == T - 10
    compare_live(d, orc, G.Game.EX_GAME)


# ---------------------------------------------------------------------------- integer stubs: bit-exact checksums
@pytest.mark.parametrize("cd,d", [(0, 0), (2, 0), (7, 2), (3, 5)])
def test_stub_parity_reference_inputs(gpu_available, cd, d):
    # tests/test_synctest_session.rs drive both handles with input i at tick i.
    S, T = 70, 200
    inputs = np.broadcast_to(np.arange(T, dtype=np.uint32)[:, None, None], (T, 2, S)).copy()
    run_parity(G.Game.STUB, S, 2, 8, cd, d, T, inputs, check_every=17)


def test_stub_parity_random_inputs(gpu_available):
    S, T = 300, 90
    inputs = synth_inputs(S, 2, T, mask=0xFFFFFFFF, dtype=np.uint32, seed=3)
    run_parity(G.Game.STUB, S, 2, 8, 7, 2, T, inputs, check_every=9)


def test_stub_enum_parity(gpu_available):
    # tests/test_synctest_session_enum.rs: alternating Val1/Val2 for both handles,
    # plus per-session random enum values.
    S, T = 64, 200
    alt = np.broadcast_to((np.arange(T) % 2).astype(np.uint8)[:, None, None], (T, 2, S)).copy()
    run_parity(G.Game.STUB_ENUM, S, 2, 8, 7, 2, T, alt, check_every=50)
    rnd = synth_inputs(S, 2, 60, mask=1, seed=8)
    run_parity(G.Game.STUB_ENUM, S, 2, 8, 7, 2, 60, rnd, check_every=7)


# ---------------------------------------------------------------------------- mismatch detection
def test_random_checksums_raise_mismatched_checksum(gpu_available):
    # tests/test_synctest_session.rs:87-103 (#[should_panic] on the unwrap).
    S = 50
    sess, orc = make_pair(G.Game.STUB_RANDOM_CS, S, 2, 8, 2, 2, seed=11)
    raised_at = None
    for i in range(12):
        for h in range(2):
            sess.add_local_input(h, i)
            orc.add_local_input(h, i)
        kinds, frames = orc.advance()
        try:
            sess.advance_frame()
            assert (kinds == 0).all(), i
        except G.MismatchedChecksum as e:
            raised_at = raised_at if raised_at is not None else i
            assert (kinds == 3).all()
            np.testing.assert_array_equal(e.frames, frames)  # same frame per session (2)
    assert raised_at == 4
    # failed sessions keep failing the same way and stop advancing
    img, _, _ = sess.read_live()
    oimg, _, _ = orc.read_live()
    np.testing.assert_array_equal(img, oimg)


@pytest.mark.parametrize("game,P,word,mask", [(G.Game.EX_GAME, 2, 0, 0x00000100), (G.Game.EX_GAME, 2, 9, 0x1),
                                              (G.Game.STUB, 2, 0, 0x4)])
def test_corrupted_snapshot_detected_like_oracle(gpu_available, game, P, word, mask):
    S, cd, T = 64, 7, 40
    dtype = np.uint32 if game == G.Game.STUB else np.uint8
    inputs = synth_inputs(S, P, T, seed=21, mask=0xFF if game == G.Game.STUB else 0x0F, dtype=dtype)
    sess, orc = make_pair(game, S, P, 8, cd, 2)
    victims = [3, 40]
    for t in range(T):
        if t == 15:
            # the cell loaded by the next tick: frame (current - cd)
            f = sess.current_frame() - cd
            for v in victims:
                sess.debug_corrupt_cell(v, f, word, mask)
                orc.corrupt_cell(v, f, word, mask)
        for h in range(P):
            sess.add_local_input(h, inputs[t, h])
            orc.add_local_input(h, inputs[t, h])
        kinds, frames = orc.advance()
        if (kinds != 0).any():
            with pytest.raises(G.MismatchedChecksum) as ei:
                sess.advance_frame()
            np.testing.assert_array_equal(ei.value.frames, np.where(kinds == 3, frames, -1))
        else:
            sess.advance_frame()
    bad = np.nonzero(sess.mismatches() != -1)[0]
    assert list(bad) == victims
    compare_live(sess, orc, game)


# ---------------------------------------------------------------------------- desync report export
def test_checksum_report_export(gpu_available):
    import torch
    S = 100
    sess, orc = make_pair(G.Game.EX_GAME, S, 2, 8, 7, 2)
    inputs = synth_inputs(S, 2, 20)
    for t in range(20):
        for h in range(2):
            sess.add_local_input(h, inputs[t, h])
        sess.advance_frame()
    f = sess.current_frame() - 1
    out = torch.zeros((S, 3), dtype=torch.int64, device="cuda")  # 24-byte rb_checksum_report
    sess.export_checksum_report(f, out.data_ptr())
    sess.synchronize()
    rep = out.cpu().numpy().view(np.uint64)
    _, cs = sess.read_cell(f)
    np.testing.assert_array_equal(rep[:, 0], cs[:, 0])
    np.testing.assert_array_equal(rep[:, 1], cs[:, 1])
    fr = np.ascontiguousarray(rep[:, 2]).view(np.int32).reshape(S, 2)
    assert (fr[:, 0] == f).all() and (fr[:, 1] == -1).all()


# ---------------------------------------------------------------------------- bench-size properties
def test_bench_config_65536_sessions_sampled_parity(gpu_available):
    """BASELINE config 2 at full size: 65,536 ex_game sessions, cd=7, delay 2.
    Properties at full size: no session reports a mismatch (the resimulation is
    deterministic) and every tick's stream matches; a sample of sessions is
    compared bit-exactly with the oracle run on the same per-session inputs."""
    import torch
    S, P, T = 65536, 2, 48
    inputs = synth_inputs(S, P, T)
    sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_check_distance(7)
            .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
    dev = torch.from_numpy(inputs).cuda()
    for t in range(T):
        for h in range(P):
            sess.add_local_input(h, dev[t, h])
        sess.advance_frame()
    assert (sess.mismatches() == -1).all()
    rng = np.random.default_rng(0)
    sample = np.sort(rng.choice(S, 64, replace=False))
    orc = O.OracleBatch(O.EX_GAME, P, 8, 7, 2, sample.size)
    for t in range(T):
        for h in range(P):
            orc.add_local_input(h, inputs[t, h, sample])
        k, _ = orc.advance()
        assert (k == 0).all()
    gimg, gdcs, _ = sess.read_live()
    oimg, odcs, _ = orc.read_live()
    np.testing.assert_array_equal(gimg[sample], oimg)
    np.testing.assert_array_equal(gdcs[sample], odcs)
    frames, oc, _, ocs = orc.read_cells()
    for w, fr in enumerate(frames):
        gi, gc = sess.read_cell(int(fr))
        np.testing.assert_array_equal(gi[sample], oc[w])
        np.testing.assert_array_equal(gc[sample], ocs[w])


def test_bench_config_65536_sessions_fused_path_sampled_parity(gpu_available):
    """BASELINE config 2 at exactly 65,536 sessions through the path bench.py
    times (rb_run_ticks: the fused steady_kernel), in the driver's chunks: 8
    start-up ticks, a 5-tick warmup launch, a 20-tick launch (the timed one),
    then a 50-tick launch and 7 one-tick calls (the realtime block).  No
    session mismatches; 64 sampled sessions are bit-exact with the oracle
    (live state, display checksums, every cell)."""
    import torch
    S, P = 65536, 2
    chunks = [8, 5, 20, 50] + [1] * 7
    T = sum(chunks)
    inputs = synth_inputs(S, P, T)
    sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_check_distance(7)
            .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
    dev = torch.from_numpy(inputs).cuda()
    t = 0
    for n in chunks:
        assert sess.run_ticks(dev[t:t + n]) == n
        t += n
    assert sess.current_frame() == T
    assert (sess.mismatches() == -1).all()
    rng = np.random.default_rng(3)
    sample = np.sort(rng.choice(S, 64, replace=False))
    orc = O.OracleBatch(O.EX_GAME, P, 8, 7, 2, sample.size)
    for t in range(T):
        for h in range(P):
            orc.add_local_input(h, inputs[t, h, sample])
        k, _ = orc.advance()
        assert (k == 0).all()
    gimg, gdcs, _ = sess.read_live()
    oimg, odcs, _ = orc.read_live()
    np.testing.assert_array_equal(gimg[sample], oimg)
    np.testing.assert_array_equal(gdcs[sample], odcs)
    frames, oc, _, ocs = orc.read_cells()
    for w, fr in enumerate(frames):
        gi, gc = sess.read_cell(int(fr))
        np.testing.assert_array_equal(gi[sample], oc[w])
        np.testing.assert_array_equal(gc[sample], ocs[w])


def test_config5_shard_131072_sessions_with_audit_replicas(gpu_available):
    """BASELINE config 5's per-GPU shard as bench.py --gpus 8 runs it on rank 7:
    global sessions [7*131072, 8*131072) plus 64 audit replicas of rank 0's
    first sessions, through the fused rb_run_ticks path (58 ticks: 8 start-up
    + one 50-tick launch).  Full size: no mismatch anywhere.  Sampled owned
    sessions and every replica are bit-exact with the oracle, and the
    replicas' checksum reports equal those of the owner's batch (rank 0's
    shard, run separately): the audit compare of bench.py finds nothing."""
    import torch
    from ggrs_amd import shard
    S, A, P, T, rank = 131072, 64, 2, 58, 7
    lo = rank * S
    inputs = np.concatenate([synth_inputs(S, P, T, first_session=lo), synth_inputs(A, P, T, first_session=0)], 2)
    dev = torch.from_numpy(np.ascontiguousarray(inputs)).cuda()
    sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S + A).with_num_players(P).with_check_distance(7)
            .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
    assert sess.run_ticks(dev[:8]) == 8 and sess.run_ticks(dev[8:]) == T - 8
    assert (sess.mismatches() == -1).all()
    rng = np.random.default_rng(5)
    sample = np.concatenate([np.sort(rng.choice(S, 64, replace=False)), np.arange(S, S + A)])
    orc = O.OracleBatch(O.EX_GAME, P, 8, 7, 2, sample.size)
    for t in range(T):
        for h in range(P):
            orc.add_local_input(h, inputs[t, h, sample])
        k, _ = orc.advance()
        assert (k == 0).all()
    gimg, gdcs, _ = sess.read_live()
    oimg, odcs, _ = orc.read_live()
    np.testing.assert_array_equal(gimg[sample], oimg)
    np.testing.assert_array_equal(gdcs[sample], odcs)
    frames, oc, _, ocs = orc.read_cells()
    for w, fr in enumerate(frames):
        gi, gc = sess.read_cell(int(fr))
        np.testing.assert_array_equal(gi[sample], oc[w])
        np.testing.assert_array_equal(gc[sample], ocs[w])
    # the owner of the replicated sessions: rank 0's first A sessions in a batch of their own
    owner = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=A).with_num_players(P).with_check_distance(7)
             .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
    owner.run_ticks(torch.from_numpy(np.ascontiguousarray(inputs[:, :, S:])).cuda())
    f = T - 1
    rep = torch.zeros((S + A, shard.REPORT_WORDS), dtype=torch.int64, device="cuda")
    own = torch.zeros((A, shard.REPORT_WORDS), dtype=torch.int64, device="cuda")
    sess.export_checksum_report(f, rep.data_ptr())
    owner.export_checksum_report(f, own.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(rep[S:], own)
    # a 2-rank gather image: this batch as rank 1 of 2, the owner's batch as rank 0's first sessions
    # (rank 0's own replicas of rank 1's first sessions are those sessions' rows themselves)
    g = torch.cat([own, torch.zeros((S - A, shard.REPORT_WORDS), dtype=torch.int64, device="cuda"), rep[:A], rep])
    n, _ = shard.audit_compare(g, 2, S, A)
    assert int(n) == 0
    sess.close()
    owner.close()


# ---------------------------------------------------------------------------- fused steady-state ticks (rb_run_ticks)
@pytest.mark.parametrize("game,P,W,cd,d", [(G.Game.EX_GAME, 2, 8, 7, 2), (G.Game.EX_GAME, 2, 8, 1, 0),
                                           (G.Game.EX_GAME, 1, 8, 4, 0), (G.Game.EX_GAME, 3, 6, 5, 1),
                                           (G.Game.EX_GAME, 4, 9, 8, 3), (G.Game.EX_GAME, 2, 12, 11, 2),
                                           (G.Game.STUB, 2, 8, 7, 2), (G.Game.STUB, 2, 8, 2, 0),
                                           (G.Game.STUB_ENUM, 2, 8, 3, 1), (G.Game.EX_GAME, 2, 4, 3, 0),
                                           (G.Game.EX_GAME, 2, 17, 16, 1), (G.Game.STUB, 2, 16, 13, 0),
                                           (G.Game.EX_GAME, 2, 24, 20, 0)])
def test_run_ticks_fused_parity(gpu_available, game, P, W, cd, d):
    """rb_run_ticks fuses consecutive steady-state ticks into one launch
    (steady_kernel<G, CD>, CD <= 16; larger cd falls back to per-tick launches,
    the cd 20 case).  Chunks of ticks are compared bit-exactly with the oracle."""
    import torch
    S, T = 150, 120
    mask, dtype = (0xFFFFFFFF, np.uint32) if game == G.Game.STUB else ((1, np.uint8) if game == G.Game.STUB_ENUM
                                                                      else (0x0F, np.uint8))
    inputs = synth_inputs(S, P, T, seed=77, mask=mask, dtype=dtype)
    sess, orc = make_pair(game, S, P, W, cd, d)
    dev = torch.from_numpy(inputs).cuda()
    t = 0
    for chunk in (3, 9, 1, 30, 13, 64):
        n = min(chunk, T - t)
        assert sess.run_ticks(dev[t:t + n]) == n
        for k in range(t, t + n):
            for h in range(P):
                orc.add_local_input(h, inputs[k, h])
            kinds, _ = orc.advance()
            assert (kinds == 0).all()
        t += n
        assert [(int(r.kind), r.frame) for r in sess.last_requests()] == orc.trace(0)
        compare_cells(sess, orc, P, game)
        compare_live(sess, orc, game)
    assert t == T


def test_run_ticks_ring_limit_falls_back_to_per_tick_launches(gpu_available, monkeypatch):
    """The fused kernel addresses ex_game's snapshot ring with 32-bit offsets (kernels.hpp
    steady_saddr), so a batch whose ring reaches 4 GiB runs per-tick launches instead.
    RB_STEADY_RING_LIMIT lowers that limit: with it the same calls run unfused (the profile
    covers only every 8th tick) and stay bit-exact with the oracle; without it they fuse."""
    import torch
    S, P, W, cd, d, T = 96, 2, 8, 7, 2, 60
    inputs = synth_inputs(S, P, T, seed=5)
    dev = torch.from_numpy(inputs).cuda()
    covered = {}
    for limit in ("1", None):
        if limit:
            monkeypatch.setenv("RB_STEADY_RING_LIMIT", limit)
        else:
            monkeypatch.delenv("RB_STEADY_RING_LIMIT", raising=False)
        sess, orc = make_pair(G.Game.EX_GAME, S, P, W, cd, d)
        assert sess.run_ticks(dev[:cd + 1]) == cd + 1  # start-up ticks
        sess.profile_enable(True)
        assert sess.run_ticks(dev[cd + 1:]) == T - cd - 1
        covered[limit] = sess.profile_take()[1]
        for k in range(T):
            for h in range(P):
                orc.add_local_input(h, inputs[k, h])
            orc.advance()
        compare_cells(sess, orc, P, G.Game.EX_GAME)
        compare_live(sess, orc, G.Game.EX_GAME)
        sess.close()
    assert covered[None] == T - cd - 1  # one fused launch covers every steady tick
    assert covered["1"] < (T - cd - 1) // 2  # per-tick launches, every 8th one timed


def test_run_ticks_fused_mismatch_and_corruption(gpu_available):
    """Mismatches detected inside a fused launch freeze exactly the sessions
    (and report exactly the frames) that per-tick execution reports."""
    import torch
    S, P, cd = 64, 2, 7
    inputs = synth_inputs(S, P, 60, seed=4)
    sess, orc = make_pair(G.Game.EX_GAME, S, P, 8, cd, 2, checked=True)
    dev = torch.from_numpy(inputs).cuda()
    sess.run_ticks(dev[:20])
    for k in range(20):
        for h in range(P):
            orc.add_local_input(h, inputs[k, h])
        orc.advance()
    f = sess.current_frame() - cd
    for v in (5, 33):
        sess.debug_corrupt_cell(v, f, 8 if v == 5 else 1, 0x10)
        orc.corrupt_cell(v, f, 8 if v == 5 else 1, 0x10)
    with pytest.raises(G.MismatchedChecksum) as ei:
        sess.run_ticks(dev[20:60])
    last_frames = None
    for k in range(20, 60):
        for h in range(P):
            orc.add_local_input(h, inputs[k, h])
        kinds, frames = orc.advance()
        if (kinds != 0).any():
            last_frames = np.where(kinds == 3, frames, -1)
    np.testing.assert_array_equal(ei.value.frames, last_frames)
    assert list(np.nonzero(ei.value.frames != -1)[0]) == [5, 33]
    compare_live(sess, orc, G.Game.EX_GAME)
    compare_cells(sess, orc, P, G.Game.EX_GAME)  # frozen sessions' cells end as after their failing tick


def test_random_checksums_fused_mismatch_like_oracle(gpu_available):
    """The random-checksum stub (tests/stubs.rs RandomChecksumGameStub) through fused
    launches: its u128 checksums go through the fused kernel's 32-bit-offset checksum
    stores, and every session fails at the frame per-tick execution reports."""
    import torch
    S, P, cd = 70, 2, 2
    inputs = np.tile(np.arange(30, dtype=np.uint32)[:, None, None], (1, P, S))
    sess, orc = make_pair(G.Game.STUB_RANDOM_CS, S, P, 8, cd, 2, seed=11)
    dev = torch.from_numpy(inputs).cuda()
    with pytest.raises(G.MismatchedChecksum) as ei:
        sess.run_ticks(dev)
    first = None
    for k in range(30):
        for h in range(P):
            orc.add_local_input(h, inputs[k, h])
        kinds, frames = orc.advance()
        if first is None and (kinds != 0).any():
            first = np.where(kinds == 3, frames, -1)
    assert first is not None and (first != -1).all()
    np.testing.assert_array_equal(ei.value.frames, first)
    img, _, _ = sess.read_live()
    oimg, _, _ = orc.read_live()
    np.testing.assert_array_equal(img, oimg)


def test_prepared_ticks_same_as_run_ticks(gpu_available):
    """session.prepare_ticks (bench.py's timed loop: the native call built
    ahead) runs exactly run_ticks: chunks of ticks through prepared calls on
    the batch stream, bit-exact with the oracle; an error status raises like
    run_ticks."""
    import torch
    S, P, cd, d, T = 130, 2, 7, 2, 70
    inputs = synth_inputs(S, P, T, seed=91)
    sess, orc = make_pair(G.Game.EX_GAME, S, P, 8, cd, d)
    stream = torch.cuda.Stream()
    sess.set_stream(stream)
    dev = torch.from_numpy(inputs).cuda()
    t = 0
    with torch.cuda.stream(stream):
        for n in (8, 5, 20, 1, 36):
            call, check = sess.prepare_ticks(dev[t:t + n])
            assert check(call()) == n
            for k in range(t, t + n):
                for h in range(P):
                    orc.add_local_input(h, inputs[k, h])
                kinds, _ = orc.advance()
                assert (kinds == 0).all()
            t += n
        assert [(int(r.kind), r.frame) for r in sess.last_requests()] == orc.trace(0)
        compare_cells(sess, orc, P, G.Game.EX_GAME)
        compare_live(sess, orc, G.Game.EX_GAME)
        with pytest.raises(G.InvalidRequest):
            sess.prepare_ticks(dev[0:0])
    with pytest.raises(G.InvalidRequest):  # torch's current stream is not the batch stream
        sess.prepare_ticks(dev[0:1])
