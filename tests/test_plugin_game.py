"""The handler plug-in path: a game defined outside the engine
(tests/plugin_game/orbit_game.hpp, written to include/ggrs_amd_game.hpp),
compiled against the engine's kernels into its own library
(ggrs_amd/csrc/plugin.hip, built by __graft_entry__.build), registered at run
time (rb_register_game_plugin) and checked against the oracle's restated
SyncTestSession / P2PSession running the same game code on the CPU
(oracle/plugin_game.hpp, oracle/build/liboracle_orbit.so).

This is the reference's Config trait + handle_requests surface (lib.rs:240-262,
ex_game.rs:76-84): nothing in ggrs_amd/csrc knows OrbitGame.
"""
import ctypes
import os

import numpy as np
import pytest

import ggrs_amd as G
from ggrs_amd.p2p import PlayerType, synth_network
from ggrs_amd.plugin import register_game_plugin
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLUGIN = os.path.join(ROOT, "tests", "plugin_game", "libggrs_game_orbit.so")
ORC = O.plugin_lib("orbit")
P, STATE_WORDS = 3, 15


def orbit_inputs(S, T, seed=7):
    return G.synth_inputs(S, P, T, seed=seed, mask=0x1F)  # 5 input bits: left/right/up/down/boost


def test_plugin_library_exports_the_contract():
    lib = ctypes.CDLL(PLUGIN)
    abi = int(open(os.path.join(ROOT, "include", "ggrs_amd_game.hpp")).read().split("#define RB_PLUGIN_ABI ")[1].split()[0])
    assert lib.rb_plugin_abi() == abi  # the engine and the plugin agree on the kernel parameter layouts
    assert lib.rb_plugin_players() == P
    assert hasattr(lib, "rb_plugin_make_ops")


def test_register_is_idempotent_and_rejects_non_plugins():
    a = register_game_plugin(PLUGIN)
    assert a >= 1000 and register_game_plugin(PLUGIN) == a
    with pytest.raises(G.InvalidRequest):
        register_game_plugin(os.path.join(ROOT, "oracle", "build", "liboracle.so"))  # no plugin entry points
    with pytest.raises(G.InvalidRequest):
        register_game_plugin("/nonexistent/libgame.so")


def test_oracle_plugin_game_passes_the_reference_synctest_test():
    # tests/test_synctest_session.rs:68-85 with the plugin game: cd 7, input delay 2,
    # 200 frames, every advance Ok and the game's frame is i + 1
    S, T = 8, 200
    orc = O.OracleBatch(O.PLUGIN, P, 8, 7, 2, S, lib_path=ORC)
    x = orbit_inputs(S, T)
    for t in range(T):
        for h in range(P):
            orc.add_local_input(h, x[t, h])
        k, _ = orc.advance()
        assert (k == 0).all(), orc.last_panic()
        img, _, _ = orc.read_live()
        assert (img[:, :4].copy().view(np.int32)[:, 0] == t + 1).all()


def test_plan_only_batch_of_a_plugin_game_emits_the_reference_stream():
    gid = register_game_plugin(PLUGIN)
    S, T = 4, 30
    plan = (G.SessionBuilder(gid, num_sessions=S, device=-1).with_num_players(P).with_check_distance(3)
            .with_input_delay(1).start_synctest_session())
    assert plan.state_bytes == 4 + 4 * STATE_WORDS
    orc = O.OracleBatch(O.PLUGIN, P, 8, 3, 1, S, lib_path=ORC)
    x = orbit_inputs(S, T)
    for t in range(T):
        for h in range(P):
            plan.add_local_input(h, x[t, h])
            orc.add_local_input(h, x[t, h])
        reqs = plan.advance_frame()
        assert (orc.advance()[0] == 0).all()
        assert [(int(r.kind), r.frame) for r in reqs] == orc.trace(0)


@pytest.mark.gpu
@pytest.mark.parametrize("cd,d", [(7, 2), (2, 0), (0, 0), (5, 3)])
def test_gpu_plugin_synctest_bit_exact(gpu_available, cd, d):
    import torch
    gid = register_game_plugin(PLUGIN)
    S, T = 300, 60
    sess = (G.SessionBuilder(gid, num_sessions=S).with_num_players(P).with_check_distance(cd)
            .with_input_delay(d).with_checked_mismatches(False).start_synctest_session())
    orc = O.OracleBatch(O.PLUGIN, P, 8, cd, d, S, lib_path=ORC)
    x = orbit_inputs(S, T)
    dx = torch.from_numpy(x).cuda()
    half = T // 2
    for t in range(half):  # per-tick calls, then fused runs
        for h in range(P):
            sess.add_local_input(h, dx[t, h])
            orc.add_local_input(h, x[t, h])
        reqs = sess.advance_frame()
        assert (orc.advance()[0] == 0).all()
        assert [(int(r.kind), r.frame) for r in reqs] == orc.trace(0)
    sess.run_ticks(dx[half:])
    for t in range(half, T):
        for h in range(P):
            orc.add_local_input(h, x[t, h])
        assert (orc.advance()[0] == 0).all()
    assert (sess.mismatches() == G.NULL_FRAME).all()
    np.testing.assert_array_equal(sess.read_live()[0], orc.read_live()[0])
    frames, cells, _, cs = orc.read_cells()
    for w, fr in enumerate(frames):
        if fr < 0:
            continue
        img, c = sess.read_cell(int(fr))
        np.testing.assert_array_equal(img, cells[w])
        np.testing.assert_array_equal(c, cs[w])
    sess.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mask,sparse,lag", [(0b001, False, (1, 4)), (0b010, True, (0, 5)), (0b101, False, (2, 6))])
def test_gpu_plugin_p2p_matches_oracle_every_tick(gpu_available, mask, sparse, lag):
    # the game folds InputStatus into its state, so Predicted / Confirmed inputs are checked too
    import torch
    gid = register_game_plugin(PLUGIN)
    S, T, W, d, rd = 96, 70, 8, 1, 2
    inputs, upto, rin = synth_network(S, P, T, mask, rd, lag[0], lag[1], mask=0x1F)
    b = (G.SessionBuilder(gid, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
         .with_input_delay(d).with_remote_input_delay(rd).with_sparse_saving_mode(sparse))
    for h in range(P):
        b.add_player(PlayerType.Local if (mask >> h) & 1 else PlayerType.Remote, h)
    sess = b.start_p2p_session()
    orc = O.OracleP2P(O.PLUGIN, P, W, d, mask, S, sparse_saving=sparse, remote_delay=rd, lib_path=ORC)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    rolled = False
    for t in range(T):
        sess.run_ticks(di[t:t + 1], du[t:t + 1], dr)
        for h in range(P):
            if not (mask >> h) & 1:
                assert orc.deliver(h, upto[t, h], rin[:, h, :]) == 0
        for h in range(P):
            if (mask >> h) & 1:
                orc.add_local_input(h, inputs[t, h])
        ost, olf, ona, ons = orc.advance()
        st, lf, na, ns = sess.status()
        np.testing.assert_array_equal(st, ost, err_msg=f"tick {t}")
        np.testing.assert_array_equal(lf, olf, err_msg=f"tick {t}")
        np.testing.assert_array_equal(na, ona)
        np.testing.assert_array_equal(ns, ons)
        rolled |= bool((lf >= 0).any())
        if t % 10 == 9:
            np.testing.assert_array_equal(sess.read_live(), orc.read_live()[0], err_msg=f"live, tick {t}")
            tags, imgs, cs = sess.read_cells()
            otags, oimgs, ocs = orc.read_cells()
            np.testing.assert_array_equal(tags, otags)
            v = otags >= 0
            np.testing.assert_array_equal(imgs[v], oimgs[v])
            np.testing.assert_array_equal(cs[v], ocs[v])
    assert rolled
    sess.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ticks_per_call", [1, 30], ids=["live", "fused"])
def test_gpu_plugin_packet_decode_status_per_endpoint(gpu_available, ticks_per_call):
    # One lane serves all three players of the plug-in game (two remote endpoints per lane): a bad
    # packet from one endpoint must be reported for that endpoint only (UdpProtocol::on_input is
    # per endpoint, protocol.rs:616-689), the other endpoint's status stays its own decode result.
    import torch

    from ggrs_amd import _lib as L
    from test_wire import _encode_schedule
    lib = L.load()
    gid = register_game_plugin(PLUGIN)
    S, T, W, mask, rd, stride = 96, 60, 8, 0b001, 1, 32
    inputs, upto, rin = synth_network(S, P, T, mask, rd, 1, 4, mask=0x1F)
    b = (G.SessionBuilder(gid, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
         .with_input_delay(1).with_remote_input_delay(rd))
    for h in range(P):
        b.add_player(PlayerType.Local if (mask >> h) & 1 else PlayerType.Remote, h)
    wired = b.start_p2p_session()
    di, dr = torch.from_numpy(inputs).cuda(), torch.from_numpy(rin).cuda()
    pk, ln, st = _encode_schedule(lib, P, S, T, mask, rd, upto, dr, stride, seed=5)
    bad_t, a_s, b_s = 30, 11, 40
    k = int(ln[bad_t, 1, a_s])
    assert k > 0 and int(ln[bad_t, 2, a_s]) > 0 and int(ln[bad_t, 2, b_s]) > 0
    pk[bad_t, 1, a_s, k - 1] |= 0x80                  # endpoint 1 of session a: truncated varint (-1)
    st[bad_t, 2, b_s] = upto[bad_t - 1, 2, b_s] + 2   # endpoint 2 of session b: skips a frame (-2)
    dstat = torch.zeros((P, S), dtype=torch.int32, device="cuda")
    t = 0
    while t < T:
        n = min(ticks_per_call, T - t)
        wired.run_ticks_packets(di[t:t + n], pk[t:t + n], ln[t:t + n], st[t:t + n], dstat)
        t += n
    d = dstat.cpu().numpy()
    assert d[1, a_s] == -1 and d[2, b_s] == -2, (d[:, a_s], d[:, b_s])
    assert d[2, a_s] >= 0 and d[1, b_s] >= 0, (d[:, a_s], d[:, b_s])  # the good endpoint of each
    status = wired.status()[0]
    assert status[a_s] == 101 and status[b_s] == 101 and wired.counters()[2] == 2
    wired.close()
