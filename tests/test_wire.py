"""Batched input packets: network/compression.rs's wire
format (XOR delta + bitfield RLE) restated in the oracle and on the device.

Pinning: the reference's only test of the format is the round trip of
compression.rs:81-90 (restated in oracle/ref_tests.cpp and here).  bitfield-rle
0.2 is not vendored: decoding follows its published format, which defines the
decoded bytes; the encoder's choice of runs to compress is this build's
(runs >= 4 bytes), so encoded bytes are "parity unpinned" against the crate
(device == oracle byte for byte is still checked).
"""
import numpy as np
import pytest

from oracle import oracle as O


def rand_inputs(rng, n, ib):
    # hold-model streams: long repeats XOR to zero runs, as on the wire
    vals = rng.integers(0, 256, (n, ib), dtype=np.uint8)
    keep = rng.random(n) < 0.7
    for i in range(1, n):
        if keep[i]:
            vals[i] = vals[i - 1]
    return vals


def test_reference_round_trip_vector():
    # compression.rs:81-90
    ref = bytes([0, 0, 0, 1])
    pend = [[0, 0, 1, 0], [0, 0, 1, 1], [0, 1, 0, 0], [0, 1, 0, 1], [0, 1, 1, 0]]
    enc = O.wire_encode(ref, pend)
    assert O.wire_decode(ref, enc).tolist() == pend


@pytest.mark.parametrize("ib", [1, 2, 4])
def test_random_round_trips_and_compression(ib):
    rng = np.random.default_rng(ib)
    saw_run = False
    for _ in range(300):
        n = int(rng.integers(1, 40))
        ref = rng.integers(0, 256, ib, dtype=np.uint8).tobytes()
        ins = rand_inputs(rng, n, ib)
        if rng.random() < 0.3:
            ins[:] = np.frombuffer(ref, np.uint8)  # all equal to the reference: one zero run
        enc = O.wire_encode(ref, ins)
        dec = O.wire_decode(ref, enc)
        np.testing.assert_array_equal(dec, ins)
        saw_run |= any(b & 1 for b in enc[:1])
    assert saw_run


def test_malformed_packets_are_rejected():
    ref = b"\x00"
    assert O.wire_decode(ref, bytes([0x80])) is None          # truncated varint
    assert O.wire_decode(ref, bytes([0x06, 0x01])) is None    # literal of 3 bytes, 1 present
    assert O.wire_decode(ref, bytes([0x02, 0x07])).tolist() == [[7]]


# ---------------------------------------------------------------------------- device
def on_input_reference(last, start, data, ref_input, max_pred, ib):
    """protocol.rs:616-689 for one endpoint: (new inputs by frame, new last, status)."""
    if len(data) == 0:
        return {}, last, 1
    if last != -1 and last + 1 < start:
        return {}, last, -2
    if last != -1 and start - 1 < last - 2 * max_pred:
        return {}, last, 1
    if last != -1 and start - 1 < -1:  # recv_inputs holds no such frame: the packet is ignored (:653)
        return {}, last, 1
    ref = bytes(ib) if (last == -1 or start - 1 == -1) else ref_input
    dec = O.wire_decode(ref, data)
    if dec is None:
        return {}, last, -1
    out = {}
    for i, inp in enumerate(dec):
        f = start + i
        if f > last:
            out[f] = inp.tobytes()
    new_last = max(out) if out else last
    return out, new_last, 0 if out else 1


@pytest.mark.gpu
@pytest.mark.parametrize("ib", [1, 4])
def test_gpu_encode_matches_oracle_and_decode_matches_on_input(gpu_available, ib):
    import ctypes

    import torch

    from ggrs_amd import _lib as L
    lib = L.load()
    rng = np.random.default_rng(100 + ib)
    S, P, h, F, W, stride = 3000, 2, 1, 64, 8, 96
    dt = np.uint8 if ib == 1 else np.uint32
    inputs = np.zeros((F, P, S), dt)
    for s in range(S):
        inputs[:, h, s] = rand_inputs(rng, F, ib).view(dt).reshape(F)
    acked = rng.integers(-1, 30, S).astype(np.int32)
    newest = (acked + rng.integers(0, 12, S)).astype(np.int32)
    d_in = torch.from_numpy(inputs).cuda()
    d_ack, d_new = torch.from_numpy(acked).cuda(), torch.from_numpy(newest).cuda()
    pk = torch.zeros((S, stride), dtype=torch.uint8, device="cuda")
    ln = torch.zeros(S, dtype=torch.int32, device="cuda")
    st = torch.zeros(S, dtype=torch.int32, device="cuda")
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    assert lib.rb_encode_input_packets(0, None, h, P, S, ib, p(d_in), F, 0, p(d_ack), p(d_new), p(pk), stride, p(ln),
                                       p(st)) == 0
    torch.cuda.synchronize()
    pk_h, ln_h, st_h = pk.cpu().numpy(), ln.cpu().numpy(), st.cpu().numpy()
    raw = inputs.view(np.uint8).reshape(F, P, S, ib)
    for s in range(S):
        assert st_h[s] == acked[s] + 1
        n = newest[s] - acked[s]
        if n <= 0:
            assert ln_h[s] == 0
            continue
        ref = bytes(ib) if acked[s] == -1 else raw[acked[s], h, s].tobytes()
        want = O.wire_encode(ref, raw[acked[s] + 1:newest[s] + 1, h, s])
        assert pk_h[s, :ln_h[s]].tobytes() == want, s
    # decode: receiver state `last` per session, some packets corrupted / gapped / stale
    last = rng.integers(-1, 40, S).astype(np.int32)
    recv = np.zeros((F, P, S), dt)
    recv[:, h, :] = inputs[:, h, :]  # frames <= last are known to the receiver
    start = st_h.copy()
    lens = ln_h.copy()
    bad = rng.random(S) < 0.05
    pk_h2 = pk_h.copy()
    for s in np.nonzero(bad)[0]:
        if lens[s] > 0:
            lens[s] = max(1, lens[s] - 1)
            pk_h2[s, lens[s] - 1] |= 0x80  # truncated varint / literal
    neg = np.nonzero(~bad & (lens > 0))[0][:25]  # packets claiming a negative start frame
    start[neg] = -3
    last[neg] = np.minimum(last[neg], 4).clip(0)
    upto = np.full((P, S), -1, np.int32)
    upto[h] = last
    d_recv = torch.from_numpy(recv).cuda()
    d_upto = torch.from_numpy(upto).cuda()
    d_pk = torch.from_numpy(pk_h2).cuda()
    d_len, d_start = torch.from_numpy(lens).cuda(), torch.from_numpy(start).cuda()
    d_st = torch.zeros(S, dtype=torch.int32, device="cuda")
    assert lib.rb_decode_input_packets(0, None, h, P, S, ib, W, p(d_pk), stride, p(d_len), p(d_start), p(d_recv), F,
                                       p(d_upto), p(d_st)) == 0
    torch.cuda.synchronize()
    got_recv = d_recv.cpu().numpy().view(np.uint8).reshape(F, P, S, ib)
    got_upto, got_st = d_upto.cpu().numpy(), d_st.cpu().numpy()
    kinds = set()
    for s in range(S):
        refin = raw[start[s] - 1, h, s].tobytes() if start[s] >= 1 else bytes(ib)
        out, nl, code = on_input_reference(int(last[s]), int(start[s]), pk_h2[s, :lens[s]].tobytes(), refin, W, ib)
        kinds.add(code)
        assert got_st[s] == code, (s, got_st[s], code)
        assert got_upto[h, s] == nl
        for f, b in out.items():
            assert got_recv[f, h, s].tobytes() == b
    assert {0, 1, -1, -2} <= kinds


@pytest.mark.gpu
@pytest.mark.parametrize("P,mask,rd", [(2, 0b01, 2), (4, 0b0001, 1)])
def test_gpu_p2p_fed_through_the_wire_equals_direct_delivery(gpu_available, P, mask, rd):
    # Remote peers encode their pending inputs on the device (re-sending up to 2
    # already-received frames, as an un-acked sender does), the receiver decodes
    # them on the device into the delivery tensors, and the P2P batch runs on
    # them: cells and state must equal a batch fed the same deliveries directly.
    import ctypes

    import torch

    import ggrs_amd as G
    from ggrs_amd import _lib as L
    from ggrs_amd.p2p import PlayerType, synth_network
    lib = L.load()
    S, W, T, stride = 512, 8, 96, 64
    inputs, upto, rin = synth_network(S, P, T, mask, rd, 1, 5)
    F = rin.shape[0]

    def batch():
        b = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
             .with_input_delay(1).with_remote_input_delay(rd))
        for hh in range(P):
            b.add_player(PlayerType.Local if (mask >> hh) & 1 else PlayerType.Remote, hh)
        return b.start_p2p_session()

    direct, wired = batch(), batch()
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    recv = torch.zeros_like(dr)
    rupto = torch.full((P, S), -1, dtype=torch.int32, device="cuda")
    pk = torch.zeros((S, stride), dtype=torch.uint8, device="cuda")
    ln = torch.zeros(S, dtype=torch.int32, device="cuda")
    st = torch.zeros(S, dtype=torch.int32, device="cuda")
    dst = torch.zeros(S, dtype=torch.int32, device="cuda")
    rng = np.random.default_rng(3)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    for t in range(T):
        direct.run_ticks(di[t:t + 1], du[t:t + 1], dr)
        for hh in range(P):
            if (mask >> hh) & 1:
                continue
            redo = torch.from_numpy(rng.integers(0, 3, S).astype(np.int32)).cuda()
            acked = torch.where(rupto[hh] < 0, rupto[hh], torch.clamp(rupto[hh] - redo, min=rd - 1))
            acked = torch.where(acked < rd, torch.full_like(acked, -1), acked).contiguous()
            newest = du[t, hh].contiguous()
            assert lib.rb_encode_input_packets(0, None, hh, P, S, 1, p(dr), F, rd, p(acked), p(newest), p(pk), stride,
                                               p(ln), p(st)) == 0
            assert lib.rb_decode_input_packets(0, None, hh, P, S, 1, W, p(pk), stride, p(ln), p(st), p(recv), F,
                                               p(rupto), p(dst)) == 0
            assert int((dst < 0).sum()) == 0
        torch.cuda.synchronize()
        wired.run_ticks(di[t:t + 1], rupto[None].clone(), recv)
    np.testing.assert_array_equal(rupto.cpu().numpy()[[hh for hh in range(P) if not (mask >> hh) & 1]],
                                  upto[-1][[hh for hh in range(P) if not (mask >> hh) & 1]])
    np.testing.assert_array_equal(wired.read_live(), direct.read_live())
    for x, y in zip(wired.read_cells(), direct.read_cells()):
        np.testing.assert_array_equal(x, y)
    assert wired.totals()[2] > 0  # rollbacks happened on the wire-fed batch too


def _encode_schedule(lib, P, S, T, mask, rd, upto, dr, stride, seed, max_redo=2):
    """Every tick's packets, encoded on the device ahead of the ticks: remote
    handle h sends frames acked+1 .. upto[t, h], acked = the frame it knows
    the receiver had one tick earlier minus 0-max_redo re-sent frames (an un-acked
    sender); [T, P, S, stride] packets and [T, P, S] lengths / start frames."""
    import ctypes

    import torch
    rng = np.random.default_rng(seed)
    F = dr.shape[0]
    pk = torch.zeros((T, P, S, stride), dtype=torch.uint8, device="cuda")
    ln = torch.zeros((T, P, S), dtype=torch.int32, device="cuda")
    st = torch.zeros((T, P, S), dtype=torch.int32, device="cuda")
    du = torch.from_numpy(upto).cuda()
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    for t in range(T):
        for h in range(P):
            if (mask >> h) & 1:
                continue
            prev = du[t - 1, h] if t > 0 else torch.full((S,), -1, dtype=torch.int32, device="cuda")
            redo = torch.from_numpy(rng.integers(0, max_redo + 1, S).astype(np.int32)).cuda()
            acked = torch.where(prev < 0, prev, torch.clamp(prev - redo, min=rd - 1))
            acked = torch.where(acked < rd, torch.full_like(acked, -1), acked).contiguous()
            newest = du[t, h].contiguous()
            assert lib.rb_encode_input_packets(0, None, h, P, S, 1, p(dr), F, rd, p(acked), p(newest), p(pk[t, h]),
                                               stride, p(ln[t, h]), p(st[t, h])) == 0
    torch.cuda.synchronize()
    assert int((ln < 0).sum()) == 0
    return pk, ln, st


@pytest.mark.gpu
@pytest.mark.parametrize("P,mask,rd,chunks", [(2, 0b01, 2, (1, 7, 30, 58)), (4, 0b0001, 1, (3, 1, 26, 66)),
                                              (3, 0b010, 0, (96,))])
def test_gpu_packet_ticks_equal_direct_delivery(gpu_available, P, mask, rd, chunks):
    # rb_p2p_run_ticks_packets decodes every endpoint's packet inside the tick's
    # poll (UdpProtocol::on_input fused into poll_remote_clients): fed the
    # packets of a delivery schedule (with re-sent frames), the batch ends
    # exactly where a batch fed the same deliveries directly does — cells,
    # states, and the acks equal the schedule's newest delivered frames —
    # over one-tick launches, HBM-cell multi-tick launches and LDS-ring ones.
    import torch

    import ggrs_amd as G
    from ggrs_amd import _lib as L
    from ggrs_amd.p2p import PlayerType, synth_network
    lib = L.load()
    S, W, T, stride = 512, 8, 96, 32
    inputs, upto, rin = synth_network(S, P, T, mask, rd, 1, 5)

    def batch():
        b = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
             .with_input_delay(1).with_remote_input_delay(rd))
        for hh in range(P):
            b.add_player(PlayerType.Local if (mask >> hh) & 1 else PlayerType.Remote, hh)
        return b.start_p2p_session()

    direct, wired = batch(), batch()
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    pk, ln, st = _encode_schedule(lib, P, S, T, mask, rd, upto, dr, stride, seed=5 + P)
    dstat = torch.zeros((P, S), dtype=torch.int32, device="cuda")
    acks = torch.full((P, S), -1, dtype=torch.int32, device="cuda")
    direct.run_ticks(di, du, dr)
    t = 0
    for n in chunks:
        wired.run_ticks_packets(di[t:t + n], pk[t:t + n], ln[t:t + n], st[t:t + n], dstat, acks)
        t += n
        torch.cuda.synchronize()
        assert int((dstat < 0).sum()) == 0
    assert t == T
    remotes = [hh for hh in range(P) if not (mask >> hh) & 1]
    np.testing.assert_array_equal(acks.cpu().numpy()[remotes], upto[-1][remotes])
    np.testing.assert_array_equal(wired.read_live(), direct.read_live())
    for x, y in zip(wired.read_cells(), direct.read_cells()):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(wired.read_queues(), direct.read_queues())
    assert wired.totals()[2] > 0 and wired.counters()[2] == 0


@pytest.mark.gpu
def test_gpu_malformed_packet_panics_only_its_session(gpu_available):
    # A packet the decoder cannot parse panics its session (the reference's
    # decode(...).expect("decoding failed"), protocol.rs:656); a packet that
    # skips frames never received is dropped (:639-642).  Every other session
    # runs on as if fed directly.
    import torch

    import ggrs_amd as G
    from ggrs_amd import _lib as L
    from ggrs_amd.p2p import PlayerType, synth_network
    lib = L.load()
    S, P, W, T, stride, mask, rd = 256, 2, 8, 40, 32, 0b01, 1
    inputs, upto, rin = synth_network(S, P, T, mask, rd, 1, 4)

    def batch():
        b = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
             .with_input_delay(1).with_remote_input_delay(rd))
        b.add_player(PlayerType.Local, 0)
        b.add_player(PlayerType.Remote, 1)
        return b.start_p2p_session()

    direct, wired = batch(), batch()
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    pk, ln, st = _encode_schedule(lib, P, S, T, mask, rd, upto, dr, stride, seed=9)
    bad_s, bad_t = 17, 20
    k = int(ln[bad_t, 1, bad_s])
    assert k > 0
    pk[bad_t, 1, bad_s, k - 1] |= 0x80  # the last byte now continues a varint: truncated
    dstat = torch.zeros((P, S), dtype=torch.int32, device="cuda")
    direct.run_ticks(di, du, dr)
    wired.run_ticks_packets(di[:bad_t], pk[:bad_t], ln[:bad_t], st[:bad_t], dstat)
    wired.run_ticks_packets(di[bad_t:bad_t + 1], pk[bad_t:bad_t + 1], ln[bad_t:bad_t + 1], st[bad_t:bad_t + 1], dstat)
    assert int(dstat[1, bad_s]) == -1
    wired.run_ticks_packets(di[bad_t + 1:], pk[bad_t + 1:], ln[bad_t + 1:], st[bad_t + 1:], dstat)
    status = wired.status()[0]
    assert status[bad_s] == 101 and wired.counters()[2] == 1
    ok = np.arange(S) != bad_s
    np.testing.assert_array_equal(wired.read_live()[ok], direct.read_live()[ok])
    with pytest.raises(G.InvalidRequest):  # packets need 16-byte rows of at least 32 bytes
        wired.run_ticks_packets(di[:1], pk[:1, :, :, :16], ln[:1], st[:1])


def _oracle_packet_deliveries(P, S, T, mask, W, F, pk, ln, st):
    """UdpProtocol::on_input (protocol.rs:616-689) restated on the host for every tick's packet
    of every remote endpoint (on_input_reference): per tick the receiver's newest frame per
    endpoint and its inputs by frame, exactly what the oracle's P2PSession is then delivered;
    plus the decode status per (tick, handle, session)."""
    pk_h, ln_h, st_h = pk.cpu().numpy(), ln.cpu().numpy(), st.cpu().numpy()
    recv = np.zeros((F, P, S), np.uint8)
    last = np.full((P, S), -1, np.int32)
    uptos = np.full((T, P, S), -1, np.int32)
    codes = np.ones((T, P, S), np.int32)
    recvs = []
    for t in range(T):
        for h in range(P):
            if (mask >> h) & 1:
                continue
            for s_ in range(S):
                n = int(ln_h[t, h, s_])
                start = int(st_h[t, h, s_])
                refin = bytes([recv[start - 1, h, s_]]) if start >= 1 else bytes(1)
                out, nl, code = on_input_reference(int(last[h, s_]), start, pk_h[t, h, s_, :n].tobytes(), refin, W, 1)
                codes[t, h, s_] = code
                for f, b in out.items():
                    recv[f, h, s_] = b[0]
                last[h, s_] = nl
        uptos[t] = last
        recvs.append(recv.copy())
    return uptos, recvs, codes


@pytest.mark.gpu
@pytest.mark.parametrize("P,mask,rd,W,stride,max_redo,chunks", [
    (2, 0b01, 2, 8, 32, 2, (1,) * 40 + (20, 20)),        # one-tick launches (live play), then multi-tick
    (4, 0b0001, 1, 8, 32, 2, (1,) * 30 + (26, 24)),
    (2, 0b01, 1, 15, 64, 28, (1,) * 50 + (30,)),        # long re-send windows: packets past 32 bytes, multi-segment
    (3, 0b010, 0, 16, 64, 30, (1,) * 20 + (60,)),        # W > 15: the general one-tick kernel
])
def test_gpu_packet_ticks_match_oracle_p2p(gpu_available, P, mask, rd, W, stride, max_redo, chunks):
    """rb_p2p_run_ticks_packets against the oracle, not against another device path: every
    packet is decoded on the host by UdpProtocol::on_input's restatement and delivered to the
    oracle's P2PSession (p2p_session.rs:253-371), the device decodes the same packets inside its
    ticks; statuses, rollback frames, request counts, decode statuses and acks must agree after
    every call, and cells, states and input queues after every call too."""
    import torch

    import ggrs_amd as G
    from ggrs_amd import _lib as L
    from ggrs_amd.p2p import PlayerType, synth_network
    from test_p2p import compare_state, drive_oracle  # noqa: F401  (the P2P parity helpers)
    lib = L.load()
    S = 192
    T = sum(chunks)
    inputs, upto, rin = synth_network(S, P, T, mask, rd, 1, 5)
    F = rin.shape[0]
    b = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
         .with_input_delay(1).with_remote_input_delay(rd))
    for hh in range(P):
        b.add_player(PlayerType.Local if (mask >> hh) & 1 else PlayerType.Remote, hh)
    wired = b.start_p2p_session()
    orc = O.OracleP2P(O.EX_GAME, P, W, 1, mask, S, sparse_saving=False, remote_delay=rd)
    di, dr = torch.from_numpy(inputs).cuda(), torch.from_numpy(rin).cuda()
    pk, ln, st = _encode_schedule(lib, P, S, T, mask, rd, upto, dr, stride, seed=11 + P, max_redo=max_redo)
    if max_redo > 20:
        assert int(ln.max()) > 32, "the schedule must produce packets past the 32-byte register window"
    uptos, recvs, codes = _oracle_packet_deliveries(P, S, T, mask, W, F, pk, ln, st)
    assert (codes >= 0).all()
    dstat = torch.zeros((P, S), dtype=torch.int32, device="cuda")
    acks = torch.full((P, S), -1, dtype=torch.int32, device="cuda")
    remotes = [hh for hh in range(P) if not (mask >> hh) & 1]
    t = 0
    for n in chunks:
        wired.run_ticks_packets(di[t:t + n], pk[t:t + n], ln[t:t + n], st[t:t + n], dstat, acks)
        for k in range(t, t + n):
            for hh in remotes:
                assert orc.deliver(hh, uptos[k, hh], recvs[k][:, hh, :]) == 0, orc.last_panic()
            for hh in range(P):
                if (mask >> hh) & 1:
                    assert orc.add_local_input(hh, inputs[k, hh]) == 0
            ost, olf, ona, ons = orc.advance()
        t += n
        st_, lf, na, ns = wired.status()
        np.testing.assert_array_equal(st_, ost, err_msg=f"status, tick {t - 1}")
        np.testing.assert_array_equal(lf, olf, err_msg=f"LoadGameState frame, tick {t - 1}")
        np.testing.assert_array_equal(na, ona, err_msg=f"AdvanceFrame count, tick {t - 1}")
        np.testing.assert_array_equal(ns, ons, err_msg=f"SaveGameState count, tick {t - 1}")
        np.testing.assert_array_equal(dstat.cpu().numpy()[remotes], codes[t - 1][remotes], err_msg=f"decode, tick {t - 1}")
        np.testing.assert_array_equal(acks.cpu().numpy()[remotes], uptos[t - 1][remotes], err_msg=f"acks, tick {t - 1}")
        if n > 1 or t % 10 == 0 or t == T:
            compare_state(wired, orc, t - 1)
    assert wired.totals()[2] > 0 and wired.counters()[2] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("ticks_per_call", [1, 30], ids=["live", "fused"])
def test_gpu_bad_packets_panic_like_the_reference(gpu_available, ticks_per_call):
    """Packets the reference would panic on panic exactly their own session: a packet whose
    start frame skips frames never received (assert!, protocol.rs:639-642), a length past the
    packet row (the row cannot hold the datagram), and a multi-segment packet longer than 32
    bytes whose last literal runs past its end (decode().expect, :656) — the general decoder,
    not the single-segment fast path.  Every other session equals a directly fed batch."""
    import torch

    import ggrs_amd as G
    from ggrs_amd import _lib as L
    from ggrs_amd.p2p import PlayerType, synth_network
    lib = L.load()
    S, P, W, T, stride, mask, rd = 256, 2, 8, 60, 64, 0b01, 1
    inputs, upto, rin = synth_network(S, P, T, mask, rd, 1, 4)

    def batch():
        b = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
             .with_input_delay(1).with_remote_input_delay(rd))
        b.add_player(PlayerType.Local, 0)
        b.add_player(PlayerType.Remote, 1)
        return b.start_p2p_session()

    direct, wired = batch(), batch()
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    pk, ln, st = _encode_schedule(lib, P, S, T, mask, rd, upto, dr, stride, seed=21)
    bad_t = 30
    gap_s, long_s, seg_s = 5, 77, 150
    for s_ in (gap_s, long_s, seg_s):
        assert int(ln[bad_t, 1, s_]) > 0
    st[bad_t, 1, gap_s] = upto[bad_t - 1, 1, gap_s] + 2  # skips the frame after the last one received
    ln[bad_t, 1, long_s] = stride + 1                     # longer than its row
    # literal(10) + run + literal claiming 40 bytes with 20 present: 33 bytes, malformed
    body = [10 << 1] + list(range(1, 11)) + [(4 << 2) | 1] + [40 << 1] + list(range(20))
    assert len(body) == 33
    pk[bad_t, 1, seg_s, :] = 0
    pk[bad_t, 1, seg_s, :len(body)] = torch.tensor(body, dtype=torch.uint8)
    ln[bad_t, 1, seg_s] = len(body)
    assert O.wire_decode(bytes(1), bytes(body)) is None
    dstat = torch.zeros((P, S), dtype=torch.int32, device="cuda")
    direct.run_ticks(di, du, dr)
    t = 0
    while t < T:
        n = min(ticks_per_call, T - t)
        wired.run_ticks_packets(di[t:t + n], pk[t:t + n], ln[t:t + n], st[t:t + n], dstat)
        t += n
    # a session stops at its panic: its decode status stays the panicking tick's
    d = dstat.cpu().numpy()[1]
    assert d[gap_s] == -2 and d[long_s] == -1 and d[seg_s] == -1, (d[gap_s], d[long_s], d[seg_s])
    status = wired.status()[0]
    dead = np.zeros(S, bool)
    dead[[gap_s, long_s, seg_s]] = True
    assert (status[dead] == 101).all() and wired.counters()[2] == 3
    np.testing.assert_array_equal(wired.read_live()[~dead], direct.read_live()[~dead])
