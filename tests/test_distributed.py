"""N>1 path on CPU: world size 2 over gloo (the GPU runs use nccl = RCCL).

Each rank owns a contiguous shard of global sessions (ggrs_amd.shard), drives
its own batch with no data-path collective, and all-gathers the per-session
desync reports (rb_checksum_report) every interval.  The CPU stand-in for a
rank's device batch is the oracle (test infrastructure) for values and a
plan-only product batch (device=-1) for the request stream; the gathered
reports must equal a single-process run over every session, and a snapshot
corrupted on rank 1 must be visible to rank 0 at its global session id.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ggrs_amd as G
from ggrs_amd import shard
from oracle import oracle as O

TOTAL, P, CD, DELAY, T, INTERVAL = 24, 2, 7, 2, 40, 10
VICTIM = 17  # global session id, owned by rank 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _reports_for(orc, frame):
    frames, _, _, cs = orc.read_cells()
    w = int(np.nonzero(frames == frame)[0][0])
    k, f = orc.last_errors
    return shard.pack_reports(cs[w], frame, np.where(k == 3, f, -1).astype(np.int32))


def _drive(orc, plan, inputs, t, victim_local):
    if t == 15 and victim_local is not None:
        f = orc.current_frame() - CD
        orc.corrupt_cell(victim_local, f, 0, 0x100)
    for h in range(P):
        orc.add_local_input(h, inputs[t, h])
        if plan is not None:
            plan.add_local_input(h, inputs[t, h])
    orc.last_errors = orc.advance()
    if plan is not None:
        reqs = plan.advance_frame()
        if (orc.last_errors[0] == 0).all():
            assert [(int(r.kind), r.frame) for r in reqs] == orc.trace(0)


def _compact_for(orc, frame):
    frames, _, _, cs = orc.read_cells()
    w = int(np.nonzero(frames == frame)[0][0])
    k, f = orc.last_errors
    return shard.pack_compact(cs[w][:, 0], frame, np.where(k == 3, f, -1).astype(np.int32))


def _rank_main(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard.shard_range(rank, world, TOTAL)
        inputs = G.synth_inputs(hi - lo, P, T, first_session=lo)
        full = G.synth_inputs(TOTAL, P, T)
        assert np.array_equal(inputs, full[:, :, lo:hi])  # inputs keyed by global session id
        orc = O.OracleBatch(O.EX_GAME, P, 8, CD, DELAY, hi - lo)
        plan = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=hi - lo, device=-1).with_num_players(P)
                .with_check_distance(CD).with_input_delay(DELAY).start_synctest_session())
        victim = VICTIM - lo if lo <= VICTIM < hi else None
        gathered_all, compact_all = [], []
        for t in range(T):
            _drive(orc, plan, inputs, t, victim)
            if orc.current_frame() % INTERVAL == 0:
                rep = _reports_for(orc, orc.current_frame() - 1)
                local = torch.from_numpy(rep.view(np.int64).reshape(-1, shard.REPORT_WORDS).copy())
                g = shard.gather_reports(local)
                gathered_all.append(g.numpy())
                bad = shard.desynced_sessions(g).tolist()
                assert bad == ([VICTIM] if t >= 15 else []), (t, bad)
                # the compact form (rb_export_compact_report): 4 B per session, same verdict
                c = shard.gather_compact(torch.from_numpy(_compact_for(orc, orc.current_frame() - 1)))
                compact_all.append(c.numpy())
                assert int(shard.count_desynced_compact(c)) == (1 if t >= 15 else 0)
                assert ((c.numpy() < 0).nonzero()[0].tolist()) == ([VICTIM] if t >= 15 else [])
        np.save(os.path.join(outdir, f"rank{rank}.npy"), np.stack(gathered_all))
        np.save(os.path.join(outdir, f"compact{rank}.npy"), np.stack(compact_all))
    finally:
        dist.destroy_process_group()


def test_shard_ranges_partition_the_batch():
    for total, world in [(24, 2), (65536 * 8, 8), (10, 3), (1, 1)]:
        rs = [shard.shard_range(r, world, total) for r in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == total
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    with pytest.raises(ValueError):
        shard.shard_range(2, 2, 10)


def test_report_layout_matches_abi():
    from ggrs_amd import _lib as L
    import ctypes
    assert shard.REPORT_DTYPE.itemsize == ctypes.sizeof(L.RbChecksumReport) == 24
    r = shard.pack_reports(np.array([[5, 7]], np.uint64), 42, np.array([-1], np.int32))
    w = r.view(np.int64)
    assert w[0] == 5 and w[1] == 7 and (w[2] >> 32) == -1 and (w[2] & 0xFFFFFFFF) == 42


def test_compact_report_layout():
    # rb_export_compact_report's record: checksum in bits 0-15, frames since the mismatch in 16-30
    # (saturated), the MismatchedChecksum flag in bit 31
    r = shard.pack_compact(np.array([0xBEEF, 0x1234, 7, 9], np.uint64), 100,
                           np.array([-1, 97, 100, -50000], np.int32)).view(np.uint32)
    assert r[0] == 0xBEEF
    assert r[1] == 0x80000000 | (3 << 16) | 0x1234
    assert r[2] == 0x80000000 | 7
    assert r[3] == 0x80000000 | (0x7FFF << 16) | 9


def test_audit_compare_compact_finds_the_corrupted_replica():
    world, owned, audit = 3, 8, 4
    rows = np.arange(world * (owned + audit), dtype=np.int32).reshape(world, owned + audit)
    for r in range(world):  # each rank's replicas = the next rank's first `audit` owned records
        rows[r, owned:] = rows[(r + 1) % world, :audit]
    g = torch.from_numpy(rows.reshape(-1).copy())
    assert int(shard.audit_compare_compact(g, world, owned, audit)) == 0
    rows[1, owned + 2] ^= 1  # rank 1's replica of rank 2's session 2
    assert int(shard.audit_compare_compact(torch.from_numpy(rows.reshape(-1).copy()), world, owned, audit)) == 1
    rows[0, 3] |= np.int32(-2 ** 31)  # a mismatch flag on an owned session
    assert int(shard.count_desynced_compact(torch.from_numpy(rows.reshape(-1).copy()), world, owned, audit)) == 1


def test_two_rank_gloo_report_allgather_equals_single_process():
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_main, args=(2, port, d), nprocs=2, join=True)
        r0 = np.load(os.path.join(d, "rank0.npy"))
        r1 = np.load(os.path.join(d, "rank1.npy"))
        c0 = np.load(os.path.join(d, "compact0.npy"))
        c1 = np.load(os.path.join(d, "compact1.npy"))
    np.testing.assert_array_equal(r0, r1)  # every rank sees the same node-wide reports
    np.testing.assert_array_equal(c0, c1)
    # the compact records carry exactly the full reports' low 16 checksum bits and mismatch flag
    lo16 = (r0[..., 0] & 0xFFFF).astype(np.int64)
    flag = (r0[..., 2] >> 32) != -1
    np.testing.assert_array_equal(c0.astype(np.int64) & 0xFFFF, lo16)
    np.testing.assert_array_equal(c0 < 0, flag)
    # single process over all sessions
    orc = O.OracleBatch(O.EX_GAME, P, 8, CD, DELAY, TOTAL)
    inputs = G.synth_inputs(TOTAL, P, T)
    ref = []
    for t in range(T):
        _drive(orc, None, inputs, t, VICTIM)
        if orc.current_frame() % INTERVAL == 0:
            ref.append(_reports_for(orc, orc.current_frame() - 1).view(np.int64).reshape(-1, shard.REPORT_WORDS))
    np.testing.assert_array_equal(r0, np.stack(ref))


def test_p2p_network_shards_are_slices_of_the_global_network():
    # bench.py --session p2p on N ranks: rank r generates its sessions
    # [g0, g1) with first_session = g0.  Weak scaling is only honest if those
    # shards are exactly the columns of the single-process network, and the
    # oracle's rollback on a shard equals its rollback on the same columns of
    # the whole batch (sessions never interact).
    from ggrs_amd.p2p import synth_network
    S, P, T, mask, world = 48, 2, 40, 0b01, 2
    full = synth_network(S, P, T, mask, 2, 1, 5)
    for rank in range(world):
        g0, g1 = shard.shard_range(rank, world, S)
        part = synth_network(g1 - g0, P, T, mask, 2, 1, 5, first_session=g0)
        for a, b in zip(full, part):
            np.testing.assert_array_equal(a[..., g0:g1], b)
    whole = O.OracleP2P(O.EX_GAME, P, 8, 2, mask, S, remote_delay=2)
    half = O.OracleP2P(O.EX_GAME, P, 8, 2, mask, S // 2, remote_delay=2)
    inputs, upto, rin = full
    for t in range(T):
        for orc, cols in ((whole, slice(0, S)), (half, slice(S // 2, S))):
            orc.deliver(1, upto[t, 1, cols], rin[:, 1, cols])
            orc.add_local_input(0, inputs[t, 0, cols])
            st = orc.advance()[0]
            assert (st == 0).all()
    np.testing.assert_array_equal(whole.read_live()[0][S // 2:], half.read_live()[0])


def test_audit_compare_finds_exactly_the_corrupted_replica():
    # rank r's batch = `owned` sessions + `audit` replicas of rank (r+1)'s first sessions
    world, owned, audit = 3, 5, 2
    gid = np.concatenate([np.concatenate([np.arange(r * owned, (r + 1) * owned),
                                          np.arange(((r + 1) % world) * owned, ((r + 1) % world) * owned + audit)])
                          for r in range(world)]).astype(np.uint64)
    cs = gid * np.uint64(1000003) + np.uint64(7)
    rep = shard.pack_reports(np.stack([cs, cs ^ np.uint64(5)], 1), 41, np.full(gid.size, -1, np.int32))
    g = torch.from_numpy(rep.view(np.int64).reshape(-1, shard.REPORT_WORDS).copy())
    n, detail = shard.audit_compare(g, world, owned, audit)
    assert int(n) == 0 and detail.shape == (0, 4)
    # rank 2's replica of rank 0's session 1 (global 1) disagrees with its owner
    g2 = g.clone()
    g2[2 * (owned + audit) + owned + 1, 1] ^= 1  # high checksum word
    n, detail = shard.audit_compare(g2, world, owned, audit)
    assert int(shard.audit_compare(g2, world, owned, audit, detail=False)[0]) == int(n)  # the bench's count-only form
    assert int(n) == 1
    assert detail.tolist() == [[1, 41, int(g[1, 0]), int(g[1, 0])]]
    # owned-row helpers skip the replicas
    assert shard.owned_rows(g, world, owned, audit).shape == (world * owned, shard.REPORT_WORDS)
    g3 = g.clone()
    g3[owned, 2] = (g3[owned, 2] & 0xFFFFFFFF) | (7 << 32)  # a replica row carrying a mismatch flag: not owned
    assert int(shard.count_desynced(g3, world, owned, audit)) == 0
    g3[owned - 1, 2] = (g3[owned - 1, 2] & 0xFFFFFFFF) | (7 << 32)
    assert shard.desynced_sessions(g3, world, owned, audit).tolist() == [owned - 1]


def _bench_rehearsal(n, corrupt):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GGRS_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    if corrupt:
        env["GGRS_REHEARSAL_CORRUPT"] = "1"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n), "--rehearsal", "--steps",
                        "20", "--warmup", "5", "--report-interval", "10"], env=env, cwd=root, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_self_launches_ranks_from_a_bare_shell():
    # bench.py --gpus 2 with no outside launcher: the parent starts the rank
    # processes (gloo here, RCCL on the GPU box), rank 0 prints one line
    d = _bench_rehearsal(2, corrupt=False)
    rep = d["config"]["desync_reports"]
    assert d["n_gpus"] == 2 and rep["ranks"] == 2 and rep["backend"] == "gloo"
    # 33 ticks (8 start-up + 5 warmup + 20 timed), a report every 10 frames
    assert rep["gathers"] == 3 and rep["audit_compared"] == 3 * 2 * 64 and rep["audit_desynced"] == 0


def test_bench_rehearsal_audit_reports_an_injected_desync():
    d = _bench_rehearsal(3, corrupt=True)
    rep = d["config"]["desync_reports"]
    assert rep["ranks"] == 3 and rep["audit_desynced"] == 1
    assert rep["first_desync"][:2] == [256, 9]  # rank 0's replica of global session 256 (rank 1's first), frame 9


def _p2p_peer_rank(rank, world, port, outdir):
    # rank 0 holds peer A (handle 0 local) of every session, rank 1 peer B:
    # the two views of the same sessions on two ranks, their ChecksumReports
    # exchanged by the all-gather every tick.  Rank 0 flips three sessions.
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ggrs_amd.p2p import synth_network
        S, P2, T, d, interval = 32, 2, 90, 2, 10
        mask = 0b01 if rank == 0 else 0b10
        inputs, upto, rin = synth_network(S, P2, T, mask, d, 0, 1)
        orc = O.OracleP2P(O.EX_GAME, P2, 8, d, mask, S, remote_delay=d)
        orc.set_desync_detection(interval)
        remote = 1 - rank  # this peer's remote handle = the other rank's local one
        for t in range(T):
            if t == 41 and rank == 0:
                for s in (4, 19, 30):
                    orc.corrupt(s, 4 * P2, 0x00100000)
            orc.deliver(remote, upto[t, remote], rin[:, remote, :])
            orc.add_local_input(rank, inputs[t, rank])
            assert (orc.advance()[0] == 0).all()
            fr, cs = orc.take_checksum_reports(8)
            g = shard.exchange_checksum_reports(torch.from_numpy(shard.p2p_reports_to_rows(fr, cs)))
            pf, pc = shard.p2p_rows_to_reports(g[1 - rank].numpy())
            assert orc.receive_checksum_reports(remote, pf, pc) == 0
        n, fr, hd, lo, ro = orc.desync_events()
        np.save(os.path.join(outdir, f"events{rank}.npy"), n)
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_p2p_checksum_exchange_detects_desync():
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_p2p_peer_rank, args=(2, port, d), nprocs=2, join=True)
        n0 = np.load(os.path.join(d, "events0.npy"))
        n1 = np.load(os.path.join(d, "events1.npy"))
    # both peers raise DesyncDetected on exactly the flipped sessions
    assert np.nonzero(n0)[0].tolist() == [4, 19, 30]
    assert np.nonzero(n1)[0].tolist() == [4, 19, 30]
