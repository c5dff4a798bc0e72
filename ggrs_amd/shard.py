"""Multi-GPU session sharding and the desync-report all-gather.

Sessions are independent (no cross-session state anywhere in SyncLayer /
SyncTestSession), so each rank owns a contiguous range of global session ids
and runs its own batch with no data-path collective.  The only exchange is the
per-session desync report that mirrors P2P ``ChecksumReport{checksum, frame}``
(/root/reference/src/network/messages.rs:75-79) plus the session's
``MismatchedChecksum`` flag, all-gathered every ``interval`` frames like
``check_checksum_send_interval`` / ``compare_local_checksums_against_peers``
(src/sessions/p2p_session.rs:873-928).  With the ``nccl`` backend this is one
RCCL all-gather over xGMI; ``gloo`` serves the CPU tests.
"""
from __future__ import annotations

import numpy as np

NULL_FRAME = -1

# rb_checksum_report (include/ggrs_amd.h): u64 lo, u64 hi, i32 frame, i32 mismatch_frame = 24 B
REPORT_DTYPE = np.dtype([("checksum_lo", "<u8"), ("checksum_hi", "<u8"), ("frame", "<i4"),
                         ("mismatch_frame", "<i4")])
REPORT_WORDS = REPORT_DTYPE.itemsize // 8  # as int64 words for collectives


def shard_range(rank: int, world: int, total_sessions: int):
    """Global session ids [lo, hi) owned by ``rank`` (contiguous, balanced)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return total_sessions * rank // world, total_sessions * (rank + 1) // world


def pack_reports(checksums_u128: np.ndarray, frame: int, mismatch_frames: np.ndarray) -> np.ndarray:
    """Host-side construction of [S] reports (what rb_export_checksum_report writes
    on the device): checksums [S, 2] u64 (lo, hi), mismatch frames [S] i32."""
    r = np.zeros(mismatch_frames.shape[0], REPORT_DTYPE)
    r["checksum_lo"] = checksums_u128[:, 0]
    r["checksum_hi"] = checksums_u128[:, 1]
    r["frame"] = frame
    r["mismatch_frame"] = mismatch_frames
    return r


def gather_reports(local, group=None):
    """All-gather [S, 3] int64 report tensors (one rb_checksum_report per row) from
    every rank; returns [world * S, 3] in rank order (= global session order)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world * local.shape[0], local.shape[1]), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local, group=group)  # RCCL all-gather over xGMI
    else:
        parts = list(out.chunk(world))
        dist.all_gather(parts, local, group=group)
        out = torch.cat(parts)
    return out


def owned_rows(gathered, world: int = 1, owned: int = 0, audit: int = 0):
    """The rows of owned sessions, in global session order: every rank's batch is
    ``owned`` sessions followed by ``audit`` replicas (audit_compare)."""
    if not audit:
        return gathered
    return gathered.view(world, owned + audit, -1)[:, :owned].reshape(world * owned, -1)


def desynced_sessions(gathered, world: int = 1, owned: int = 0, audit: int = 0):
    """Global ids of sessions whose report carries a mismatch frame (as a tensor)."""
    rows = owned_rows(gathered, world, owned, audit)
    mismatch = rows[:, 2] >> 32  # high half of the last word = mismatch_frame (little endian)
    return (mismatch != NULL_FRAME).nonzero().flatten()


def count_desynced(gathered, world: int = 1, owned: int = 0, audit: int = 0):
    return ((owned_rows(gathered, world, owned, audit)[:, 2] >> 32) != NULL_FRAME).sum()


def audit_compare(gathered, world: int, owned: int, audit: int, detail: bool = True):
    """Cross-GPU desync detection over the all-gathered reports.

    Rank r's batch holds its ``owned`` sessions and, after them, ``audit``
    replicas of the first ``audit`` sessions of rank (r+1) % world: the same
    session simulated independently on two GPUs, like the two peers of a P2P
    session.  Their ChecksumReports must agree; where they do not, that is the
    reference's DesyncDetected{frame, local_checksum, remote_checksum}
    (compare_local_checksums_against_peers, p2p_session.rs:873-898), with the
    owner as "local".  Returns (count, [k, 4] int64 tensor of (global session
    id, frame, owner checksum lo, replica checksum lo)) — the count as a tensor,
    so the call does not synchronise.  detail=False skips the list (its nonzero()
    synchronises the host with the device) and returns (count, None): the
    bench's timed loop only adds the count up."""
    import torch
    if world < 2 or audit <= 0:
        z = torch.zeros((), dtype=torch.int64, device=gathered.device)
        return z, torch.zeros((0, 4), dtype=torch.int64, device=gathered.device)
    rows = gathered.view(world, owned + audit, -1)
    replica = rows[:, owned:owned + audit]  # rank r's replicas of rank r+1's first sessions
    owner = torch.roll(rows[:, :audit], shifts=-1, dims=0)  # row r = rank r+1's own reports
    frame = lambda x: x[..., 2] & 0xFFFFFFFF
    bad = (replica[..., 0] != owner[..., 0]) | (replica[..., 1] != owner[..., 1]) | (frame(replica) != frame(owner))
    if not detail:
        return bad.sum(), None
    idx = bad.nonzero()
    sid = ((idx[:, 0] + 1) % world) * owned + idx[:, 1]
    own = owner[idx[:, 0], idx[:, 1]]
    rep = replica[idx[:, 0], idx[:, 1]]
    detail = torch.stack([sid, frame(own), own[:, 0], rep[:, 0]], 1) if idx.numel() else \
        torch.zeros((0, 4), dtype=torch.int64, device=gathered.device)
    return bad.sum(), detail


# ---------------------------------------------------------------------------- compact reports (4 B)
# rb_export_compact_report: one uint32 per session, for 16-bit checksums (ex_game's fletcher16, the
# brawler's): bits 0-15 the checksum, 16-30 the frames since the MismatchedChecksum (saturated),
# bit 31 the mismatch flag.  The report frame is batch-uniform (every rank reports the same tick),
# so it is not repeated per session: 4 B instead of 24 per session and all-gather.
COMPACT_MISMATCH = 1 << 31


def pack_compact(checksums16: np.ndarray, frame: int, mismatch_frames: np.ndarray) -> np.ndarray:
    """Host mirror of rb_export_compact_report: [S] int32 records (the bit pattern of the uint32s)."""
    r = checksums16.astype(np.uint32) & np.uint32(0xFFFF)
    bad = mismatch_frames != NULL_FRAME
    delta = np.clip(frame - mismatch_frames.astype(np.int64), 0, 0x7FFF).astype(np.uint32)
    r = np.where(bad, r | np.uint32(COMPACT_MISMATCH) | (delta << np.uint32(16)), r)
    return r.astype(np.uint32).view(np.int32)


def gather_compact(local, group=None):
    """All-gather [S] int32 compact reports from every rank: [world * S] in rank order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world * local.shape[0],), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local, group=group)  # RCCL all-gather over xGMI
    else:
        parts = list(out.chunk(world))
        dist.all_gather(parts, local, group=group)
        out = torch.cat(parts)
    return out


def _owned_compact(gathered, world, owned, audit):
    if not audit:
        return gathered
    return gathered.view(world, owned + audit)[:, :owned].reshape(-1)


def count_desynced_compact(gathered, world: int = 1, owned: int = 0, audit: int = 0):
    """Sessions reporting MismatchedChecksum (bit 31 set: negative as int32)."""
    return (_owned_compact(gathered, world, owned, audit) < 0).sum()


def audit_compare_compact(gathered, world: int, owned: int, audit: int):
    """audit_compare over compact reports: owner and replica records must be equal (checksum,
    mismatch flag and delta); returns the count of disagreeing replicas as a tensor."""
    import torch
    if world < 2 or audit <= 0:
        return torch.zeros((), dtype=torch.int64, device=gathered.device)
    rows = gathered.view(world, owned + audit)
    replica = rows[:, owned:owned + audit]
    owner = torch.roll(rows[:, :audit], shifts=-1, dims=0)
    return (replica != owner).sum()


# ---------------------------------------------------------------------------- P2P ChecksumReports
def p2p_reports_to_rows(frames: np.ndarray, checksums: np.ndarray) -> np.ndarray:
    """[K, S] frames + [K, S, 2] u128 (lo, hi) -> [K, S, 3] int64 rows in the
    rb_checksum_report layout rb_p2p_take_checksum_reports writes."""
    r = np.zeros(frames.shape, REPORT_DTYPE)
    r["checksum_lo"] = checksums[..., 0]
    r["checksum_hi"] = checksums[..., 1]
    r["frame"] = frames
    r["mismatch_frame"] = NULL_FRAME
    return r.view(np.int64).reshape(frames.shape + (REPORT_WORDS,))


def p2p_rows_to_reports(rows: np.ndarray):
    """Inverse of p2p_reports_to_rows: (frames [K, S] i32, checksums [K, S, 2] u64)."""
    r = np.ascontiguousarray(rows).reshape(-1, REPORT_WORDS).view(REPORT_DTYPE).reshape(rows.shape[:-1])
    return r["frame"].copy(), np.stack([r["checksum_lo"], r["checksum_hi"]], -1)


def exchange_checksum_reports(local, group=None):
    """The ChecksumReport exchange of P2P desync detection on one node: every
    rank contributes the [K, S, 3] reports its peers' batch sent this tick
    (rb_p2p_take_checksum_reports) and receives everybody's as [world, K, S, 3];
    a rank holding peer B of a session hands rank(peer A)'s slice to
    rb_p2p_receive_checksum_reports.  One RCCL all-gather over xGMI (gloo on
    the CPU tests) replaces the datagrams UdpProtocol::send_checksum_report
    sends (protocol.rs:736-742)."""
    flat = local.reshape(-1, local.shape[-1])
    g = gather_reports(flat.contiguous(), group)
    import torch.distributed as dist
    return g.view((dist.get_world_size(group),) + tuple(local.shape))

