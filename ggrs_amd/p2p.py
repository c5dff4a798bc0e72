"""P2PSession batches over the C ABI (include/ggrs_amd.h rb_p2p_*).

Mirrors sessions/p2p_session.rs for ``num_sessions`` independent sessions seen
from one peer.  The network layer is the caller's: per tick it hands over, for
every remote handle, the newest delivered frame and the inputs by frame — what
UdpProtocol's Event::Input stream (p2p_session.rs:838-852) carries.  Built by
``SessionBuilder.add_player(...).start_p2p_session()`` (builder.rs:251-308).

``synth_network`` produces a deterministic synthetic delivery schedule (per
session latency + jitter) for tests and the bench.
"""
from __future__ import annotations

import ctypes
import enum

import numpy as np

from . import _lib as L
from .session import DeviceError, InvalidRequest, Panic, _StreamOrdered, input_dtype
from .synth import SEED, splitmix64


class PlayerType(enum.Enum):  # lib.rs:115-124 (Spectator is not part of the batch)
    Local = "local"
    Remote = "remote"


def _dev_ptr(x):
    """(pointer, keepalive) of a torch CUDA tensor."""
    import torch
    if not isinstance(x, torch.Tensor) or not x.is_cuda:
        raise TypeError("P2P tensors must be torch CUDA tensors (device memory, stream ordered)")
    x = x.contiguous()
    return ctypes.c_void_p(x.data_ptr()), x


class P2PSession(_StreamOrdered):
    """p2p_session.rs:116-929 (rollback path) for ``num_sessions`` sessions.

    Device work runs on the batch's own HIP stream (or the one set_stream
    chose) and is ordered against torch's current stream at every call
    (_StreamOrdered): inputs made on torch's stream are complete before a
    launch reads them, and tensors a call writes (checksum reports) are
    complete before later torch work on the current stream reads them."""

    def __init__(self, lib, handle, game, cfg):
        self._lib = lib
        self._h = handle
        self.game = game
        self.num_sessions = int(cfg.num_sessions)
        self.num_players = int(cfg.num_players)
        self.max_prediction = int(cfg.max_prediction)
        self.input_delay = int(cfg.input_delay)
        self.remote_delay = int(cfg.remote_delay)
        self.sparse_saving = bool(cfg.sparse_saving)
        self.local_mask = int(cfg.local_mask)
        self.desync_interval = int(cfg.desync_interval)
        self.state_bytes = lib.rb_p2p_state_bytes(handle)
        self.input_dtype = input_dtype(game, lib.rb_p2p_input_bytes(handle))
        self._device = int(cfg.device)
        self._bind(self._device, lib.rb_p2p_get_stream(handle) or 0)

    def close(self):
        if self._h:
            self._lib.rb_p2p_destroy(self._h)  # synchronises the batch stream first
            self._h = None
            self._stream = None
            self._drain()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        if st != L.RB_OK:
            msg = (self._lib.rb_p2p_last_error(self._h) or b"").decode()
            if st == L.RB_INVALID_REQUEST:
                raise InvalidRequest(msg)
            raise DeviceError(msg) if st == L.RB_DEVICE_ERROR else Panic(msg)

    def local_player_handles(self):  # p2p_session.rs:416-419
        return [h for h in range(self.num_players) if (self.local_mask >> h) & 1]

    def remote_player_handles(self):  # :421-424
        return [h for h in range(self.num_players) if not (self.local_mask >> h) & 1]

    def set_stream(self, stream) -> None:
        self._check(self._lib.rb_p2p_set_stream(self._h, ctypes.c_void_p(stream.cuda_stream if stream else 0)))
        self._bind(self._device, self._lib.rb_p2p_get_stream(self._h) or 0)

    def fanout_state(self):
        """The adaptive fan-out (rb_p2p_fanout_state): (active, select fraction of the last
        measured window or -1, windows measured, times turned off)."""
        a, w, o = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        f = ctypes.c_double()
        self._check(self._lib.rb_p2p_fanout_state(self._h, ctypes.byref(a), ctypes.byref(f), ctypes.byref(w),
                                                  ctypes.byref(o)))
        return bool(a.value), f.value, w.value, o.value

    def run_ticks(self, local_inputs, remote_upto, remote_inputs) -> None:
        """T ticks: [poll_remote_clients, add_local_input for every local handle,
        advance_frame, handle_requests] x T in one device launch.

        local_inputs  [T, P, S] Input values (remote handles' rows ignored)
        remote_upto   [T, P, S] int32 newest delivered frame per remote handle
        remote_inputs [F, P, S] Input values by frame (local handles' rows ignored)
        All torch CUDA tensors on the batch's device."""
        T = int(local_inputs.shape[0])
        assert tuple(local_inputs.shape[1:]) == (self.num_players, self.num_sessions)
        assert tuple(remote_upto.shape) == (T, self.num_players, self.num_sessions)
        assert tuple(remote_inputs.shape[1:]) == (self.num_players, self.num_sessions)
        lp, lk = _dev_ptr(local_inputs)
        up, uk = _dev_ptr(remote_upto)
        rp, rk = _dev_ptr(remote_inputs)
        cur = self._pre()
        stride = self.num_players * self.num_sessions * lk.element_size()
        self._check(self._lib.rb_p2p_run_ticks(self._h, T, lp, stride, up, rp, int(remote_inputs.shape[0])))
        self._post(cur, (lk, uk, rk))

    def run_ticks_packets(self, local_inputs, packets, lengths, start_frames, decode_status=None, acks=None) -> None:
        """T ticks fed by the peers' input packets (rb_p2p_run_ticks_packets):
        each tick decodes every remote endpoint's packet inside its poll
        (UdpProtocol::on_input), then runs as run_ticks.

        local_inputs  [T, P, S] Input values (remote handles' rows ignored)
        packets       [T, P, S, stride] uint8 (stride a multiple of 16, >= 32)
        lengths, start_frames [T, P, S] int32 (length 0: no packet)
        decode_status, acks   None or [P, S] int32 outputs: the last tick's decode
                      result per endpoint, the newest frame received per endpoint"""
        import torch
        T = int(local_inputs.shape[0])
        assert tuple(local_inputs.shape[1:]) == (self.num_players, self.num_sessions)
        assert tuple(packets.shape[:3]) == (T, self.num_players, self.num_sessions) and packets.dim() == 4
        assert tuple(lengths.shape) == tuple(start_frames.shape) == (T, self.num_players, self.num_sessions)
        # the kernel reads packets as bytes and lengths / start frames as int32, and writes int32 outputs
        assert packets.dtype == torch.uint8, "packets must be uint8 (the row stride is a byte count)"
        assert lengths.dtype == start_frames.dtype == torch.int32, "lengths and start_frames must be int32"
        for o in (decode_status, acks):
            assert o is None or o.dtype == torch.int32, "decode_status / acks must be int32"
        lp, lk = _dev_ptr(local_inputs)
        pp, pk = _dev_ptr(packets)
        np_, nk = _dev_ptr(lengths)
        sp, sk = _dev_ptr(start_frames)
        keep = [lk, pk, nk, sk]
        outs = []
        for o in (decode_status, acks):
            if o is None:
                outs.append(None)
            else:
                assert tuple(o.shape) == (self.num_players, self.num_sessions) and o.is_contiguous()
                op, ok = _dev_ptr(o)
                outs.append(op)
                keep.append(ok)
        cur = self._pre()
        stride = self.num_players * self.num_sessions * lk.element_size()
        self._check(self._lib.rb_p2p_run_ticks_packets(self._h, T, lp, stride, pp, int(packets.shape[3]), np_, sp,
                                                       outs[0], outs[1]))
        self._post(cur, tuple(keep), outputs=decode_status is not None or acks is not None)

    def disconnect_player(self, handle: int, sessions=None) -> None:
        """P2PSession::disconnect_player(handle) (p2p_session.rs:430-456) in every
        session where `sessions` is true (None: all), between ticks.  Raises
        InvalidRequest like the reference (invalid handle, local player, already
        disconnected) and then applies nothing."""
        m = None
        if sessions is not None:
            m = np.ascontiguousarray(np.broadcast_to(np.asarray(sessions), (self.num_sessions,)), dtype=np.uint8)
        st = self._lib.rb_p2p_disconnect_player(self._h, int(handle),
                                               None if m is None else m.ctypes.data_as(ctypes.c_void_p))
        if st == L.RB_INVALID_REQUEST:
            raise InvalidRequest((self._lib.rb_p2p_last_error(self._h) or b"").decode())
        self._check(st)

    def advance_frame(self, local_inputs, remote_upto, remote_inputs) -> None:
        """One tick (run_ticks with T = 1): local_inputs [P, S], remote_upto [P, S]."""
        self.run_ticks(local_inputs[None], remote_upto[None], remote_inputs)

    def status(self):
        """(rb_status [S], LoadGameState frame [S] (NULL_FRAME = no rollback),
        AdvanceFrame count [S], SaveGameState count [S]) of the last tick."""
        st, lf, na, ns = (np.empty(self.num_sessions, np.int32) for _ in range(4))
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        self._check(self._lib.rb_p2p_read_status(self._h, p(st), p(lf), p(na), p(ns)))
        return st, lf, na, ns

    def frames(self):
        """(current_frame [S], last confirmed frame [S])."""
        c = np.empty(self.num_sessions, np.int32)
        k = np.empty(self.num_sessions, np.int32)
        self._check(self._lib.rb_p2p_read_frames(self._h, c.ctypes.data_as(ctypes.c_void_p),
                                                 k.ctypes.data_as(ctypes.c_void_p)))
        return c, k

    def read_queues(self):
        """InputQueue / ConnectionStatus bookkeeping [S, P, 8]: last_added_frame, inputs[tail].frame,
        length, last_requested_frame, prediction.frame, first_incorrect_frame, connect-status
        last_frame, disconnected (input_queue.rs:12-34, messages.rs:5-18)."""
        out = np.empty((self.num_sessions, self.num_players, 8), np.int32)
        self._check(self._lib.rb_p2p_read_queues(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def read_cells(self):
        """(frame tags [W, S], images [W, S, B], checksums [W, S, 2])."""
        W, S = self.max_prediction, self.num_sessions
        tags = np.empty((W, S), np.int32)
        img = np.zeros((W, S, self.state_bytes), np.uint8)
        cs = np.zeros((W, S, 2), np.uint64)
        self._check(self._lib.rb_p2p_read_cells(self._h, tags.ctypes.data_as(ctypes.c_void_p),
                                                img.ctypes.data_as(ctypes.c_void_p), cs.ctypes.data_as(ctypes.c_void_p)))
        return tags, img, cs

    def read_live(self):
        img = np.zeros((self.num_sessions, self.state_bytes), np.uint8)
        self._check(self._lib.rb_p2p_read_live(self._h, img.ctypes.data_as(ctypes.c_void_p)))
        return img

    def counters(self):
        """(PredictionThreshold hits, unexpected math paths, panicked sessions) since create."""
        c = (ctypes.c_uint32 * 3)()
        self._check(self._lib.rb_p2p_counters(self._h, c))
        return tuple(c)

    def totals(self):
        """Work executed since create: (AdvanceFrames, SaveGameStates, LoadGameStates,
        speculative selects, branch frames presimulated)."""
        c = (ctypes.c_uint64 * 5)()
        self._check(self._lib.rb_p2p_totals(self._h, c))
        return tuple(int(x) for x in c)

    # -- desync detection (p2p_session.rs:873-928)
    def take_checksum_reports(self, out=None):
        """The ChecksumReports every session sent since the last call, oldest
        first, as a CUDA int64 tensor [RB_P2P_REPORTS_PER_TAKE, S, 3] (one
        rb_checksum_report per row: checksum lo, hi, frame | mismatch << 32;
        frame NULL_FRAME = none).  Ordered against torch's current stream
        (_StreamOrdered): later work on it sees the reports; `out` may be reused."""
        import torch
        from .shard import REPORT_WORDS
        K = L.RB_P2P_REPORTS_PER_TAKE
        if out is None:
            out = torch.empty((K, self.num_sessions, REPORT_WORDS), dtype=torch.int64, device="cuda")
        assert out.is_cuda and out.is_contiguous() and tuple(out.shape) == (K, self.num_sessions, REPORT_WORDS)
        cur = self._pre()
        self._check(self._lib.rb_p2p_take_checksum_reports(self._h, ctypes.c_void_p(out.data_ptr())))
        self._post(cur, (out,), outputs=True)
        return out

    def receive_checksum_reports(self, handle: int, reports) -> None:
        """The peer behind remote `handle` sent `reports` ([K, S, 3] int64 CUDA
        tensor, take_checksum_reports layout): UdpProtocol::on_checksum_report."""
        r, keep = _dev_ptr(reports)
        assert keep.dim() == 3 and keep.shape[1] == self.num_sessions
        cur = self._pre()
        st = self._lib.rb_p2p_receive_checksum_reports(self._h, int(handle), r, int(keep.shape[0]))
        self._post(cur, (keep,))
        if st == L.RB_INVALID_REQUEST:
            raise InvalidRequest((self._lib.rb_p2p_last_error(self._h) or b"").decode())
        self._check(st)

    def desync_events(self):
        """(counts [S], frames [S, E], handles [S, E], local [S, E], remote [S, E]):
        GGRSEvent::DesyncDetected per session since create, the newest E in order."""
        E = L.RB_P2P_EVENTS_KEPT
        n = np.empty(self.num_sessions, np.uint32)
        fr = np.empty((self.num_sessions, E), np.int32)
        hd = np.empty((self.num_sessions, E), np.int32)
        lo = np.empty((self.num_sessions, E), np.uint64)
        ro = np.empty((self.num_sessions, E), np.uint64)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        self._check(self._lib.rb_p2p_read_desync_events(self._h, p(n), p(fr), p(hd), p(lo), p(ro)))
        return n, fr, hd, lo, ro

    def receive_peer_connect_status(self, endpoint: int, last_frames, disconnected) -> None:
        """The peer behind remote handle `endpoint` reports every player's ConnectionStatus
        (UdpProtocol::on_input, protocol.rs:627-636): last_frames [P, S] int32 and
        disconnected [P, S] uint8, CUDA tensors.  Needs with_peer_connect_status(True)."""
        lp, lk = _dev_ptr(last_frames)
        dp, dk = _dev_ptr(disconnected)
        assert tuple(lk.shape) == (self.num_players, self.num_sessions) and tuple(dk.shape) == tuple(lk.shape)
        cur = self._pre()
        st = self._lib.rb_p2p_receive_peer_connect_status(self._h, int(endpoint), lp, dp)
        self._post(cur, (lk, dk))
        if st == L.RB_INVALID_REQUEST:
            raise InvalidRequest((self._lib.rb_p2p_last_error(self._h) or b"").decode())
        self._check(st)

    def debug_corrupt(self, session: int, word: int, xor_mask: int) -> None:
        """Flip canonical state word `word` of the live state and every cell of `session`."""
        st = self._lib.rb_p2p_debug_corrupt(self._h, int(session), int(word), ctypes.c_uint32(xor_mask & 0xFFFFFFFF))
        if st == L.RB_INVALID_REQUEST:
            raise InvalidRequest((self._lib.rb_p2p_last_error(self._h) or b"").decode())
        self._check(st)

    def profile_enable(self, on: bool) -> None:
        self._check(self._lib.rb_p2p_profile_enable(self._h, int(on)))

    def profile_take(self):
        ms = ctypes.c_double()
        n = ctypes.c_int32()
        self._check(self._lib.rb_p2p_profile_take(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def launch_clock_arm(self, launches: int) -> None:
        """The kernel's own clock for the next ``launches`` launches (rb_p2p_launch_clock_arm)."""
        self._check(self._lib.rb_p2p_launch_clock_arm(self._h, int(launches)))

    def launch_clock_read(self, cap: int):
        """Per launch since the arm: microseconds from its first wave's start to its last wave's end."""
        out = (ctypes.c_uint64 * (2 * cap))()
        n = ctypes.c_int32()
        self._check(self._lib.rb_p2p_launch_clock_read(self._h, out, int(cap), ctypes.byref(n)))
        return [(out[2 * i + 1] - out[2 * i]) / 100.0 for i in range(n.value)]


def synth_network(num_sessions: int, num_players: int, ticks: int, local_mask: int, remote_delay: int,
                  min_lag: int = 1, max_lag: int = 4, seed: int = SEED, first_session: int = 0,
                  dtype=np.uint8, mask: int = 0x0F):
    """A deterministic two-way network of peers in lock-step (numpy).

    Remote handle h's peer adds its local input for its frame f at frame
    f + remote_delay and sends it; it reaches us ``lag`` ticks later, with lag
    drawn per (session, tick) in [min_lag, max_lag] by splitmix64.  Deliveries
    are in order (UdpProtocol's sequencing): remote_upto[t] is the running
    maximum of (t - 1 - lag + remote_delay).

    Returns (local_inputs [T, P, S], remote_upto int32 [T, P, S],
    remote_inputs [T + remote_delay, P, S] by frame)."""
    from .synth import synth_inputs
    S, P, T = num_sessions, num_players, ticks
    inputs = synth_inputs(S, P, T, seed=seed, mask=mask, dtype=dtype, first_session=first_session)
    remote_in = np.zeros((T + remote_delay, P, S), dtype)
    remote_in[remote_delay:] = inputs  # the peer's input for its frame f lands at frame f + delay
    s = np.arange(first_session, first_session + S, dtype=np.uint64)[None, :]
    p = np.arange(P, dtype=np.uint64)[:, None]
    upto = np.empty((T, P, S), np.int32)
    run = np.full((P, S), -1, np.int64)
    span = max_lag - min_lag + 1
    for t in range(T):
        h = splitmix64(np.uint64(seed ^ 0x6E6574) ^ ((s << np.uint64(24)) + (p << np.uint64(20)) + np.uint64(t)))
        lag = min_lag + (h % np.uint64(span)).astype(np.int64)
        run = np.maximum(run, t - 1 - lag + remote_delay)
        upto[t] = np.minimum(run, T + remote_delay - 1)
    for hnd in range(P):
        if (local_mask >> hnd) & 1:
            upto[:, hnd] = -1
    return inputs, upto, remote_in
