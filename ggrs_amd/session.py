"""Host-side mirror of the GGRS session API over the C ABI.

Same names, argument meaning and error behaviour as the reference
(``SessionBuilder`` builder.rs:32-377, ``SyncTestSession``
sync_test_session.rs:11-204, ``GGRSError`` error.rs:11-36,
``GGRSRequest`` lib.rs:170-194), batched: one object drives ``num_sessions``
independent sessions in lock-step on one GPU, and ``advance_frame`` executes
the request stream it returns on the device (the game handler is compiled in,
selected by ``Game``).
"""
from __future__ import annotations

import ctypes
import enum
from collections import namedtuple
from typing import List, Optional

import numpy as np

from . import _lib as L


# --------------------------------------------------------------------------- errors (error.rs)
class GGRSError(Exception):
    """Base of the reference's GGRSError variants."""


class PredictionThreshold(GGRSError):
    """error.rs:13"""


class InvalidRequest(GGRSError):
    """error.rs:15-18; ``info`` carries the reference's message."""

    def __init__(self, info: str):
        super().__init__(f"Invalid Request: {info}")
        self.info = info


class MismatchedChecksum(GGRSError):
    """error.rs:22-25.  Batched: ``frames[s]`` is the frame reported by session s
    (``NULL_FRAME`` for sessions that advanced), ``frame`` the first failing one."""

    def __init__(self, frames: np.ndarray):
        failed = np.nonzero(frames != NULL_FRAME)[0]
        self.frames = frames
        self.sessions = failed
        self.frame = int(frames[failed[0]]) if failed.size else NULL_FRAME
        super().__init__(f"Detected checksum mismatch during rollback on frame {self.frame} "
                         f"({failed.size} session(s)).")


class NotSynchronized(GGRSError):
    """error.rs:27"""


class SpectatorTooFarBehind(GGRSError):
    """error.rs:29"""


class DeviceError(GGRSError):
    """HIP runtime failure (no reference analogue)."""


class Panic(GGRSError):
    """A condition the reference enforces with assert!/panic!."""


NULL_FRAME = L.RB_NULL_FRAME


class InputStatus(enum.IntEnum):  # lib.rs:104-112
    Confirmed = 0
    Predicted = 1
    Disconnected = 2


class RequestKind(enum.IntEnum):  # lib.rs:170-194
    SaveGameState = 0
    LoadGameState = 1
    AdvanceFrame = 2


# (kind, frame): Save/Load carry the cell's frame; AdvanceFrame carries the
# frame it advances from (the reference's AdvanceFrame carries the inputs).
GGRSRequest = namedtuple("GGRSRequest", ["kind", "frame"])


class Game(enum.IntEnum):
    EX_GAME = L.RB_GAME_EX_GAME
    STUB = L.RB_GAME_STUB
    STUB_ENUM = L.RB_GAME_STUB_ENUM
    STUB_RANDOM_CS = L.RB_GAME_STUB_RANDOM_CS
    BRAWLER = L.RB_GAME_BRAWLER


INPUT_DTYPE = {Game.EX_GAME: np.uint8, Game.STUB: np.uint32, Game.STUB_ENUM: np.uint8,
               Game.STUB_RANDOM_CS: np.uint32, Game.BRAWLER: np.uint8}
_DTYPE_OF_BYTES = {1: np.uint8, 2: np.uint16, 4: np.uint32}


def game_of(game_id: int):
    """Game for the built-in ids, the plain int for a registered plugin game."""
    try:
        return Game(game_id)
    except ValueError:
        return int(game_id)


def input_dtype(game, input_bytes: int):
    """numpy dtype of one Input of `game` (plugin games: by their Input size)."""
    return INPUT_DTYPE.get(game) or _DTYPE_OF_BYTES[input_bytes]


def _raise(lib, handle, status: int):
    if status == L.RB_OK:
        return
    msg = (lib.rb_last_error(handle) or b"").decode()
    if status == L.RB_INVALID_REQUEST:
        raise InvalidRequest(msg)
    if status == L.RB_PREDICTION_THRESHOLD:
        raise PredictionThreshold(msg)
    if status == L.RB_NOT_SYNCHRONIZED:
        raise NotSynchronized(msg)
    if status == L.RB_SPECTATOR_TOO_FAR_BEHIND:
        raise SpectatorTooFarBehind(msg)
    if status == L.RB_DEVICE_ERROR:
        raise DeviceError(msg)
    raise Panic(msg or f"rb_status {status}")


class RequestList:
    """The Vec<GGRSRequest> of one advance_frame, decoded on first access."""

    __slots__ = ("_k", "_f", "_n", "_items")

    def __init__(self, kinds, frames, n):
        self._k, self._f, self._n, self._items = kinds, frames, n, None

    def _decode(self):
        if self._items is None:
            self._items = [GGRSRequest(RequestKind(self._k[i]), self._f[i]) for i in range(self._n)]
        return self._items

    def __len__(self):
        return self._n

    def __iter__(self):
        return iter(self._decode())

    def __getitem__(self, i):
        return self._decode()[i]

    def __eq__(self, other):
        return list(self._decode()) == list(other)

    def __repr__(self):
        return repr(self._decode())


# --------------------------------------------------------------------------- builder (builder.rs)
class SessionBuilder:
    """builder.rs:32-377, SyncTest subset, plus the batch size and device."""

    def __init__(self, game=Game.EX_GAME, num_sessions: int = 1, device: int = 0):
        """game: a Game, or the id ggrs_amd.plugin.register_game_plugin returned."""
        self._cfg = L.RbConfig()
        L.load().rb_config_init(ctypes.byref(self._cfg))
        self._cfg.game = int(game)
        self._cfg.num_sessions = int(num_sessions)
        self._cfg.device = int(device)

    def with_num_players(self, num_players: int) -> "SessionBuilder":  # :154-157
        self._cfg.num_players = int(num_players)
        return self

    def with_max_prediction_window(self, window: int) -> "SessionBuilder":  # :136-145
        if window == 0:
            raise InvalidRequest("Currently, only prediction windows above 0 are supported")
        self._cfg.max_prediction = int(window)
        return self

    def with_input_delay(self, delay: int) -> "SessionBuilder":  # :148-151
        self._cfg.input_delay = int(delay)
        return self

    def with_check_distance(self, check_distance: int) -> "SessionBuilder":  # :202-205
        self._cfg.check_distance = int(check_distance)
        return self

    def with_num_sessions(self, num_sessions: int) -> "SessionBuilder":
        self._cfg.num_sessions = int(num_sessions)
        return self

    def with_device(self, device: int) -> "SessionBuilder":
        """HIP device ordinal; -1 builds a plan-only batch (host bookkeeping only)."""
        self._cfg.device = int(device)
        return self

    def with_checked_mismatches(self, checked: bool) -> "SessionBuilder":
        """True (default): advance_frame raises MismatchedChecksum in the call
        the reference would (one host/device sync per call).  False: fully
        asynchronous ticks; read failures with ``mismatches()``."""
        if checked:
            self._cfg.flags |= L.RB_FLAG_CHECKED
        else:
            self._cfg.flags &= ~L.RB_FLAG_CHECKED
        return self

    def with_seed(self, seed: int) -> "SessionBuilder":
        self._cfg.seed = int(seed) & (2**64 - 1)
        return self

    def with_lane_per_session(self, on: bool) -> "SessionBuilder":
        """ex_game: one lane per session (True) instead of one lane per player."""
        if on:
            self._cfg.flags |= L.RB_FLAG_LANE_PER_SESSION
        else:
            self._cfg.flags &= ~L.RB_FLAG_LANE_PER_SESSION
        return self

    def with_debug_flags(self, flags: int) -> "SessionBuilder":
        """Experiment knobs for kernel attribution (results are WRONG when set)."""
        self._cfg.reserved[0] = int(flags)
        return self

    def with_block_size(self, block: int) -> "SessionBuilder":
        self._cfg.block_size = int(block)
        return self

    # -- P2P (builder.rs:90-128, 159-166, 251-308)
    def add_player(self, player_type: "PlayerType", player_handle: int) -> "SessionBuilder":
        """PlayerType.Local or PlayerType.Remote for handle < num_players.  The
        remote's address is not needed: the batch takes delivered inputs
        directly (P2PSession.run_ticks)."""
        from .p2p import PlayerType
        players = getattr(self, "_players", {})
        if player_handle in players:
            raise InvalidRequest("Player handle already in use.")
        if player_type not in (PlayerType.Local, PlayerType.Remote):
            raise InvalidRequest("spectators are not part of the P2P batch")
        players[int(player_handle)] = player_type
        self._players = players
        return self

    def with_sparse_saving_mode(self, sparse_saving: bool) -> "SessionBuilder":  # :159-166
        self._sparse = bool(sparse_saving)
        return self

    def with_speculative_fanout(self, on: bool, candidates: int = 16, adaptive: bool = True,
                                min_select_permille: int = 0, per_player=None) -> "SessionBuilder":
        """P2P: presimulate `candidates` (1..16) candidate inputs of the
        most-lagging remote handle after every tick (RB_P2P_FLAG_FANOUT,
        BASELINE config 4): the whole input alphabet when it has at most that
        many values (ex_game), else the most likely ones (include/ggrs_amd.h).
        adaptive: pause it while too few rollbacks become selects (below
        min_select_permille, 0 = the engine's default; RB_P2P_FLAG_FANOUT_ALWAYS
        when False).  per_player: speculate every remote player
        (RB_P2P_FLAG_FANOUT_PER_PLAYER) rather than the one with the oldest
        unconfirmed input; None (default) = per player where the game's players
        move independently and the candidates cover its input alphabet
        (ex_game at 16: 66% of C4's rollbacks become selects instead of 31%)."""
        self._fanout = bool(on)
        self._fanout_k = int(candidates)
        self._fanout_adaptive = bool(adaptive)
        self._fanout_permille = int(min_select_permille)
        self._fanout_per_player = per_player  # RB_P2P_FLAG_FANOUT_PER_PLAYER: every remote player (None: start decides)
        return self

    def _per_player_resolved(self) -> bool:
        pp = getattr(self, "_fanout_per_player", False)
        if pp is None:  # the games whose players move independently (games.hpp kIndependentPlayers)
            pp = (self._cfg.game == Game.EX_GAME and int(self._cfg.num_players) >= 2
                  and getattr(self, "_fanout_k", 16) >= 16)
        return bool(pp) and getattr(self, "_fanout", False)

    def with_desync_detection_mode(self, interval: int) -> "SessionBuilder":  # builder.rs:169-172
        """P2P: DesyncDetection::On{interval} for interval > 0, Off for 0 (default)."""
        if interval < 0:
            raise InvalidRequest("desync detection interval must be >= 0")
        self._desync = int(interval)
        return self

    def with_peer_connect_status(self, on: bool) -> "SessionBuilder":
        """P2P: track the peers' connect-status reports (P2PSession.receive_peer_connect_status)
        and run update_player_disconnects (p2p_session.rs:707-742) every tick."""
        self._peer_status = bool(on)
        return self

    def with_remote_input_delay(self, delay: int) -> "SessionBuilder":
        """Frame of each remote handle's first input (the peers' input delay)."""
        self._remote_delay = int(delay)
        return self

    def start_p2p_session(self) -> "P2PSession":  # :251-308
        from .p2p import P2PSession, PlayerType
        players = getattr(self, "_players", {})
        n = int(self._cfg.num_players)
        for h in range(n):
            if h not in players:
                raise InvalidRequest("Not enough players have been added. Keep registering players up to the "
                                     "defined player number.")
        if any(h >= n for h in players):
            raise InvalidRequest("The player handle you provided is invalid. For a local player, the handle "
                                 "should be between 0 and num_players")
        pc = L.RbP2PConfig()
        lib = L.load()
        lib.rb_p2p_config_init(ctypes.byref(pc))
        pc.game = self._cfg.game
        pc.num_sessions = self._cfg.num_sessions
        pc.num_players = n
        pc.max_prediction = self._cfg.max_prediction
        pc.input_delay = self._cfg.input_delay
        pc.device = self._cfg.device
        pc.local_mask = sum(1 << h for h, t in players.items() if t == PlayerType.Local)
        pc.remote_delay = getattr(self, "_remote_delay", 0)
        pc.sparse_saving = int(getattr(self, "_sparse", False))
        pc.flags = (self._cfg.flags & L.RB_FLAG_LANE_PER_SESSION) | (
            L.RB_P2P_FLAG_FANOUT if getattr(self, "_fanout", False) else 0) | (
            L.RB_P2P_FLAG_FANOUT_ALWAYS if not getattr(self, "_fanout_adaptive", True) else 0) | (
            L.RB_P2P_FLAG_FANOUT_PER_PLAYER if self._per_player_resolved() else 0) | (
            L.RB_P2P_FLAG_PEER_STATUS if getattr(self, "_peer_status", False) else 0)
        pc.block_size = self._cfg.block_size
        pc.desync_interval = getattr(self, "_desync", 0)
        pc.fanout_candidates = getattr(self, "_fanout_k", 16)
        pc.fanout_min_select_permille = getattr(self, "_fanout_permille", 0)
        h = ctypes.c_void_p()
        st = lib.rb_p2p_create(ctypes.byref(pc), ctypes.byref(h))
        if st != L.RB_OK:
            msg = (lib.rb_p2p_last_error(None) or b"").decode()
            raise InvalidRequest(msg) if st == L.RB_INVALID_REQUEST else DeviceError(msg)
        return P2PSession(lib, h, game_of(pc.game), pc)

    def start_synctest_session(self) -> "SyncTestSession":  # :342-354
        lib = L.load()
        h = ctypes.c_void_p()
        st = lib.rb_synctest_create(ctypes.byref(self._cfg), ctypes.byref(h))
        _raise(lib, None, st)
        return SyncTestSession(lib, h, game_of(self._cfg.game), self._cfg)


# --------------------------------------------------------------------------- stream ordering
class _StreamOrdered:
    """Orders a batch's device work against torch's current stream.

    A device batch runs on its own HIP stream unless ``set_stream`` chose
    another (rb_get_stream says which).  When torch's current stream is not
    that stream at a call, the call (1) makes the batch stream wait for the
    work queued on torch's stream so far (device inputs made there are
    complete before a launch reads them), (2) keeps the tensors it handed to
    the device referenced until an event recorded after its launches has
    completed (the caching allocator cannot hand their memory to torch's
    stream while a launch may still read it), and (3) for calls that write a
    caller tensor, makes torch's stream wait for the batch stream.  When the
    streams are the same, stream order already gives all three and nothing is
    added."""

    _stream = None  # the batch's HIP stream as a torch stream object, or None (plan-only)
    _inflight = None  # deque of (event, tensors) of calls still possibly reading their tensors

    def _bind(self, device: int, handle: int):
        """Wrap the batch's stream (rb_get_stream / rb_p2p_get_stream) for torch."""
        self._stream = None
        if device < 0 or not handle:
            return
        import torch
        if torch.cuda.is_available():
            self._stream = torch.cuda.ExternalStream(int(handle), device=torch.device("cuda", device))

    def _pre(self):
        """Before a launching call: the torch stream to order against, or None (same stream)."""
        st = self._stream
        if st is None:
            return None
        import torch
        cur = torch.cuda.current_stream(st.device)
        if cur.cuda_stream == st.cuda_stream:
            return None
        st.wait_stream(cur)
        return cur

    def _post(self, cur, tensors=(), outputs=False):
        """After a launching call that _pre ordered against `cur`."""
        if cur is None:
            return
        import collections

        import torch
        st = self._stream
        if tensors:
            if self._inflight is None:
                self._inflight = collections.deque()
            ev = torch.cuda.Event()
            ev.record(st)
            self._inflight.append((ev, tensors))
        while self._inflight and self._inflight[0][0].query():
            self._inflight.popleft()
        if outputs:
            cur.wait_stream(st)

    def _drain(self):
        """After the batch stream was synchronised (close): nothing is in flight."""
        if self._inflight:
            self._inflight.clear()


# --------------------------------------------------------------------------- session
class SyncTestSession(_StreamOrdered):
    """sync_test_session.rs:11-204 for ``num_sessions`` sessions at once."""

    def __init__(self, lib, handle, game: Game, cfg):
        self._lib = lib
        self._h = handle
        self.game = game
        self.num_sessions = int(cfg.num_sessions)
        self._num_players = int(cfg.num_players)
        self._max_prediction = int(cfg.max_prediction)
        self.check_distance = int(cfg.check_distance)
        self.input_delay = int(cfg.input_delay)
        self.checked = bool(cfg.flags & L.RB_FLAG_CHECKED)
        self.state_bytes = lib.rb_state_bytes(handle)
        self.input_dtype = input_dtype(game, lib.rb_input_bytes(handle))
        self._keep = []  # host arrays referenced by queued copies
        self._device = int(cfg.device)
        self._bind(self._device, lib.rb_get_stream(handle) or 0)

    # -- lifetime
    def close(self):
        if self._h:
            self._lib.rb_destroy(self._h)  # synchronises the batch stream first
            self._h = None
            self._stream = None
            self._drain()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- reference API
    def num_players(self) -> int:  # :149-151
        return self._num_players

    def max_prediction(self) -> int:  # :154-156
        return self._max_prediction

    def current_frame(self) -> int:
        return self._lib.rb_current_frame(self._h)

    def _as_input(self, inputs, count):
        """numpy/int -> (pointer, on_device, keepalive); torch CUDA tensors pass through."""
        if hasattr(inputs, "data_ptr") and getattr(inputs, "is_cuda", False):
            if inputs.numel() != count or not inputs.is_contiguous():
                raise InvalidRequest("device inputs must be a contiguous tensor of num_sessions values")
            if inputs.element_size() != np.dtype(self.input_dtype).itemsize:
                raise InvalidRequest("device inputs have the wrong element size for this game's Input")
            return ctypes.c_void_p(inputs.data_ptr()), 1, inputs
        a = np.asarray(inputs)
        a = a.reshape(-1) if a.size == count else np.broadcast_to(a, (count,))
        arr = np.ascontiguousarray(a, dtype=self.input_dtype)
        return arr.ctypes.data_as(ctypes.c_void_p), 0, arr

    def add_local_input(self, player_handle: int, inputs) -> None:  # :61-74
        """Input of ``player_handle`` for the current frame in every session:
        an array of num_sessions values, a scalar (same input everywhere) or a
        CUDA tensor (stays on the device)."""
        ptr, dev, keep = self._as_input(inputs, self.num_sessions)
        self._keep.append(keep)
        cur = self._pre() if dev else None
        _raise(self._lib, self._h, self._lib.rb_add_local_input(self._h, int(player_handle), ptr, dev))
        self._post(cur)  # the tensor stays in _keep until advance_frame has launched

    def add_local_inputs(self, inputs) -> None:
        """All handles at once: [num_sessions, num_players] values."""
        ptr, dev, keep = self._as_input(inputs, self.num_sessions * self._num_players)
        self._keep.append(keep)
        cur = self._pre() if dev else None
        _raise(self._lib, self._h, self._lib.rb_add_local_inputs_packed(self._h, ptr, dev))
        self._post(cur)

    def advance_frame(self) -> "RequestList":  # :85-146
        """Runs SyncTestSession::advance_frame and the game's handle_requests
        for every session; returns the request stream that was executed
        (a list of GGRSRequest, decoded lazily)."""
        cur = self._pre()
        st = self._lib.rb_advance_frame(self._h)
        self._post(cur, tuple(k for k in self._keep if hasattr(k, "data_ptr")))
        self._keep.clear()
        if st == L.RB_MISMATCHED_CHECKSUM:
            raise MismatchedChecksum(self.mismatches())
        _raise(self._lib, self._h, st)
        return self.last_requests()

    def run_ticks(self, inputs) -> int:
        """``len(inputs)`` x (add_local_input for every handle + advance_frame)
        in one native call; ``inputs`` is [T, num_players, num_sessions]
        (numpy, or a CUDA tensor kept on the device)."""
        T = int(inputs.shape[0])
        per_tick = self._num_players * self.num_sessions
        ptr, dev, keep = self._as_input(inputs, T * per_tick) if T else (None, 0, None)
        cur = self._pre() if dev else None
        done = ctypes.c_int32()
        st = self._lib.rb_run_ticks(self._h, T, ptr, per_tick * np.dtype(self.input_dtype).itemsize, dev,
                                    ctypes.byref(done))
        self._post(cur, (keep,))
        if st == L.RB_MISMATCHED_CHECKSUM:
            raise MismatchedChecksum(self.mismatches())
        _raise(self._lib, self._h, st)
        return done.value

    def prepare_ticks(self, inputs):
        """run_ticks(inputs) as a prepared native call, for a host loop whose
        per-call cost matters (a compiled host calls rb_run_ticks directly):
        the pointer, stride and status slot are built here, once, and the
        returned ``call()`` is the bare C call.  ``call()`` returns the
        rb_status and ``check(status)`` turns it into run_ticks' return value
        or exception.  ``inputs`` must be a CUDA tensor [T, num_players,
        num_sessions] that outlives the calls, and they must be made with
        torch's current stream equal to the batch stream (set_stream), so
        that stream order alone orders them against torch's work."""
        T = int(inputs.shape[0])
        per_tick = self._num_players * self.num_sessions
        ptr, dev, _ = self._as_input(inputs, T * per_tick)
        if not dev or T <= 0:
            raise InvalidRequest("prepare_ticks takes a non-empty CUDA tensor")
        if self._pre() is not None:
            raise InvalidRequest("prepare_ticks: torch's current stream must be the batch stream (set_stream)")
        done = ctypes.c_int32()
        fn, args = self._lib.rb_run_ticks, (self._h, T, ptr, per_tick * np.dtype(self.input_dtype).itemsize, 1,
                                            ctypes.byref(done))

        def call():
            return fn(*args)

        def check(st):
            if st == L.RB_MISMATCHED_CHECKSUM:
                raise MismatchedChecksum(self.mismatches())
            _raise(self._lib, self._h, st)
            return done.value

        return call, check

    # -- batch extras
    def last_requests(self) -> "RequestList":
        cap = 4 * self._max_prediction + 8
        k = (ctypes.c_int32 * cap)()
        f = (ctypes.c_int32 * cap)()
        n = self._lib.rb_last_requests(self._h, k, f, cap)
        return RequestList(k, f, n)

    def mismatches(self) -> np.ndarray:
        out = np.empty(self.num_sessions, dtype=np.int32)
        cnt = ctypes.c_int32()
        _raise(self._lib, self._h, self._lib.rb_mismatches(
            self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ctypes.byref(cnt)))
        return out

    def synchronize(self) -> None:
        _raise(self._lib, self._h, self._lib.rb_synchronize(self._h))

    def set_stream(self, stream) -> None:
        """Run on a caller stream (int handle or torch.cuda.Stream)."""
        ptr = getattr(stream, "cuda_stream", stream)
        _raise(self._lib, self._h, self._lib.rb_set_stream(self._h, ctypes.c_void_p(ptr)))
        self._bind(self._device, self._lib.rb_get_stream(self._h) or 0)

    def read_cell(self, frame: int):
        """(images [S, state_bytes] u8, checksums [S, 2] u64 lo/hi) of the cell holding ``frame``."""
        img = np.empty((self.num_sessions, self.state_bytes), dtype=np.uint8)
        cs = np.empty((self.num_sessions, 2), dtype=np.uint64)
        _raise(self._lib, self._h, self._lib.rb_read_cell(
            self._h, int(frame), img.ctypes.data_as(ctypes.c_void_p),
            cs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
        return img, cs

    def read_live(self):
        """(images [S, state_bytes], display checksums [S] u64, display frames [S] i32)."""
        img = np.empty((self.num_sessions, self.state_bytes), dtype=np.uint8)
        dcs = np.empty(self.num_sessions, dtype=np.uint64)
        fr = np.empty(self.num_sessions, dtype=np.int32)
        _raise(self._lib, self._h, self._lib.rb_read_live(
            self._h, img.ctypes.data_as(ctypes.c_void_p),
            dcs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), fr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return img, dcs, fr

    def export_compact_report(self, frame: int, dev_ptr) -> None:
        """Write [S] uint32 compact reports (rb_export_compact_report: 16-bit checksum,
        mismatch delta and flag) for ``frame`` to device memory; 16-bit-checksum games only."""
        is_t = hasattr(dev_ptr, "data_ptr")
        ptr = dev_ptr.data_ptr() if is_t else dev_ptr
        cur = self._pre()
        _raise(self._lib, self._h, self._lib.rb_export_compact_report(self._h, int(frame), ctypes.c_void_p(ptr)))
        self._post(cur, (dev_ptr,) if is_t else (), outputs=True)

    def export_checksum_report(self, frame: int, dev_ptr: int) -> None:
        """Write [S] rb_checksum_report (24 B each) for ``frame`` to device memory
        (a pointer, or a CUDA tensor); torch's current stream waits for it."""
        is_t = hasattr(dev_ptr, "data_ptr")
        ptr = dev_ptr.data_ptr() if is_t else dev_ptr
        cur = self._pre()
        _raise(self._lib, self._h, self._lib.rb_export_checksum_report(self._h, int(frame), ctypes.c_void_p(ptr)))
        self._post(cur, (dev_ptr,) if is_t else (), outputs=True)

    def debug_corrupt_cell(self, session: int, frame: int, word: int, xor_mask: int) -> None:
        _raise(self._lib, self._h, self._lib.rb_debug_corrupt_cell(
            self._h, int(session), int(frame), int(word), ctypes.c_uint32(xor_mask & 0xFFFFFFFF)))

    def profile_enable(self, on: bool = True) -> None:
        _raise(self._lib, self._h, self._lib.rb_profile_enable(self._h, 1 if on else 0))

    def profile_take(self):
        """(summed tick-kernel milliseconds, launches) since the last call."""
        ms = ctypes.c_double()
        n = ctypes.c_int32()
        _raise(self._lib, self._h, self._lib.rb_profile_take(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def launch_clock_arm(self, launches: int) -> None:
        """The kernel's own clock for the next ``launches`` fused launches (rb_launch_clock_arm)."""
        _raise(self._lib, self._h, self._lib.rb_launch_clock_arm(self._h, int(launches)))

    def launch_clock_read(self, cap: int):
        """Per fused launch since the arm: microseconds from its first wave's start to its last wave's end."""
        out = (ctypes.c_uint64 * (2 * cap))()
        n = ctypes.c_int32()
        _raise(self._lib, self._h, self._lib.rb_launch_clock_read(self._h, out, int(cap), ctypes.byref(n)))
        return [(out[2 * i + 1] - out[2 * i]) / 100.0 for i in range(n.value)]


# --------------------------------------------------------------------------- decoding helpers
def decode_ex_game(images: np.ndarray, num_players: int) -> dict:
    """Split bincode images of ex_game State (ex_game.rs:224-231) into fields."""
    P = num_players
    assert images.shape[-1] == 36 + 20 * P
    out = {"frame": images[..., 0:4].copy().view(np.int32)[..., 0]}
    out["num_players"] = images[..., 4:12].copy().view(np.uint64)[..., 0]
    out["positions"] = images[..., 20:20 + 8 * P].copy().view(np.float32).reshape(images.shape[:-1] + (P, 2))
    o = 28 + 8 * P
    out["velocities"] = images[..., o:o + 8 * P].copy().view(np.float32).reshape(images.shape[:-1] + (P, 2))
    o = 36 + 16 * P
    out["rotations"] = images[..., o:o + 4 * P].copy().view(np.float32)
    return out
