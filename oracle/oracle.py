"""TEST INFRASTRUCTURE ONLY — ctypes driver of the CPU restatement (oracle/).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It loads oracle/build/liboracle.so (built by oracle/Makefile)
and exposes S independent reference sessions (SyncTestSession + game,
driven like ex_game_synctest.rs:59-72).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
REF_TESTS = os.path.join(_HERE, "build", "ref_tests")

EX_GAME, STUB, STUB_ENUM, STUB_RANDOM_CS, BRAWLER = 1, 2, 3, 4, 5
PLUGIN = 100  # the include/ggrs_amd_game.hpp game compiled into an oracle plugin build
KIND_PANIC = 99
_libs = {}


def plugin_lib(name: str) -> str:
    """Path of the oracle built with a plugin game (oracle/Makefile `plugin`, PLUGIN_NAME=name)."""
    return os.path.join(_HERE, "build", f"liboracle_{name}.so")


def load(path: str = LIB_PATH):
    """The oracle library at `path` (the standard build, or a plugin build)."""
    if path not in _libs:
        if not os.path.exists(path):
            raise ImportError(f"{path} missing: run `make -C oracle`")
        lib = ctypes.CDLL(path)
        P, I32, U64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64
        PI32 = ctypes.POINTER(ctypes.c_int32)
        sig = {
            "orc_image_bytes": (I32, [I32, I32]),
            "orc_input_bytes": (I32, [I32]),
            "orc_batch_create": (P, [I32, I32, I32, I32, I32, I32, U64]),
            "orc_last_error": (ctypes.c_char_p, []),
            "orc_last_panic": (ctypes.c_char_p, [P]),
            "orc_batch_destroy": (None, [P]),
            "orc_batch_add_local_input": (I32, [P, I32, P]),
            "orc_batch_advance": (I32, [P, PI32, PI32]),
            "orc_batch_trace": (I32, [P, I32, PI32, PI32, I32]),
            "orc_batch_read_cells": (I32, [P, PI32, P, P, P]),
            "orc_batch_read_live": (I32, [P, P, P, PI32]),
            "orc_batch_current_frame": (I32, [P]),
            "orc_fletcher16": (ctypes.c_uint16, [P, U64]),
            "orc_siphash": (U64, [I32, I32, U64, U64, P, U64]),
            "orc_cosf": (ctypes.c_float, [ctypes.c_float]),
            "orc_sinf": (ctypes.c_float, [ctypes.c_float]),
            "orc_sincosf_array": (None, [P, P, P, ctypes.c_int64]),
            "orc_check_exgame_inrange": (ctypes.c_int64, [ctypes.c_uint32, ctypes.c_int64, P, I32, P]),
            "orc_batch_corrupt_cell": (I32, [P, I32, I32, I32, ctypes.c_uint32]),
            "orc_synth_inputs": (None, [U64, ctypes.c_uint32, I32, I32, I32, I32, I32, P]),
            "orc_bench_exgame": (ctypes.c_double, [I32, I32, I32, I32, I32, I32, I32, I32, U64, PI32]),
            "orc_bench_brawler": (ctypes.c_double, [I32, I32, I32, I32, I32, I32, I32, I32, U64, PI32]),
            "orc_bench_exgame_soa": (ctypes.c_double, [I32, I32, I32, I32, I32, I32, I32, I32, U64, PI32]),
            "orc_soa_exgame_run": (I32, [I32, I32, I32, I32, I32, I32, I32, P, P, P]),
            "orc_p2p_create": (P, [I32, I32, I32, I32, ctypes.c_uint32, I32, I32, I32]),
            "orc_p2p_destroy": (None, [P]),
            "orc_p2p_last_panic": (ctypes.c_char_p, [P]),
            "orc_p2p_deliver": (I32, [P, I32, P, P, I32]),
            "orc_p2p_add_local_input": (I32, [P, I32, P]),
            "orc_p2p_advance": (I32, [P, P, P, P, P]),
            "orc_p2p_disconnect": (I32, [P, I32, P]),
            "orc_p2p_trace": (I32, [P, I32, PI32, PI32, I32]),
            "orc_p2p_read_cells": (I32, [P, P, P, P]),
            "orc_p2p_read_live": (I32, [P, P, P]),
            "orc_p2p_frames": (I32, [P, P, P]),
            "orc_p2p_queues": (I32, [P, P]),
            "orc_p2p_set_desync": (None, [P, ctypes.c_uint32]),
            "orc_p2p_take_reports": (I32, [P, P, P, I32]),
            "orc_p2p_receive_reports": (I32, [P, I32, P, P, I32]),
            "orc_p2p_events": (I32, [P, P, P, P, P, P, I32]),
            "orc_p2p_corrupt": (I32, [P, I32, I32, ctypes.c_uint32]),
            "orc_p2p_receive_peer_status": (I32, [P, I32, P, P]),
            "orc_wire_encode": (I32, [P, I32, P, I32, P, I32]),
            "orc_bench_p2p_exgame": (ctypes.c_double, [I32, I32, I32, ctypes.c_uint32, I32, I32, I32, I32, I32, P,
                                                        P, P, I32, P, P]),
            "orc_wire_decode": (I32, [P, I32, P, I32, P, I32]),
            "orc_bench_p2p_brawler": (ctypes.c_double, [I32, I32, I32, ctypes.c_uint32, I32, I32, I32, I32, I32, P,
                                                         P, P, I32, P, P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _libs[path] = lib
    return _libs[path]


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleBatch:
    """S independent reference sessions of one game (TEST ONLY)."""

    def __init__(self, game: int, num_players: int, max_prediction: int, check_distance: int,
                 input_delay: int, num_sessions: int, seed: int = 0, lib_path: str = LIB_PATH):
        lib = load(lib_path)
        self._lib = lib
        self._h = lib.orc_batch_create(game, num_players, max_prediction, check_distance, input_delay,
                                       num_sessions, seed)
        if not self._h:
            raise ValueError(lib.orc_last_error().decode())
        self.game, self.P, self.W, self.S = game, num_players, max_prediction, num_sessions
        self.image_bytes = lib.orc_image_bytes(game, num_players)
        self.input_dtype = {1: np.uint8, 2: np.uint16, 4: np.uint32}[lib.orc_input_bytes(game)]

    def close(self):
        if self._h:
            self._lib.orc_batch_destroy(self._h)
            self._h = None

    __del__ = close

    def add_local_input(self, handle: int, inputs) -> int:
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(inputs), (self.S,)), dtype=self.input_dtype)
        return self._lib.orc_batch_add_local_input(self._h, handle, _ptr(a))

    def advance(self):
        """(error kinds [S], error frames [S]); kind 0 = Ok, 3 = MismatchedChecksum, 99 = panic."""
        k = np.empty(self.S, np.int32)
        f = np.empty(self.S, np.int32)
        self._lib.orc_batch_advance(self._h, k.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                    f.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        return k, f

    def last_panic(self) -> str:
        return self._lib.orc_last_panic(self._h).decode()

    def trace(self, session: int = 0):
        cap = 4 * self.W + 8
        k = (ctypes.c_int32 * cap)()
        f = (ctypes.c_int32 * cap)()
        n = self._lib.orc_batch_trace(self._h, session, k, f, cap)
        return [(k[i], f[i]) for i in range(n)]

    def read_cells(self):
        """(cell frames [W], images [W, S, B], cs_valid [W, S], checksums [W, S, 2])."""
        fr = np.empty(self.W, np.int32)
        img = np.zeros((self.W, self.S, self.image_bytes), np.uint8)
        val = np.zeros((self.W, self.S), np.uint8)
        cs = np.zeros((self.W, self.S, 2), np.uint64)
        self._lib.orc_batch_read_cells(self._h, fr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _ptr(img),
                                       _ptr(val), _ptr(cs))
        return fr, img, val, cs

    def read_live(self):
        """(images [S, B], display checksums [S], display frames [S])."""
        img = np.zeros((self.S, self.image_bytes), np.uint8)
        cs = np.zeros(self.S, np.uint64)
        fr = np.zeros(self.S, np.int32)
        self._lib.orc_batch_read_live(self._h, _ptr(img), _ptr(cs), fr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        return img, cs, fr

    def current_frame(self) -> int:
        return self._lib.orc_batch_current_frame(self._h)

    def corrupt_cell(self, session: int, frame: int, word: int, xor_mask: int) -> None:
        rc = self._lib.orc_batch_corrupt_cell(self._h, session, frame, word, xor_mask & 0xFFFFFFFF)
        assert rc == 0, "no cell holds that frame"


class OracleP2P:
    """S independent network-free reference P2PSessions + games (TEST ONLY).

    Per tick: deliver(handle, upto, by_frame) for every remote handle (the
    Event::Input stream poll_remote_clients would produce: frames up to
    upto[s], values by_frame[f, s]), add_local_input for every local handle,
    advance()."""

    def __init__(self, game: int, num_players: int, max_prediction: int, input_delay: int, local_mask: int,
                 num_sessions: int, sparse_saving: bool = False, remote_delay: int = 0, lib_path: str = LIB_PATH):
        lib = load(lib_path)
        self._lib = lib
        self._h = lib.orc_p2p_create(game, num_players, max_prediction, input_delay, local_mask,
                                     int(sparse_saving), remote_delay, num_sessions)
        if not self._h:
            raise ValueError(lib.orc_last_error().decode())
        self.game, self.P, self.W, self.S = game, num_players, max_prediction, num_sessions
        self.image_bytes = lib.orc_image_bytes(game, num_players)
        self.input_dtype = {1: np.uint8, 2: np.uint16, 4: np.uint32}[lib.orc_input_bytes(game)]

    def close(self):
        if self._h:
            self._lib.orc_p2p_destroy(self._h)
            self._h = None

    __del__ = close

    def last_panic(self) -> str:
        return self._lib.orc_p2p_last_panic(self._h).decode()

    def deliver(self, handle: int, upto, by_frame) -> int:
        u = np.ascontiguousarray(np.broadcast_to(np.asarray(upto), (self.S,)), dtype=np.int32)
        b = np.ascontiguousarray(by_frame, dtype=self.input_dtype)
        assert b.ndim == 2 and b.shape[1] == self.S
        return self._lib.orc_p2p_deliver(self._h, handle, _ptr(u), _ptr(b), b.shape[0])

    def add_local_input(self, handle: int, inputs) -> int:
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(inputs), (self.S,)), dtype=self.input_dtype)
        return self._lib.orc_p2p_add_local_input(self._h, handle, _ptr(a))

    def disconnect_player(self, handle: int, sessions=None) -> int:
        """P2PSession::disconnect_player(handle) (p2p_session.rs:430-456) in the
        sessions whose `sessions` entry is true (None: all); first error kind or 0."""
        m = None if sessions is None else np.ascontiguousarray(np.broadcast_to(np.asarray(sessions), (self.S,)),
                                                                dtype=np.uint8)
        return self._lib.orc_p2p_disconnect(self._h, handle, None if m is None else _ptr(m))

    def advance(self):
        """(status [S] (0 Ok, 1 PredictionThreshold, 99 panic), load frame [S], AdvanceFrames [S], saves [S])."""
        st, lf, na, ns = (np.empty(self.S, np.int32) for _ in range(4))
        self._lib.orc_p2p_advance(self._h, _ptr(st), _ptr(lf), _ptr(na), _ptr(ns))
        return st, lf, na, ns

    def trace(self, session: int = 0):
        cap = 6 * self.W + 8
        k = (ctypes.c_int32 * cap)()
        f = (ctypes.c_int32 * cap)()
        n = self._lib.orc_p2p_trace(self._h, session, k, f, cap)
        return [(k[i], f[i]) for i in range(n)]

    def read_cells(self):
        """(cell frames [W, S], images [W, S, B], checksums [W, S, 2])."""
        fr = np.empty((self.W, self.S), np.int32)
        img = np.zeros((self.W, self.S, self.image_bytes), np.uint8)
        cs = np.zeros((self.W, self.S, 2), np.uint64)
        self._lib.orc_p2p_read_cells(self._h, _ptr(fr), _ptr(img), _ptr(cs))
        return fr, img, cs

    def read_live(self):
        """(images [S, B], current frames [S])."""
        img = np.zeros((self.S, self.image_bytes), np.uint8)
        fr = np.zeros(self.S, np.int32)
        self._lib.orc_p2p_read_live(self._h, _ptr(img), _ptr(fr))
        return img, fr

    def frames(self):
        """(current frames [S], last confirmed frames [S])."""
        c = np.empty(self.S, np.int32)
        k = np.empty(self.S, np.int32)
        self._lib.orc_p2p_frames(self._h, _ptr(c), _ptr(k))
        return c, k

    def queues(self):
        """InputQueue / ConnectionStatus bookkeeping [S, P, 8] (rb_p2p_read_queues's layout)."""
        out = np.empty((self.S, self.P, 8), np.int32)
        self._lib.orc_p2p_queues(self._h, _ptr(out))
        return out

    # -- desync detection (p2p_session.rs:873-928)
    def set_desync_detection(self, interval: int) -> None:
        """DesyncDetection::On{interval} (0 = Off)."""
        self._lib.orc_p2p_set_desync(self._h, int(interval))

    def take_checksum_reports(self, K: int = 8):
        """ChecksumReports sent since the last call, oldest first: (frames [K, S]
        (NULL_FRAME = none), checksums [K, S, 2] u128 lo/hi)."""
        fr = np.empty((K, self.S), np.int32)
        cs = np.empty((K, self.S, 2), np.uint64)
        self._lib.orc_p2p_take_reports(self._h, _ptr(fr), _ptr(cs), K)
        return fr, cs

    def receive_checksum_reports(self, handle: int, frames, checksums) -> int:
        """The peer of remote `handle` sent these reports (take_checksum_reports layout)."""
        fr = np.ascontiguousarray(frames, np.int32)
        cs = np.ascontiguousarray(checksums, np.uint64)
        return self._lib.orc_p2p_receive_reports(self._h, handle, _ptr(fr), _ptr(cs), fr.shape[0])

    def desync_events(self, E: int = 16):
        """(counts [S], frames [S, E], handles [S, E], local [S, E], remote [S, E]):
        DesyncDetected events since create, the newest E of each session in order."""
        n = np.empty(self.S, np.uint32)
        fr = np.empty((self.S, E), np.int32)
        hd = np.empty((self.S, E), np.int32)
        lo = np.empty((self.S, E), np.uint64)
        ro = np.empty((self.S, E), np.uint64)
        self._lib.orc_p2p_events(self._h, _ptr(n), _ptr(fr), _ptr(hd), _ptr(lo), _ptr(ro), E)
        return n, fr, hd, lo, ro

    def receive_peer_connect_status(self, endpoint: int, last_frames, disconnected) -> None:
        """The peer behind remote handle `endpoint` reports every player's
        ConnectionStatus: last_frames [P, S] i32, disconnected [P, S] bool."""
        lf = np.ascontiguousarray(np.broadcast_to(last_frames, (self.P, self.S)), np.int32)
        dc = np.ascontiguousarray(np.broadcast_to(disconnected, (self.P, self.S)), np.uint8)
        self._lib.orc_p2p_receive_peer_status(self._h, endpoint, _ptr(lf), _ptr(dc))

    def corrupt(self, session: int, word: int, xor_mask: int) -> None:
        """Flip canonical state word `word` of the live state and every saved cell."""
        self._lib.orc_p2p_corrupt(self._h, session, word, xor_mask & 0xFFFFFFFF)


def fletcher16(data: bytes) -> int:
    b = np.frombuffer(bytes(data), np.uint8)
    return load().orc_fletcher16(_ptr(b) if b.size else None, b.size)


def siphash(c: int, d: int, k0: int, k1: int, msg: bytes) -> int:
    b = np.frombuffer(bytes(msg) or b"\0", np.uint8)
    return load().orc_siphash(c, d, k0, k1, _ptr(b), len(msg))


def sincosf(x: np.ndarray):
    """glibc sinf/cosf of every element (host libm; what Rust's f32::sin/cos call)."""
    x = np.ascontiguousarray(x, np.float32)
    s = np.empty_like(x)
    c = np.empty_like(x)
    load().orc_sincosf_array(_ptr(x), _ptr(s), _ptr(c), x.size)
    return s, c


def check_exgame_inrange(first_bits: int, dev: np.ndarray, threads: int):
    """(mismatches, bits of the first mismatching float or None) of the device's in-range ex_game
    arithmetic dev [6, n] (rb_debug_exgame_inrange) for the floats with bits first_bits + i
    against this host's glibc sinf / cosf / fmodf (Rust's f32::sin / cos / rem_euclid)."""
    dev = np.ascontiguousarray(dev, np.float32)
    assert dev.ndim == 2 and dev.shape[0] == 6
    fb = np.zeros(1, np.uint32)
    n = load().orc_check_exgame_inrange(first_bits, dev.shape[1], _ptr(dev), threads, _ptr(fb))
    return int(n), (None if fb[0] == 0xFFFFFFFF else int(fb[0]))


def synth_inputs(seed: int, mask: int, S: int, P: int, T: int, f0: int = 0, input_bytes: int = 1) -> np.ndarray:
    out = np.empty((T, P, S), np.uint8 if input_bytes == 1 else np.uint32)
    load().orc_synth_inputs(seed, mask, S, P, T, f0, input_bytes, _ptr(out))
    return out


def bench_exgame(num_players: int, check_distance: int, input_delay: int, max_prediction: int, sessions: int,
                 warmup: int, ticks: int, threads: int, seed: int):
    """CPU 'port' baseline: wall seconds for `ticks` ticks of `sessions` reference sessions."""
    ne = ctypes.c_int32()
    t = load().orc_bench_exgame(num_players, check_distance, input_delay, max_prediction, sessions, warmup, ticks,
                                threads, seed, ctypes.byref(ne))
    return t, ne.value


def bench_exgame_soa(num_players: int, check_distance: int, input_delay: int, max_prediction: int, sessions: int,
                     warmup: int, ticks: int, threads: int, seed: int):
    """CPU 'optimized' baseline (oracle/soa_baseline.cpp: no per-request allocation,
    closed-form fletcher16, cache-blocked sessions): wall seconds of `ticks` ticks."""
    ne = ctypes.c_int32()
    t = load().orc_bench_exgame_soa(num_players, check_distance, input_delay, max_prediction, sessions, warmup, ticks,
                                    threads, seed, ctypes.byref(ne))
    return t, ne.value


def soa_exgame_run(num_players: int, check_distance: int, input_delay: int, max_prediction: int, inputs,
                   threads: int = 2):
    """The optimized baseline's results after len(inputs) ticks from frame 0 (TEST ONLY):
    (live states [S, P, 5] f32 as x, y, vx, vy, rot; Game::last_checksum [S] u16; errors)."""
    T, P, S = inputs.shape
    a = np.ascontiguousarray(inputs, np.uint8)
    st = np.zeros((S, P, 5), np.float32)
    cs = np.zeros(S, np.uint16)
    ne = load().orc_soa_exgame_run(P, check_distance, input_delay, max_prediction, S, T, threads, _ptr(a), _ptr(st),
                                   _ptr(cs))
    return st, cs, ne


def bench_brawler(num_players: int, check_distance: int, input_delay: int, max_prediction: int, sessions: int,
                  warmup: int, ticks: int, threads: int, seed: int):
    """CPU 'port' baseline for the brawler (BASELINE config 3): wall seconds."""
    ne = ctypes.c_int32()
    t = load().orc_bench_brawler(num_players, check_distance, input_delay, max_prediction, sessions, warmup, ticks,
                                 threads, seed, ctypes.byref(ne))
    return t, ne.value


def wire_encode(ref: bytes, inputs) -> bytes:
    """compression.rs encode: XOR delta of every input against ref, then bitfield RLE (TEST ONLY)."""
    r = np.frombuffer(bytes(ref), np.uint8)
    a = np.ascontiguousarray(np.asarray(inputs, np.uint8).reshape(-1, r.size))
    out = np.zeros(16 + 2 * a.size + 8, np.uint8)
    n = load().orc_wire_encode(_ptr(r), r.size, _ptr(a) if a.size else None, a.shape[0], _ptr(out), out.size)
    assert n >= 0
    return out[:n].tobytes()


def wire_decode(ref: bytes, data: bytes, cap: int = 4096):
    """compression.rs decode; None when malformed (the reference panics) (TEST ONLY)."""
    r = np.frombuffer(bytes(ref), np.uint8)
    d = np.frombuffer(bytes(data) or b"\0", np.uint8)
    out = np.zeros((cap, r.size), np.uint8)
    n = load().orc_wire_decode(_ptr(r), r.size, _ptr(d), len(data), _ptr(out), cap)
    if n == -1:
        return None
    assert n >= 0
    return out[:n]


def bench_p2p_exgame(P: int, W: int, delay: int, local_mask: int, remote_delay: int, inputs, upto, remote_in,
                     warmup: int, threads: int, game: int = EX_GAME):
    """CPU 'port' baseline of the P2P rollback path on the given synthetic
    network arrays: (wall seconds of ticks [warmup, T), AdvanceFrames executed, errors)."""
    T, _, S = inputs.shape
    a = np.ascontiguousarray(inputs, np.uint8)
    u = np.ascontiguousarray(upto, np.int32)
    r = np.ascontiguousarray(remote_in, np.uint8)
    adv = np.zeros(1, np.int64)
    ne = np.zeros(1, np.int32)
    fn = load().orc_bench_p2p_brawler if game == BRAWLER else load().orc_bench_p2p_exgame
    t = fn(P, W, delay, local_mask, remote_delay, S, T, warmup, threads, _ptr(a), _ptr(u), _ptr(r), r.shape[0],
           _ptr(adv), _ptr(ne))
    return t, int(adv[0]), int(ne[0])
