"""ctypes binding of libggrs_amd.so (include/ggrs_amd.h).

The shared library is built in-tree by ``ggrs_amd/csrc/Makefile`` (see
``__graft_entry__.build``).  There is no fallback: importing this module
without the library raises, so nothing can silently run on the CPU.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# GGRS_AMD_LIB: load another build of the same library (kernel experiments, tools/)
LIB_PATH = os.environ.get("GGRS_AMD_LIB") or os.path.join(_HERE, "libggrs_amd.so")

RB_ABI_VERSION = 1
RB_NULL_FRAME = -1

# rb_status
RB_OK = 0
RB_PREDICTION_THRESHOLD = 1
RB_INVALID_REQUEST = 2
RB_MISMATCHED_CHECKSUM = 3
RB_NOT_SYNCHRONIZED = 4
RB_SPECTATOR_TOO_FAR_BEHIND = 5
RB_DEVICE_ERROR = 100
RB_PANIC = 101

# rb_game
RB_GAME_EX_GAME = 1
RB_GAME_STUB = 2
RB_GAME_STUB_ENUM = 3
RB_GAME_STUB_RANDOM_CS = 4
RB_GAME_BRAWLER = 5

RB_FLAG_CHECKED = 1
RB_FLAG_LANE_PER_SESSION = 2
RB_P2P_FLAG_FANOUT = 4
RB_P2P_FLAG_PEER_STATUS = 8
RB_P2P_FLAG_FANOUT_ALWAYS = 16
RB_P2P_FLAG_FANOUT_PER_PLAYER = 32
RB_GAME_PLUGIN_BASE = 1000
RB_P2P_REPORTS_PER_TAKE = 8
RB_P2P_EVENTS_KEPT = 16


class RbConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("game", ctypes.c_int32),
        ("num_sessions", ctypes.c_int32),
        ("num_players", ctypes.c_int32),
        ("max_prediction", ctypes.c_int32),
        ("check_distance", ctypes.c_int32),
        ("input_delay", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("flags", ctypes.c_uint32),
        ("block_size", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32 * 6),
    ]


class RbP2PConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("game", ctypes.c_int32),
        ("num_sessions", ctypes.c_int32),
        ("num_players", ctypes.c_int32),
        ("max_prediction", ctypes.c_int32),
        ("input_delay", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("local_mask", ctypes.c_uint32),
        ("remote_delay", ctypes.c_int32),
        ("sparse_saving", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("block_size", ctypes.c_uint32),
        ("desync_interval", ctypes.c_int32),
        ("fanout_candidates", ctypes.c_int32),
        ("fanout_min_select_permille", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32 * 1),
    ]


class RbChecksumReport(ctypes.Structure):
    _fields_ = [
        ("checksum_lo", ctypes.c_uint64),
        ("checksum_hi", ctypes.c_uint64),
        ("frame", ctypes.c_int32),
        ("mismatch_frame", ctypes.c_int32),
    ]


# Every symbol declared in include/ggrs_amd.h: (name, restype, argtypes).
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PU64 = ctypes.POINTER(ctypes.c_uint64)
SIGNATURES = [
    ("rb_config_init", None, [ctypes.POINTER(RbConfig)]),
    ("rb_synctest_create", _I32, [ctypes.POINTER(RbConfig), ctypes.POINTER(_P)]),
    ("rb_destroy", None, [_P]),
    ("rb_last_error", ctypes.c_char_p, [_P]),
    ("rb_set_stream", _I32, [_P, _P]),
    ("rb_get_stream", _P, [_P]),
    ("rb_add_local_input", _I32, [_P, _I32, _P, _I32]),
    ("rb_add_local_inputs_packed", _I32, [_P, _P, _I32]),
    ("rb_advance_frame", _I32, [_P]),
    ("rb_run_ticks", _I32, [_P, _I32, _P, ctypes.c_int64, _I32, _PI32]),
    ("rb_current_frame", _I32, [_P]),
    ("rb_num_sessions", _I32, [_P]),
    ("rb_state_bytes", _I32, [_P]),
    ("rb_input_bytes", _I32, [_P]),
    ("rb_synchronize", _I32, [_P]),
    ("rb_mismatches", _I32, [_P, _PI32, _PI32]),
    ("rb_last_requests", _I32, [_P, _PI32, _PI32, _I32]),
    ("rb_read_cell", _I32, [_P, _I32, _P, _PU64]),
    ("rb_read_live", _I32, [_P, _P, _PU64, _PI32]),
    ("rb_export_checksum_report", _I32, [_P, _I32, _P]),
    ("rb_export_compact_report", _I32, [_P, _I32, _P]),
    ("rb_p2p_fanout_state", _I32, [_P, _PI32, ctypes.POINTER(ctypes.c_double), _PI32, _PI32]),
    ("rb_debug_corrupt_cell", _I32, [_P, _I32, _I32, _I32, ctypes.c_uint32]),
    ("rb_debug_sincosf", _I32, [_I32, _P, _P, _P, ctypes.c_int64]),
    ("rb_debug_speed_clamp", _I32, [_I32, _P, _P, _P, _P, ctypes.c_int64]),
    ("rb_debug_exgame_inrange", _I32, [_I32, ctypes.c_uint32, ctypes.c_int64, _P]),
    ("rb_profile_enable", _I32, [_P, _I32]),
    ("rb_profile_take", _I32, [_P, ctypes.POINTER(ctypes.c_double), _PI32]),
    ("rb_launch_clock_arm", _I32, [_P, _I32]),
    ("rb_launch_clock_read", _I32, [_P, _PU64, _I32, _PI32]),
    ("rb_register_game_plugin", _I32, [ctypes.c_char_p, _PI32]),
    ("rb_p2p_config_init", None, [ctypes.POINTER(RbP2PConfig)]),
    ("rb_p2p_create", _I32, [ctypes.POINTER(RbP2PConfig), ctypes.POINTER(_P)]),
    ("rb_p2p_destroy", None, [_P]),
    ("rb_p2p_last_error", ctypes.c_char_p, [_P]),
    ("rb_p2p_set_stream", _I32, [_P, _P]),
    ("rb_p2p_get_stream", _P, [_P]),
    ("rb_p2p_run_ticks", _I32, [_P, _I32, _P, ctypes.c_int64, _P, _P, _I32]),
    ("rb_p2p_run_ticks_packets", _I32, [_P, _I32, _P, ctypes.c_int64, _P, ctypes.c_int64, _P, _P, _P, _P]),
    ("rb_p2p_read_status", _I32, [_P, _P, _P, _P, _P]),
    ("rb_p2p_disconnect_player", _I32, [_P, _I32, _P]),
    ("rb_p2p_read_frames", _I32, [_P, _P, _P]),
    ("rb_p2p_read_queues", _I32, [_P, _P]),
    ("rb_p2p_read_cells", _I32, [_P, _P, _P, _P]),
    ("rb_p2p_read_live", _I32, [_P, _P]),
    ("rb_p2p_state_bytes", _I32, [_P]),
    ("rb_p2p_input_bytes", _I32, [_P]),
    ("rb_p2p_counters", _I32, [_P, _P]),
    ("rb_p2p_totals", _I32, [_P, _P]),
    ("rb_p2p_take_checksum_reports", _I32, [_P, _P]),
    ("rb_p2p_receive_checksum_reports", _I32, [_P, _I32, _P, _I32]),
    ("rb_p2p_read_desync_events", _I32, [_P, _P, _P, _P, _P, _P]),
    ("rb_p2p_debug_corrupt", _I32, [_P, _I32, _I32, ctypes.c_uint32]),
    ("rb_p2p_receive_peer_connect_status", _I32, [_P, _I32, _P, _P]),
    ("rb_p2p_profile_enable", _I32, [_P, _I32]),
    ("rb_p2p_profile_take", _I32, [_P, ctypes.POINTER(ctypes.c_double), _PI32]),
    ("rb_p2p_launch_clock_arm", _I32, [_P, _I32]),
    ("rb_p2p_launch_clock_read", _I32, [_P, _PU64, _I32, _PI32]),
    ("rb_decode_input_packets", _I32, [_I32, _P, _I32, _I32, _I32, _I32, _I32, _P, ctypes.c_int64, _P, _P, _P, _I32,
                                        _P, _P]),
    ("rb_encode_input_packets", _I32, [_I32, _P, _I32, _I32, _I32, _I32, _P, _I32, _I32, _P, _P, _P, ctypes.c_int64,
                                        _P, _P]),
]

_lib = None


def load() -> ctypes.CDLL:
    """Load the HIP engine library; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C ggrs_amd/csrc` "
            "(or __graft_entry__.build()); the engine has no CPU fallback."
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        if os.environ.get("GGRS_AMD_LIB") and not hasattr(lib, name):
            continue  # an older experiment build may lack newer entry points
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
