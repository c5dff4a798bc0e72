"""User games as plugins (include/ggrs_amd_game.hpp).

The reference lets a user plug any game into the request stream through the
`Config` trait and their own `handle_requests` (lib.rs:240-262,
ex_game.rs:76-84).  Here a game is a header with a struct that follows the
device-handler contract of include/ggrs_amd_game.hpp.  ``build_game_plugin``
compiles it against the engine's kernels (ggrs_amd/csrc/plugin.hip, hipcc,
gfx950) into a shared library; ``register_game_plugin`` loads that library
into the engine and returns the game id to pass to ``SessionBuilder``.

Build plugins ahead of time (like the engine itself): the GPU box runs
prebuilt libraries.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

from . import _lib as L

_CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")


def build_game_plugin(header: str, game: str, out: str) -> str:
    """hipcc the game struct `game` from `header` into the plugin library `out`
    (make -C ggrs_amd/csrc plugin).  Returns `out`."""
    subprocess.run(["make", "-s", "-C", _CSRC, "plugin", f"GAME_HEADER={os.path.abspath(header)}", f"GAME={game}",
                    f"PLUGIN_OUT={os.path.abspath(out)}"], check=True)
    return out


def register_game_plugin(path: str) -> int:
    """rb_register_game_plugin: load a plugin library, return its game id
    (RB_GAME_PLUGIN_BASE + k; the same id for the same path)."""
    from .session import InvalidRequest
    lib = L.load()
    gid = ctypes.c_int32()
    st = lib.rb_register_game_plugin(os.path.abspath(path).encode(), ctypes.byref(gid))
    if st != L.RB_OK:
        raise InvalidRequest((lib.rb_last_error(None) or b"").decode())
    return gid.value
