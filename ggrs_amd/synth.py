"""Synthetic input streams, numpy.

``h = splitmix64(seed ^ (s*2^20 + p*2^16 + f))``; frame 0 and, with
probability 1/8 (``h & 7 == 0``), any later frame takes a new value
``(h >> 32) & mask``; otherwise the previous frame's input is held.
The C restatement in oracle/ggrs_oracle.hpp (SynthInput) must agree
(tests/test_oracle.py checks it).
"""
from __future__ import annotations

import numpy as np

SEED = 0x67677273  # "ggrs"
_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x += np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def synth_inputs(num_sessions: int, num_players: int, frames: int, seed: int = SEED, mask: int = 0x0F,
                 first_frame: int = 0, dtype=np.uint8, first_session: int = 0) -> np.ndarray:
    """Inputs for frames [first_frame, first_frame + frames) of global sessions
    [first_session, first_session + num_sessions) as [frames, P, S]."""
    S, P = num_sessions, num_players
    s = np.arange(first_session, first_session + S, dtype=np.uint64)[None, :]
    p = np.arange(P, dtype=np.uint64)[:, None]
    key = (s << np.uint64(20)) + (p << np.uint64(16))  # [P, S]
    out = np.empty((frames, P, S), dtype=dtype)
    prev = np.zeros((P, S), dtype=np.uint64)
    seed = np.uint64(seed)
    for f in range(first_frame + frames):
        h = splitmix64(seed ^ (key + np.uint64(f)))
        new = (h >> np.uint64(32)) & np.uint64(mask)
        if f == 0:
            prev = new
        else:
            prev = np.where((h & np.uint64(7)) == 0, new, prev)
        if f >= first_frame:
            out[f - first_frame] = prev.astype(dtype)
    return out
