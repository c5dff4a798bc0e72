"""Generate the golden fixtures in tests/golden/ from the CPU oracle.

    python3 tests/golden/make_golden.py

The Rust reference cannot run here (no cargo/rustc, crates not vendored), so
these fixtures come from the oracle/ restatement (pinned by the reference's own
known-answer tests).  They freeze request traces, live state
images, display checksums and snapshot cells of small seeded runs, so a change
to either the oracle or the HIP path that alters any byte is caught
(tests/test_golden.py on CPU, tests/test_gpu_golden.py on the GPU).

Each fixture is an .npz of plain arrays (loaded with allow_pickle=False):
  inputs [T, P, S], kinds/frames [T, 4W+8] (request stream of session 0, -1 padded),
  err_kinds/err_frames [T, S], live [T, S, B], display_cs [T, S], display_frame [T, S],
  cell_frames [W], cells [W, S, B], cell_cs [W, S, 2]
plus meta [game, P, W, cd, delay, S, T, seed].
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from ggrs_amd.synth import synth_inputs  # noqa: E402
from oracle import oracle as O  # noqa: E402

# name: (game, P, W, cd, delay, S, T, input source, seed)
CASES = {
    # BASELINE config 1: ex_game SyncTest, 2 players, check_distance 7, delay 2 (ex_game_synctest.rs:37-41)
    "exgame_p2_cd7_d2": (O.EX_GAME, 2, 8, 7, 2, 3, 300, "synth", 0),
    "exgame_p4_cd7_d2": (O.EX_GAME, 4, 8, 7, 2, 2, 120, "synth", 0),
    "exgame_p2_cd2_d0": (O.EX_GAME, 2, 8, 2, 0, 2, 120, "synth", 0),
    # tests/test_synctest_session.rs:68-85 inputs (input i at tick i), GameStub
    "stub_cd7_d2": (O.STUB, 2, 8, 7, 2, 1, 200, "ramp", 0),
    "stub_cd2_d0": (O.STUB, 2, 8, 2, 0, 1, 60, "ramp", 0),
    # tests/test_synctest_session_enum.rs alternating Val1/Val2
    "stub_enum_cd7_d2": (O.STUB_ENUM, 2, 8, 7, 2, 1, 200, "alt", 0),
    # tests/test_synctest_session.rs:87-103: random checksums -> MismatchedChecksum
    "stub_random_cs_cd2_d2": (O.STUB_RANDOM_CS, 2, 8, 2, 2, 4, 8, "ramp", 11),
}


def make_inputs(game, P, S, T, source):
    if source == "ramp":
        return np.broadcast_to(np.arange(T, dtype=np.uint32)[:, None, None], (T, P, S)).copy()
    if source == "alt":
        return np.broadcast_to((np.arange(T) % 2).astype(np.uint8)[:, None, None], (T, P, S)).copy()
    return synth_inputs(S, P, T)


def run_case(game, P, W, cd, d, S, T, source, seed):
    inputs = make_inputs(game, P, S, T, source)
    orc = O.OracleBatch(game, P, W, cd, d, S, seed)
    cap = 4 * W + 8
    kinds = np.full((T, cap), -1, np.int32)
    frames = np.full((T, cap), -1, np.int32)
    ek = np.zeros((T, S), np.int32)
    ef = np.zeros((T, S), np.int32)
    live = np.zeros((T, S, orc.image_bytes), np.uint8)
    dcs = np.zeros((T, S), np.uint64)
    dfr = np.zeros((T, S), np.int32)
    for t in range(T):
        for h in range(P):
            orc.add_local_input(h, inputs[t, h])
        ek[t], ef[t] = orc.advance()
        tr = orc.trace(0)
        for i, (k, f) in enumerate(tr):
            kinds[t, i], frames[t, i] = k, f
        live[t], dcs[t], dfr[t] = orc.read_live()
    cf, cells, _, ccs = orc.read_cells()
    meta = np.array([game, P, W, cd, d, S, T, seed], np.int64)
    return dict(meta=meta, inputs=inputs, kinds=kinds, frames=frames, err_kinds=ek, err_frames=ef, live=live,
                display_cs=dcs, display_frame=dfr, cell_frames=cf, cells=cells, cell_cs=ccs)


def main():
    for name, case in CASES.items():
        d = run_case(*case)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **d)
        print(f"{name}: {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
