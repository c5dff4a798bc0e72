"""The HIP path (through the C ABI) against the committed golden fixtures,
tick by tick: request streams, errors, live state images and display
checksums, and the final snapshot cells, all bit-exact.  The random-checksum
stub's values are the engine's own counter-based draw (the reference uses
thread_rng), so only its MismatchedChecksum frames are compared."""
import os

import numpy as np
import pytest

import ggrs_amd as G
from tests.golden.make_golden import CASES

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GAME = {1: G.Game.EX_GAME, 2: G.Game.STUB, 3: G.Game.STUB_ENUM, 4: G.Game.STUB_RANDOM_CS}


def load(name):
    with np.load(os.path.join(HERE, "golden", f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("fused", [False, True], ids=["per_tick", "run_ticks"])
def test_hip_path_matches_golden(gpu_available, name, fused):
    z = load(name)
    game, P, W, cd, d, S, T, seed = (int(x) for x in z["meta"])
    g = GAME[game]
    random_cs = g == G.Game.STUB_RANDOM_CS
    sess = (G.SessionBuilder(g, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
            .with_check_distance(cd).with_input_delay(d).with_seed(seed).start_synctest_session())
    inputs = z["inputs"]
    if fused and not random_cs:
        done = sess.run_ticks(inputs)
        assert done == T
        t_checked = [T - 1]
    else:
        t_checked = range(T)
    for t in (t_checked if not fused or random_cs else []):
        for h in range(P):
            sess.add_local_input(h, inputs[t, h])
        if (z["err_kinds"][t] == 3).any():
            with pytest.raises(G.MismatchedChecksum) as ei:
                sess.advance_frame()
            np.testing.assert_array_equal(ei.value.frames, np.where(z["err_kinds"][t] == 3, z["err_frames"][t], -1))
            continue
        reqs = sess.advance_frame()
        n = int((z["kinds"][t] >= 0).sum())
        assert [(int(r.kind), r.frame) for r in reqs] == list(zip(z["kinds"][t, :n].tolist(), z["frames"][t, :n].tolist()))
        if random_cs:
            continue
        img, dcs, dfr = sess.read_live()
        np.testing.assert_array_equal(img, z["live"][t], err_msg=f"{name} live state, tick {t}")
        if g == G.Game.EX_GAME:
            np.testing.assert_array_equal(dcs, z["display_cs"][t], err_msg=f"{name} display checksum, tick {t}")
            np.testing.assert_array_equal(dfr, z["display_frame"][t])
    if random_cs:
        return
    t = T - 1
    img, dcs, _ = sess.read_live()
    np.testing.assert_array_equal(img, z["live"][t])
    n = int((z["kinds"][t] >= 0).sum())
    assert [(int(r.kind), r.frame) for r in sess.last_requests()] == list(
        zip(z["kinds"][t, :n].tolist(), z["frames"][t, :n].tolist()))
    for w, fr in enumerate(z["cell_frames"]):
        if fr < 0:
            continue
        gi, gc = sess.read_cell(int(fr))
        np.testing.assert_array_equal(gi, z["cells"][w], err_msg=f"{name} cell {fr}")
        np.testing.assert_array_equal(gc, z["cell_cs"][w], err_msg=f"{name} cell checksum {fr}")
    sess.close()
