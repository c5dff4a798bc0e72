"""GPU parity for BASELINE config 3: the fixed-point 256-entity brawler.

The reference has no such game; its definition is
oracle/ggrs_oracle.hpp namespace brawler (sequential, entity order) and the
device restatement is ggrs_amd/csrc/games.hpp Brawler (one wavefront per
session).  Integer-only: state images, checksums, request streams and
mismatch frames are all asserted bit-exact.
"""
import numpy as np
import pytest

import ggrs_amd as G
from ggrs_amd.synth import synth_inputs
from oracle import oracle as O
from test_gpu_parity import compare_cells, compare_live, make_pair, run_parity

pytestmark = pytest.mark.gpu

B = G.Game.BRAWLER
MASK = 0x1F  # UP, DOWN, LEFT, RIGHT, ATTACK


@pytest.mark.parametrize("P,W,cd,d", [(2, 8, 7, 2), (1, 8, 3, 0), (3, 8, 5, 1), (4, 8, 7, 2), (2, 8, 0, 0),
                                      (4, 12, 11, 3)])
def test_brawler_parity_every_tick(gpu_available, P, W, cd, d):
    S, T = 48, 40
    run_parity(B, S, P, W, cd, d, T, synth_inputs(S, P, T, seed=31, mask=MASK), check_every=3)


def test_brawler_parity_long_run_contacts(gpu_available):
    # long enough for AI entities to reach the players: damage, kills, player hits
    S, P, T = 40, 4, 300
    inputs = synth_inputs(S, P, T, seed=5, mask=MASK)
    run_parity(B, S, P, 8, 7, 2, T, inputs, check_every=50)


@pytest.mark.parametrize("P,cd,d", [(2, 7, 2), (4, 7, 0), (3, 2, 1)])
def test_brawler_run_ticks_fused_parity(gpu_available, P, cd, d):
    import torch
    S, T = 72, 90
    inputs = synth_inputs(S, P, T, seed=9, mask=0xFF)
    sess, orc = make_pair(B, S, P, 8, cd, d)
    dev = torch.from_numpy(inputs).cuda()
    t = 0
    for chunk in (5, 1, 30, 54):
        n = min(chunk, T - t)
        assert sess.run_ticks(dev[t:t + n]) == n
        for k in range(t, t + n):
            for h in range(P):
                orc.add_local_input(h, inputs[k, h])
            kinds, _ = orc.advance()
            assert (kinds == 0).all()
        t += n
        assert [(int(r.kind), r.frame) for r in sess.last_requests()] == orc.trace(0)
        compare_cells(sess, orc, P, B)
        compare_live(sess, orc, B)
    assert t == T


@pytest.mark.parametrize("word,mask", [(0, 0x1), (8 * 200 + 4, 0x40), (8 * 63 + 6, 0x80000000)])
def test_brawler_corruption_detected_like_oracle(gpu_available, word, mask):
    S, P, cd, T = 64, 2, 7, 30
    inputs = synth_inputs(S, P, T, seed=21, mask=MASK)
    sess, orc = make_pair(B, S, P, 8, cd, 2)
    victims = [0, 17, 63]
    for t in range(T):
        if t == 12:
            f = sess.current_frame() - cd
            for v in victims:
                sess.debug_corrupt_cell(v, f, word, mask)
                orc.corrupt_cell(v, f, word, mask)
        for h in range(P):
            sess.add_local_input(h, inputs[t, h])
            orc.add_local_input(h, inputs[t, h])
        kinds, frames = orc.advance()
        if (kinds != 0).any():
            with pytest.raises(G.MismatchedChecksum) as ei:
                sess.advance_frame()
            np.testing.assert_array_equal(ei.value.frames, np.where(kinds == 3, frames, -1))
        else:
            sess.advance_frame()
    assert list(np.nonzero(sess.mismatches() != -1)[0]) == victims
    compare_live(sess, orc, B)


def test_brawler_bench_config_sampled_parity(gpu_available):
    """BASELINE config 3 at bench size (65,536 sessions, 4 GiB snapshot ring):
    no session mismatches, and a sample is bit-exact with the oracle."""
    import torch
    S, P, T = 65536, 2, 24
    inputs = synth_inputs(S, P, T, mask=0xFF)
    sess = (G.SessionBuilder(B, num_sessions=S).with_num_players(P).with_check_distance(7)
            .with_input_delay(2).with_checked_mismatches(False).start_synctest_session())
    dev = torch.from_numpy(inputs).cuda()
    assert sess.run_ticks(dev) == T
    assert (sess.mismatches() == -1).all()
    rng = np.random.default_rng(1)
    sample = np.sort(rng.choice(S, 16, replace=False))
    orc = O.OracleBatch(O.BRAWLER, P, 8, 7, 2, sample.size)
    for t in range(T):
        for h in range(P):
            orc.add_local_input(h, inputs[t, h, sample])
        k, _ = orc.advance()
        assert (k == 0).all()
    gimg, _, _ = sess.read_live()
    oimg, _, _ = orc.read_live()
    np.testing.assert_array_equal(gimg[sample], oimg)
    frames, oc, _, ocs = orc.read_cells()
    for w, fr in enumerate(frames):
        gi, gc = sess.read_cell(int(fr))
        np.testing.assert_array_equal(gi[sample], oc[w])
        np.testing.assert_array_equal(gc[sample], ocs[w])
    sess.close()
