"""Host logic without a GPU: the C-ABI library loads and exports every symbol
include/ggrs_amd.h declares, and the batch's host bookkeeping (plan-only
batches, device=-1) produces the reference's request stream and errors."""
import ctypes
import itertools
import os
import re

import numpy as np
import pytest

import ggrs_amd as G
from ggrs_amd import _lib as L
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "ggrs_amd.h")).read()
    declared = set(re.findall(r"^(?:void|int32_t|rb_status|const char\s*\*)\s*\*?\s*(rb_[a-z0-9_]+)\s*\(", hdr, re.M))
    assert len(declared) >= 20
    lib = ctypes.CDLL(L.LIB_PATH)
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert declared == {name for name, _, _ in L.SIGNATURES}


def test_config_defaults_match_builder():
    cfg = L.RbConfig()
    L.load().rb_config_init(ctypes.byref(cfg))
    assert (cfg.num_players, cfg.max_prediction, cfg.check_distance, cfg.input_delay) == (2, 8, 2, 0)


def _plan(game=G.Game.STUB, S=4, P=2, W=8, cd=2, d=0):
    b = G.SessionBuilder(game, num_sessions=S, device=-1).with_num_players(P).with_check_distance(cd).with_input_delay(d)
    b.with_max_prediction_window(W)
    return b.start_synctest_session()


@pytest.mark.parametrize("W,cd,d", [(8, 0, 0), (8, 1, 0), (8, 2, 0), (8, 7, 2), (9, 8, 0), (1, 0, 3),
                                     (4, 3, 1), (16, 9, 5), (64, 63, 0), (2, 1, 7)])
def test_plan_request_stream_equals_oracle(W, cd, d):
    # tests/test_synctest_session.rs:35-65 generalised: the host bookkeeping
    # emits exactly the reference's Vec<GGRSRequest> every tick.
    sess = _plan(W=W, cd=cd, d=d)
    orc = O.OracleBatch(O.STUB, 2, W, cd, d, 1)
    for i in range(3 * W + 20):
        for h in (0, 1):
            sess.add_local_input(h, i)
            orc.add_local_input(h, i)
        reqs = sess.advance_frame()
        k, _ = orc.advance()
        assert k[0] == 0
        assert [(int(r.kind), r.frame) for r in reqs] == orc.trace(0), i
        assert sess.current_frame() == orc.current_frame() == i + 1


def test_plan_reference_shapes_cd0_and_cd2():
    s = _plan(cd=0)
    for i in range(20):
        s.add_local_input(0, i)
        s.add_local_input(1, i)
        assert len(s.advance_frame()) == 1  # test_synctest_session.rs:15-32
    s = _plan(cd=2)
    for i in range(20):
        s.add_local_input(0, i)
        s.add_local_input(1, i)
        r = s.advance_frame()
        kinds = [x.kind for x in r]
        K = G.RequestKind
        if i <= 2:
            assert kinds == [K.SaveGameState, K.AdvanceFrame]
        else:
            assert kinds == [K.LoadGameState, K.AdvanceFrame, K.SaveGameState, K.AdvanceFrame,
                             K.SaveGameState, K.AdvanceFrame]


def test_builder_validation_errors():
    with pytest.raises(G.InvalidRequest, match="Check distance too big."):
        _plan(W=8, cd=8)
    with pytest.raises(G.InvalidRequest, match="prediction windows above 0"):
        G.SessionBuilder(G.Game.STUB, device=-1).with_max_prediction_window(0)
    with pytest.raises(G.InvalidRequest):
        G.SessionBuilder(G.Game.EX_GAME, device=-1).with_num_players(5).start_synctest_session()


def test_invalid_handle_and_missing_input():
    s = _plan()
    with pytest.raises(G.InvalidRequest, match="player handle you provided is not valid"):
        s.add_local_input(2, 0)
    s.add_local_input(0, 1)
    with pytest.raises(G.InvalidRequest, match="Missing local input"):
        s.advance_frame()
    s.add_local_input(1, 1)  # the earlier input for handle 0 is still registered
    assert len(s.advance_frame()) == 2
    # inputs are consumed by a successful advance
    with pytest.raises(G.InvalidRequest, match="Missing local input"):
        s.advance_frame()


def test_plan_matches_oracle_errors_for_missing_input_mid_game():
    s = _plan(cd=3, d=1)
    orc = O.OracleBatch(O.STUB, 2, 8, 3, 1, 1)
    for i in range(12):
        s.add_local_input(0, i)
        orc.add_local_input(0, i)
        if i % 4 == 3:  # forget handle 1 once, then supply it
            with pytest.raises(G.InvalidRequest):
                s.advance_frame()
            k, _ = orc.advance()
            assert k[0] == 2  # InvalidRequest
        s.add_local_input(1, i)
        orc.add_local_input(1, i)
        r = s.advance_frame()
        k, _ = orc.advance()
        assert k[0] == 0
        assert [(int(x.kind), x.frame) for x in r] == orc.trace(0)


def test_p2p_create_rejects_fanout_planes_beyond_int_offsets():
    """a fan-out batch whose branch planes would need more than 2^31 words per
    snapshot slot is refused at create (no GPU needed: the check runs before any allocation)."""
    import pytest

    import ggrs_amd as G
    from ggrs_amd.p2p import PlayerType
    b = (G.SessionBuilder(G.Game.BRAWLER, num_sessions=65536 + 64).with_num_players(2)
         .with_speculative_fanout(True, 16))
    for h in range(2):
        b.add_player(PlayerType.Local if h == 0 else PlayerType.Remote, h)
    with pytest.raises(G.InvalidRequest, match="31-bit branch-plane"):
        b.start_p2p_session()
