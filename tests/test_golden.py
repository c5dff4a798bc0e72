"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture byte for byte, and the fixtures obey
the properties the reference's own tests state (request-stream shapes of
tests/test_synctest_session.rs, frame == tick + 1, the random-checksum stub's
MismatchedChecksum, GameStub's arithmetic).  The GPU twin is
tests/test_gpu_golden.py.
"""
import glob
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden.make_golden import CASES, run_case

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


def load(name):
    with np.load(os.path.join(HERE, "golden", f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_every_case_has_a_fixture():
    assert {os.path.basename(p)[:-4] for p in FIXTURES} == set(CASES)


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_reproduces_fixture(name):
    want = load(name)
    got = run_case(*CASES[name])
    for k, v in want.items():
        np.testing.assert_array_equal(got[k], v, err_msg=f"{name}:{k}")


@pytest.mark.parametrize("name", ["exgame_p2_cd7_d2", "stub_cd7_d2", "stub_enum_cd7_d2", "exgame_p4_cd7_d2"])
def test_fixture_request_stream_shape_cd7(name):
    # tests/test_synctest_session.rs:68-85: cd=7, delay 2, every tick advances;
    # [Save(c), Adv] for c <= 7, then Load(c-7) + 7x[Save, Adv] + Adv.
    z = load(name)
    T = z["kinds"].shape[0]
    assert (z["err_kinds"] == 0).all()
    for t in range(T):
        k = z["kinds"][t][z["kinds"][t] >= 0].tolist()
        f = z["frames"][t][: len(k)].tolist()
        if t <= 7:
            assert list(zip(k, f)) == [(0, t), (2, t)]
        else:
            assert k == [1, 2] + [0, 2] * 7
            assert f[0] == t - 7 and f[-2:] == [t, t]
    frames = z["live"][:, :, 0:4].copy().view(np.int32)[..., 0]
    np.testing.assert_array_equal(frames, np.arange(1, T + 1)[:, None].repeat(frames.shape[1], 1))


def test_fixture_stub_cd2_shape():
    # tests/test_synctest_session.rs:35-65: 2 requests for i <= 2, then exactly Load, Adv, Save, Adv, Save, Adv
    z = load("stub_cd2_d0")
    for t in range(z["kinds"].shape[0]):
        k = z["kinds"][t][z["kinds"][t] >= 0].tolist()
        assert k == ([0, 2] if t <= 2 else [1, 2, 0, 2, 0, 2])


def test_fixture_stub_arithmetic():
    # stubs.rs:115-125 with both handles fed input i at tick i: p0 + p1 is even
    # every frame (blank for the delayed frames 0, 1), so state == 2 * frame; the
    # cell checksum is DefaultHasher (SipHash-1-3, keys 0) of (frame, state).
    z = load("stub_cd7_d2")
    img = z["live"][:, 0, :].copy().view(np.int32)
    np.testing.assert_array_equal(img[:, 1], 2 * img[:, 0])
    for w, fr in enumerate(z["cell_frames"]):
        st = z["cells"][w, 0].copy().view(np.int32)
        assert st[0] == fr and st[1] == 2 * fr
        msg = np.array([fr, 2 * fr], np.int32).tobytes()
        assert int(z["cell_cs"][w, 0, 0]) == O.siphash(1, 3, 0, 0, msg)
        assert int(z["cell_cs"][w, 0, 1]) == 0


def test_fixture_random_checksum_mismatch():
    # tests/test_synctest_session.rs:87-103 (#[should_panic]): with cd=2 the first
    # re-saved frame (2) is compared at tick 4 and every later call fails the same way.
    z = load("stub_random_cs_cd2_d2")
    assert (z["err_kinds"][:4] == 0).all()
    assert (z["err_kinds"][4:] == 3).all() and (z["err_frames"][4:] == 2).all()


def test_fixture_exgame_display_checksum_is_fletcher16_of_live_image():
    # ex_game.rs:104-108: last_checksum = fletcher16(bincode(state)) after every advance.
    z = load("exgame_p2_cd7_d2")
    for t in (0, 7, 8, 150, 299):
        for s in range(z["live"].shape[1]):
            assert int(z["display_cs"][t, s]) == O.fletcher16(z["live"][t, s].tobytes())
            assert z["display_frame"][t, s] == t + 1
