"""The CPU oracle, pinned against the reference's own known-answer tests and
published vectors (no GPU).  See oracle/ggrs_oracle.hpp header."""
import os
import subprocess

import numpy as np

from oracle import oracle as O
from ggrs_amd.synth import synth_inputs


def test_restated_reference_tests_pass():
    # oracle/ref_tests.cpp restates every KAT of frame_info.rs, input_queue.rs,
    # sync_layer.rs, tests/test_synctest_session*.rs (+ fletcher16/SipHash vectors).
    r = subprocess.run([O.REF_TESTS], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fail=0" in r.stdout
    assert r.stdout.count("PASS") >= 20


def test_fletcher16_wikipedia_vectors():
    assert O.fletcher16(b"abcde") == 0xC8F0
    assert O.fletcher16(b"abcdef") == 0x2057
    assert O.fletcher16(b"abcdefgh") == 0x0627


def _siphash24_python(msg: bytes) -> int:
    """CPython 3.10 hashes bytes with SipHash-2-4; PYTHONHASHSEED=0 gives a zero key."""
    code = f"import sys; sys.stdout.write(str(hash({msg!r}) & 0xFFFFFFFFFFFFFFFF))"
    env = dict(os.environ, PYTHONHASHSEED="0")
    return int(subprocess.check_output(["python3", "-c", code], env=env))


def test_siphash_core_matches_cpython_siphash24():
    # Independent implementation of the same SipHash core (c=2, d=4, key 0):
    # pins the round function and finalisation the c=1, d=3 DefaultHasher uses.
    import sys
    if sys.hash_info.algorithm != "siphash24":
        import pytest
        pytest.skip("interpreter does not use siphash24")
    for msg in [b"\x01", b"abcdefg", b"abcdefgh", bytes(range(8)), bytes(range(15)), b"x" * 23]:
        ours = O.siphash(2, 4, 0, 0, msg)
        theirs = _siphash24_python(msg)
        if theirs == 0xFFFFFFFFFFFFFFFE and ours == 0xFFFFFFFFFFFFFFFF:  # CPython maps -1 -> -2
            continue
        assert ours == theirs, msg


def test_synth_generator_c_and_numpy_agree():
    for (S, P, T, f0) in [(37, 2, 50, 0), (5, 4, 20, 11)]:
        a = synth_inputs(S, P, T, first_frame=f0)
        b = O.synth_inputs(0x67677273, 0x0F, S, P, T, f0, 1)
        np.testing.assert_array_equal(a, b)
    a = synth_inputs(9, 2, 30, mask=0xFFFFFFFF, dtype=np.uint32)
    b = O.synth_inputs(0x67677273, 0xFFFFFFFF, 9, 2, 30, 0, 4)
    np.testing.assert_array_equal(a, b)


def test_oracle_request_stream_cd7_delay2():
    # steady-state stream at cd=7 is Load + 7 Saves + 8 Advances.
    b = O.OracleBatch(O.EX_GAME, 2, 8, 7, 2, 3)
    for i in range(20):
        b.add_local_input(0, i % 16)
        b.add_local_input(1, (i * 3) % 16)
        k, f = b.advance()
        assert (k == 0).all()
        tr = b.trace(0)
        if i <= 7:
            assert tr == [(0, i), (2, i)]
        else:
            assert len(tr) == 16
            assert tr[0] == (1, i - 7)
            assert [t[0] for t in tr[1:]] == [2] + [0, 2] * 7
    assert b.current_frame() == 20


def test_oracle_random_checksum_stub_mismatch_frame():
    # tests/test_synctest_session.rs:87-103: random checksums must fail; with
    # cd=2 the first comparable re-save is frame 2, reported at tick 4.
    b = O.OracleBatch(O.STUB_RANDOM_CS, 2, 8, 2, 2, 4, seed=7)
    for i in range(10):
        b.add_local_input(0, i)
        b.add_local_input(1, i)
        k, f = b.advance()
        if i < 4:
            assert (k == 0).all()
        else:
            assert (k == 3).all() and (f == 2).all()
            break


def test_oracle_exgame_state_new_and_bincode_image():
    b = O.OracleBatch(O.EX_GAME, 2, 8, 2, 0, 1)
    img, cs, fr = b.read_live()
    assert img.shape == (1, 76)
    f = np.frombuffer(img[0].tobytes(), np.uint8)
    assert int.from_bytes(f[4:12].tobytes(), "little") == 2  # num_players
    pos = f[20:36].view(np.float32)
    assert np.allclose(pos, [450.0, 400.0, 150.0, 400.0], atol=1e-3)


def test_oracle_brawler_synctest_runs_and_exercises_the_rules():
    # BASELINE config 3 (no reference game; oracle/ggrs_oracle.hpp brawler):
    # deterministic resimulation never mismatches, and over 300 frames the AI
    # reaches the players (damage both ways), so every rule is exercised.
    S, P, T = 12, 4, 300
    inputs = synth_inputs(S, P, T, seed=5, mask=0x1F)
    b = O.OracleBatch(O.BRAWLER, P, 8, 7, 2, S)
    img, _, _ = b.read_live()
    assert img.shape == (S, 4 + 256 * 32)
    for t in range(T):
        for h in range(P):
            b.add_local_input(h, inputs[t, h])
        k, _ = b.advance()
        assert (k == 0).all(), t
    img, _, _ = b.read_live()
    ent = img[:, 4:].copy().view(np.int32).reshape(S, 256, 8)
    assert (img[:, :4].copy().view(np.int32) == T).all()
    assert (ent[:, :, 0] >= 0).all() and (ent[:, :, 0] < (1 << 20)).all()
    assert (ent[:, :P, 7] > 0).any(), "no player took damage"
    assert (ent[:, P:, 4] < 100).any(), "no AI entity took damage"
    assert (ent[:, P:, 7] > 0).all() or (ent[:, P:, 4] <= 0).any()


def test_speed_clamp_compare_without_sqrt():
    # games.hpp ExGame::advance_player tests `vx*vx + vy*vy > 49` where the
    # reference tests `sqrt(vx*vx + vy*vy) > 7` (ex_game.rs:300-304).  f32 sqrt
    # is correctly rounded (numpy too), so check the equivalence on every float
    # in [40, 60) and on a log-uniform sample of the whole range.
    lo, hi = np.float32(40.0).view(np.uint32), np.float32(60.0).view(np.uint32)
    m2 = np.arange(lo, hi, dtype=np.uint32).view(np.float32)
    rng = np.random.default_rng(7)
    m2 = np.concatenate([m2, rng.integers(0, 0x7F800000, 1 << 20, dtype=np.uint32).view(np.float32),
                         np.array([0.0, 49.0, np.inf, np.nan], np.float32)])
    with np.errstate(invalid="ignore"):
        assert ((np.sqrt(m2) > np.float32(7.0)) == (m2 > np.float32(49.0))).all()


def test_sincos_quadrant_f32_equals_glibc_reduction(tmp_path):
    # device_math.hpp sincosf_glibc<kInRange> takes glibc's reduce_fast quadrant
    # from one f32 fma on [0, 6.5) (the range games.hpp ExGame::in_range admits):
    # checked here for every float of that range (about 4 s).
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "check_sincos_quadrant.c")
    exe = str(tmp_path / "check_sincos_quadrant")
    subprocess.run(["gcc", "-O2", "-o", exe, src, "-lm"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert r.stdout.startswith("1087373312 floats, 0 mismatches")


def test_sincos_in_range_evaluation_equals_glibc(tmp_path):
    # device_math.hpp sincosf_glibc<kInRange> (f32 quadrant, no tiny-argument
    # branch) against this host's glibc sinf/cosf for every float in [+0, 6.5)
    # (OpenMP, a few seconds on 8 cores).
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "check_sincos_inrange.c")
    exe = str(tmp_path / "check_sincos_inrange")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-o", exe, src, "-lm"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert r.stdout.startswith("1087373312 floats, 0 mismatches")


def test_optimized_cpu_baseline_matches_oracle():
    # bench.py's second CPU baseline (oracle/soa_baseline.cpp, kind "optimized")
    # must do the same work as the port: same live states and display checksums
    # as the oracle's SyncTestSession + ex_game after T ticks, no mismatches.
    from ggrs_amd.session import decode_ex_game
    for P, cd, d, W, T in [(2, 7, 2, 8, 260), (3, 2, 0, 8, 90), (4, 7, 2, 8, 150), (2, 0, 1, 8, 40), (1, 5, 3, 9, 70)]:
        S = 37
        inputs = synth_inputs(S, P, T)
        st, cs, ne = O.soa_exgame_run(P, cd, d, W, inputs)
        assert ne == 0
        b = O.OracleBatch(O.EX_GAME, P, W, cd, d, S)
        for t in range(T):
            for h in range(P):
                b.add_local_input(h, inputs[t, h])
            k, _ = b.advance()
            assert (k == 0).all()
        img, ocs, _ = b.read_live()
        f = decode_ex_game(img, P)
        want = np.concatenate([f["positions"], f["velocities"], f["rotations"][..., None]], -1)
        np.testing.assert_array_equal(st.view(np.uint32), want.astype(np.float32).view(np.uint32))
        np.testing.assert_array_equal(cs.astype(np.uint64), ocs)


def _exgame_canon(v):
    """ggrs_amd/csrc/games.hpp ExGame::canon_input: the fan-out's input class."""
    up, down, left, right = v & 1, (v >> 1) & 1, (v >> 2) & 1, (v >> 3) & 1
    return (0 if up == down else (1 if up else 2)) | (0 if left == right else (4 if left else 8))


def test_exgame_input_classes_move_players_alike():
    """The in-kernel fan-out presimulates one branch per input class
    (p2p.hpp InputCanon): every input must act on the state exactly as its
    class representative does.  Two oracle batches (the restated
    ex_game.rs:259-321), one fed random inputs and one fed their
    representatives, stay bit-identical through hundreds of frames (speed
    clamps, wraps and all), and the 16 inputs fall into 9 classes."""
    assert len({_exgame_canon(v) for v in range(16)}) == 9
    S, P, T = 256, 2, 300
    rng = np.random.default_rng(7)
    ins = rng.integers(0, 16, (T, P, S)).astype(np.uint8)
    rep = np.vectorize(_exgame_canon)(ins).astype(np.uint8)
    a = O.OracleBatch(O.EX_GAME, P, 8, 7, 2, S)
    b = O.OracleBatch(O.EX_GAME, P, 8, 7, 2, S)
    for t in range(T):
        for h in range(P):
            a.add_local_input(h, ins[t, h])
            b.add_local_input(h, rep[t, h])
        ka, _ = a.advance()
        kb, _ = b.advance()
        assert (ka == 0).all() and (kb == 0).all()
        if t % 50 == 49:
            np.testing.assert_array_equal(a.read_live()[0], b.read_live()[0])
    fa, ia, _, ca = a.read_cells()
    fb, ib, _, cb = b.read_cells()
    np.testing.assert_array_equal(ia, ib)
    np.testing.assert_array_equal(ca, cb)
