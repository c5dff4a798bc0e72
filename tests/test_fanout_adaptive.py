"""The adaptive speculative fan-out (include/ggrs_amd.h RB_P2P_FLAG_FANOUT_ALWAYS,
VERDICT r04 item 6): a batch measures, over windows of 64 ticks, the fraction of
its rollbacks that became branch selects and pauses the presimulation while it is
below the threshold.  Whether it presimulates never changes a result: the batch
equals a plain rollback batch on the same inputs (cells, states, queues, frames)."""
import numpy as np
import pytest

import ggrs_amd as G
from ggrs_amd.p2p import PlayerType, synth_network

pytestmark = pytest.mark.gpu
W, D, RD = 8, 2, 2


def batch(game, P, S, fanout, **kw):
    kw.setdefault("per_player", False)  # the one-player form (the default for ex_game is per player)
    b = (G.SessionBuilder(game, num_sessions=S).with_num_players(P).with_max_prediction_window(W)
         .with_input_delay(D).with_remote_input_delay(RD).with_speculative_fanout(fanout, 16, **kw))
    for h in range(P):
        b.add_player(PlayerType.Local if h == 0 else PlayerType.Remote, h)
    return b.start_p2p_session()


def same(a, b):
    np.testing.assert_array_equal(a.read_live(), b.read_live())
    for x, y in zip(a.read_cells(), b.read_cells()):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a.read_queues(), b.read_queues())


def drive(sessions, di, du, dr, T, tpl):
    import torch
    for t0 in range(0, T, tpl):
        for s in sessions:
            s.run_ticks(di[t0:t0 + tpl], du[t0:t0 + tpl], dr)
        torch.cuda.synchronize()  # (lets each measurement land before the next call decides)


@pytest.mark.parametrize("tpl", [1, 16])
def test_gpu_brawler_fanout_turns_itself_off(gpu_available, tpl):
    """The brawler's 256-value inputs: its 16 candidates rarely hold the next input (3.8% of
    rollbacks in the bench line), so after one window the batch stops presimulating."""
    import torch
    P, S, T = 2, 128, 160
    inputs, upto, rin = synth_network(S, P, T, 0b1, RD, 1, 4, mask=0xFF)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    fan, plain = batch(G.Game.BRAWLER, P, S, True), batch(G.Game.BRAWLER, P, S, False)
    drive([fan, plain], di, du, dr, T, tpl)
    active, frac, windows, off = fan.fanout_state()
    assert windows >= 1 and off == 1 and not active, (active, frac, windows, off)
    assert 0.0 <= frac < 0.15
    same(fan, plain)
    tf, tp = fan.totals(), plain.totals()
    assert tf[2] + tf[3] == tp[2]  # every rollback a load or a select
    assert 0 < tf[4] < 16 * T * S  # branch frames: presimulated in the first window only


def test_gpu_exgame_c4_fanout_stays_on_and_a_high_threshold_pauses_it(gpu_available):
    """ex_game at P = 4 (C4): about a third of rollbacks become selects, above the default 15%, so
    the fan-out stays on; with the threshold at 100% the same batch pauses it.  Both equal plain."""
    import torch
    P, S, T, tpl = 4, 256, 200, 25
    inputs, upto, rin = synth_network(S, P, T, 0b1, RD, 1, 4)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    on = batch(G.Game.EX_GAME, P, S, True)
    strict = batch(G.Game.EX_GAME, P, S, True, min_select_permille=1000)
    always = batch(G.Game.EX_GAME, P, S, True, adaptive=False)
    plain = batch(G.Game.EX_GAME, P, S, False)
    drive([on, strict, always, plain], di, du, dr, T, tpl)
    a, frac, windows, off = on.fanout_state()
    assert a and off == 0 and windows >= 2 and frac >= 0.15, (a, frac, windows, off)
    a2, frac2, _, off2 = strict.fanout_state()
    assert not a2 and off2 >= 1 and frac2 < 1.0
    assert always.fanout_state()[0]
    for x in (on, strict, always):
        same(x, plain)
        assert x.totals()[2] + x.totals()[3] == plain.totals()[2]
    assert strict.totals()[4] < always.totals()[4]  # the paused batch presimulated fewer branch frames


def test_gpu_fanout_pause_and_resume_equals_plain(gpu_available):
    """a paused fan-out leaves the branch metadata and the move-to-front lists as they
    were; presimulation restarts after 960 plain ticks.  The branch rows are invalidated when it
    stops and when it restarts, so the first ticks after the resume select only branches made
    after it.  1,200 ticks: a window, a pause, the resumed window and the second pause, each tick
    equal to a plain rollback batch; branch frames are presimulated again after the resume, and
    the decisions fall at the same ticks in two identical batches (no race with the measurement)."""
    import torch
    P, S, T, tpl = 4, 256, 1200, 25
    inputs, upto, rin = synth_network(S, P, T, 0b1, RD, 1, 4)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    strict = batch(G.Game.EX_GAME, P, S, True, min_select_permille=1000)
    twin = batch(G.Game.EX_GAME, P, S, True, min_select_permille=1000)
    plain = batch(G.Game.EX_GAME, P, S, False)
    branch_at = {}
    for t0 in range(0, T, tpl):
        for s in (strict, twin, plain):
            s.run_ticks(di[t0:t0 + tpl], du[t0:t0 + tpl], dr)  # no synchronisation: decisions must not race
        if t0 + tpl in (1000, T):
            branch_at[t0 + tpl] = strict.totals()[4]
            assert strict.fanout_state() == twin.fanout_state()
        if t0 % 200 == 0:
            same(strict, plain)
    same(strict, plain)
    same(twin, plain)
    a, frac, windows, off = strict.fanout_state()
    assert off >= 2 and windows >= 2, (a, frac, windows, off)
    assert branch_at[T] > branch_at[1000], branch_at  # presimulated again after the resume
    assert strict.totals() == twin.totals()
    assert strict.totals()[2] + strict.totals()[3] == plain.totals()[2]
    assert strict.totals()[3] > 0


def test_gpu_brawler_fanout_branch_slots_above_4g_words(gpu_available):
    """the brawler's branch cells are [W][32 planes][Spad x 64 lanes x 16 branches]
    words; at 32,768 sessions one slot is 2^30 words, so a 32-bit slot offset wraps from slot 4 on.
    The offsets are 64-bit now: with the fan-out always on, a batch of that size equals plain
    rollback (cells, live states, queues) and selects branches."""
    import torch
    P, S, T = 2, 32768, 24
    inputs, upto, rin = synth_network(S, P, T, 0b1, RD, 1, 4, mask=0xFF)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    fan = batch(G.Game.BRAWLER, P, S, True, adaptive=False)
    plain = batch(G.Game.BRAWLER, P, S, False)
    for t0 in range(0, T, 4):
        for s in (fan, plain):
            s.run_ticks(di[t0:t0 + 4], du[t0:t0 + 4], dr)
    torch.cuda.synchronize()
    same(fan, plain)
    tf, tp = fan.totals(), plain.totals()
    assert tf[3] > 0, tf  # selects happened, so branch cells of every slot were read back
    assert tf[2] + tf[3] == tp[2]
    fan.close()
    plain.close()


def test_gpu_default_fanout_is_per_player_for_ex_game(gpu_available):
    """with_speculative_fanout's default for a game whose players move independently (ex_game, K
    covering its alphabet) is the per-player form; it equals plain rollback and selects more
    rollbacks than the one-player form on the same inputs."""
    import torch
    P, S, T, tpl = 4, 256, 120, 20
    inputs, upto, rin = synth_network(S, P, T, 0b1, RD, 1, 4)
    di, du, dr = (torch.from_numpy(a).cuda() for a in (inputs, upto, rin))
    auto = batch(G.Game.EX_GAME, P, S, True, per_player=None, adaptive=False)
    one = batch(G.Game.EX_GAME, P, S, True, adaptive=False)
    plain = batch(G.Game.EX_GAME, P, S, False)
    drive([auto, one, plain], di, du, dr, T, tpl)
    same(auto, plain)
    same(one, plain)
    ta, to, tp = auto.totals(), one.totals(), plain.totals()
    assert ta[2] + ta[3] == tp[2] and to[2] + to[3] == tp[2]
    assert ta[3] > to[3] > 0, (ta, to)  # selects: per player > one player
