"""Feature planes (spec: reference tests/test_preprocessing.py, preprocessing.py:14-294)."""
import numpy as np
import pytest

from rocalphago_amd.engine import BLACK, EMPTY, WHITE, GameState
from rocalphago_amd.features.preprocessing import (DEFAULT_FEATURES, FEATURES, VALUE_FEATURES,
                                                   Preprocess)

from boards import parse


def ko_board():
    """7x7; white to move; black just captured at (4,3) creating a ko; ladder shape top-left."""
    gs = GameState(size=7)
    for m in [(0, 0), (1, 0), (0, 1), (1, 1), (0, 2), (3, 4), (3, 3), (4, 5), (4, 2), (5, 4),
              (5, 3), (4, 3), (4, 4)]:
        gs.do_move(m)
    return gs


def self_atari_board():
    gs = GameState(size=7)
    for p in [(2, 4), (4, 4), (6, 0)]:
        gs.do_move(p, BLACK)
    for p in [(1, 0), (5, 0), (2, 3), (4, 3), (1, 4), (5, 4), (2, 5), (3, 5), (4, 5)]:
        gs.do_move(p, WHITE)
    return gs


def capture_board():
    gs = GameState(size=7)
    for p in [(2, 0), (3, 0), (1, 1), (4, 1), (1, 2), (2, 3), (5, 4), (6, 5), (5, 6)]:
        gs.do_move(p, BLACK)
    for p in [(2, 1), (3, 1), (2, 2), (4, 4), (3, 5), (5, 5), (4, 6)]:
        gs.do_move(p, WHITE)
    gs.current_player = BLACK
    return gs


def planes(gs, name):
    """(S, S, F) view of one feature, as the reference tests index it."""
    return Preprocess([name]).state_to_tensor(gs)[0].transpose((1, 2, 0))


def test_registry_sizes():
    assert Preprocess(DEFAULT_FEATURES).output_dim == 48
    assert Preprocess(VALUE_FEATURES).output_dim == 49
    assert {k: v["size"] for k, v in FEATURES.items()}["liberties_after"] == 8
    with pytest.raises(ValueError):
        Preprocess(["not_a_feature"])
    assert Preprocess(["BOARD"]).output_dim == 3  # names are lower-cased


def test_board_planes_relative_to_player():
    gs = ko_board()
    assert gs.current_player == WHITE
    f = planes(gs, "board")
    assert np.all(f[:, :, 0] == (gs.board == WHITE))
    assert np.all(f[:, :, 1] == (gs.board == BLACK))
    assert np.all(f[:, :, 2] == (gs.board == EMPTY))
    assert f[4, 4, 1] == 1 and f[1, 0, 0] == 1


def test_turns_since_matches_history():
    gs = ko_board()
    f = planes(gs, "turns_since")
    expect = np.zeros((7, 7, 8))
    rev = gs.history[::-1]
    for x in range(7):
        for y in range(7):
            if gs.board[x, y] != EMPTY:
                expect[x, y, min(rev.index((x, y)), 7)] = 1
    assert np.all(f == expect)


def test_liberties_hand_coded():
    f = planes(ko_board(), "liberties")
    e = np.zeros((7, 7, 8))
    e[4, 4, 0] = 1
    e[0, 0:3, 1] = 1
    e[3, 4, 1] = e[5, 4, 1] = 1
    e[1, 0:2, 2] = 1
    e[4, 5, 2] = e[3, 3, 2] = e[5, 3, 2] = 1
    e[4, 2, 3] = 1
    assert np.all(f == e)


def test_liberties_eight_or_more_on_last_plane():
    gs = GameState(9)
    for y in range(9):
        gs.do_move((4, y), BLACK)
    f = planes(gs, "liberties")
    assert f[4, 0, 7] == 1 and f[4, 0, :7].sum() == 0  # 18 liberties


@pytest.mark.parametrize("make", [capture_board, ko_board])
def test_capture_size_brute_force(make):
    gs = make()
    f = planes(gs, "capture_size")
    e = np.zeros((7, 7, 8))
    before = gs.num_white_prisoners + gs.num_black_prisoners
    for (x, y) in gs.get_legal_moves():
        c = gs.copy()
        c.do_move((x, y))
        e[x, y, min(7, c.num_white_prisoners + c.num_black_prisoners - before)] = 1
    assert np.all(f == e)


def test_self_atari_hand_coded():
    f = planes(self_atari_board(), "self_atari_size")
    e = np.zeros((7, 7, 8))
    e[0, 0, 0] = 1
    e[3, 4, 2] = 1
    assert np.all(f == e)
    f = planes(capture_board(), "self_atari_size")
    e = np.zeros((7, 7, 8))
    e[4, 5, 0] = e[3, 6, 0] = 1
    e[6, 6, 2] = 1
    assert np.all(f == e)


@pytest.mark.parametrize("make", [capture_board, ko_board, self_atari_board])
def test_liberties_after_brute_force(make):
    gs = make()
    f = planes(gs, "liberties_after")
    e = np.zeros((7, 7, 8))
    for (x, y) in gs.get_legal_moves():
        c = gs.copy()
        c.do_move((x, y))
        e[x, y, min(c.liberty_counts[x, y] - 1, 7)] = 1
    assert np.all(f == e)


def test_ladder_planes():
    gs, m = parse(". . . . . . .|"
                  "B W a . . . .|"
                  ". B . . . . .|"
                  ". . . . . . .|"
                  ". . . . . . .|"
                  ". . . . . W .|")
    f = Preprocess(["ladder_capture"]).state_to_tensor(gs)[0, 0]
    e = np.zeros((7, 7))
    e[m['a']] = 1
    assert np.all(f == e)
    gs, m = parse(". B B . . . .|"
                  "B W a . . . .|"
                  ". B . . . . .|"
                  ". . . . . W .|"
                  ". . . . . . .|"
                  ". . . . . . .|")
    gs.current_player = WHITE
    f = Preprocess(["ladder_escape"]).state_to_tensor(gs)[0, 0]
    e = np.zeros((7, 7))
    e[m['a']] = 1
    assert np.all(f == e)


def test_sensibleness_and_legal():
    gs = ko_board()
    sens = Preprocess(["sensibleness"]).state_to_tensor(gs)[0, 0]
    leg = Preprocess(["legal"]).state_to_tensor(gs)[0, 0]
    e_s, e_l = np.zeros((7, 7)), np.zeros((7, 7))
    for (x, y) in gs.get_legal_moves():
        e_l[x, y] = 1
        if not gs.is_eye((x, y), WHITE):
            e_s[x, y] = 1
    assert np.all(sens == e_s) and np.all(leg == e_l)
    assert leg[4, 3] == 0  # ko point


def test_concatenation_order():
    gs = ko_board()
    f = Preprocess(["board", "sensibleness", "capture_size"]).state_to_tensor(gs)[0]
    f = f.transpose((1, 2, 0))
    assert f.shape == (7, 7, 12)
    assert np.all(f[:, :, 0] == (gs.board == WHITE))
    assert np.all(f[:, :, 3] == Preprocess(["sensibleness"]).state_to_tensor(gs)[0, 0])
    for (x, y) in gs.get_legal_moves():
        assert f[x, y, 4] == 1  # no captures available on this board


def test_color_plane():
    gs = GameState(5)
    assert np.all(Preprocess(["color"]).state_to_tensor(gs) == 1)
    gs.do_move((0, 0))
    assert np.all(Preprocess(["color"]).state_to_tensor(gs) == 0)


def test_batch_matches_single():
    pp = Preprocess(DEFAULT_FEATURES)
    states = [ko_board(), capture_board(), self_atari_board(), GameState(7)]
    batch = pp.states_to_tensor(states)
    for i, s in enumerate(states):
        assert np.array_equal(batch[i], pp.state_to_tensor(s)[0])
    with pytest.raises(Exception):
        pp.states_to_tensor([GameState(7), GameState(9)])
