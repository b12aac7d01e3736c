"""Differential test: the C++ rules engine (through the GameState facade) against the naive
pure-Python oracle in tests/pyoracle.py, on hypothesis-generated random games.
Every ply compares the board, liberty counts, stone ages, ko point, player to move, prisoners,
passes, end-of-game flag, both legal-move lists (sensible and eye moves, in order) and the
area score."""
import os
import random

import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from rocalphago_amd.engine import GameState
from tests.pyoracle import BLACK, WHITE, Oracle


def _compare(o, g, S):
    assert np.array_equal(np.asarray(g.board).reshape(-1), np.array(o.board))
    assert np.array_equal(np.asarray(g.liberty_counts).reshape(-1), np.array(o.liberty_counts()))
    assert np.array_equal(np.asarray(g.stone_ages).reshape(-1), np.array(o.stone_ages()))
    assert (g.ko is None and o.ko is None) or g.ko == divmod(o.ko, S)
    assert g.current_player == o.player
    assert g.num_black_prisoners == o.captured[BLACK]
    assert g.num_white_prisoners == o.captured[WHITE]
    assert (g.passes_black, g.passes_white) == (o.passes[BLACK], o.passes[WHITE])
    assert bool(g.is_end_of_game) == o.end
    non_eye, eyes = o.legal_moves()
    assert g.get_legal_moves(include_eyes=False) == [divmod(p, S) for p in non_eye]
    assert g.get_legal_moves() == [divmod(p, S) for p in non_eye + eyes]
    assert g.get_winner() == o.winner()
    return non_eye, eyes


# RAG_ORACLE_EXAMPLES=300: the longer run (all 300 random games matched when this was written)
@settings(max_examples=int(os.environ.get("RAG_ORACLE_EXAMPLES", "30")), deadline=None)
@given(size=st.sampled_from([5, 7, 9]), seed=st.integers(0, 2 ** 31 - 1),
       superko=st.booleans(), pass_p=st.sampled_from([0.0, 0.03, 0.25]),
       handicap=st.sampled_from([0, 0, 2, 3]))
def test_engine_matches_python_oracle(size, seed, superko, pass_p, handicap):
    rng = random.Random(seed)
    o = Oracle(size, superko=superko)
    g = GameState(size=size, enforce_superko=superko)
    if handicap:
        pts = rng.sample(range(size * size), handicap)
        o.place_handicaps(pts)
        g.place_handicaps([divmod(p, size) for p in pts])
    for _ in range(3 * size * size):
        non_eye, eyes = _compare(o, g, size)
        if o.end:
            break
        cand = non_eye + eyes
        mv = None if not cand or rng.random() < pass_p else rng.choice(cand)
        o.play(mv)
        g.do_move(None if mv is None else divmod(mv, size))
    _compare(o, g, size)
    b, w = o.score()
    assert g.get_score() == (w, b)
