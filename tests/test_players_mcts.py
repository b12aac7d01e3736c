"""Players and reference-semantics MCTS (spec: reference tests/test_players.py, test_policy.py
player cases, tests/test_mcts.py)."""
from operator import itemgetter

import numpy as np
import pytest

from rocalphago_amd.engine import BLACK, GameState
from rocalphago_amd.models.policy import CNNPolicy
from rocalphago_amd.players.ai import GreedyPolicyPlayer, ProbabilisticPolicyPlayer
from rocalphago_amd.search.mcts import MCTS, TreeNode


def entropy(d):
    d = np.asarray(d).flatten()
    return -np.dot(np.log(d), d)


def test_temperature_changes_entropy():
    lo = ProbabilisticPolicyPlayer(None, temperature=0.9)
    hi = ProbabilisticPolicyPlayer(None, temperature=1.1)
    d = np.random.random(361)
    d /= d.sum()
    assert entropy(hi.apply_temperature(d)) > entropy(d) > entropy(lo.apply_temperature(d))


def test_extreme_temperatures_are_stable():
    d = np.random.random(361)
    d /= d.sum()
    for t in (1e-12, 1e12):
        assert not np.any(np.isnan(ProbabilisticPolicyPlayer(None, temperature=t)
                                   .apply_temperature(d)))


@pytest.fixture(scope="module")
def tiny_policy():
    return CNNPolicy(["board", "ones", "turns_since"], layers=2, filters_per_layer=8,
                     device="cpu")


@pytest.mark.parametrize("cls", [GreedyPolicyPlayer, ProbabilisticPolicyPlayer])
def test_players_play_twenty_moves(tiny_policy, cls):
    gs = GameState()
    player = cls(tiny_policy)
    for _ in range(20):
        mv = player.get_move(gs)
        assert mv is not None
        gs.do_move(mv)


@pytest.mark.parametrize("cls", [GreedyPolicyPlayer, ProbabilisticPolicyPlayer])
def test_players_pass_when_only_own_eye_left(tiny_policy, cls):
    gs = GameState()
    for x in range(19):
        for y in range(19):
            if (x, y) != (10, 10):
                gs.do_move((x, y), BLACK)
    gs.current_player = BLACK
    assert cls(tiny_policy).get_move(gs) is None


def test_batched_get_moves_and_move_limit(tiny_policy):
    p = ProbabilisticPolicyPlayer(tiny_policy, move_limit=None)
    states = [GameState() for _ in range(3)]
    moves = p.get_moves(states)
    assert all(m is not None for m in moves)  # quirk Q6 fixed: None = no limit
    p2 = ProbabilisticPolicyPlayer(tiny_policy, move_limit=0)
    states[0].do_move((3, 3))
    assert p2.get_moves(states[:1]) == [None]
    g = GreedyPolicyPlayer(tiny_policy)
    assert len(g.get_moves(states)) == 3


# ---------------------------------------------------------------- reference-semantics MCTS
dummy_distribution = np.arange(361, dtype=np.float64)
dummy_distribution = dummy_distribution / dummy_distribution.sum()


def dummy_policy(state):
    moves = state.get_legal_moves(include_eyes=False)
    return list(zip(moves, dummy_distribution))


def dummy_value(state):
    return 0.0


def test_selection_and_expansion():
    node = TreeNode(None, 1.0)
    node.expand(dummy_policy(GameState()))
    assert len(node._children) == 361
    action, child = node.select()
    assert action == (18, 18) and child is not None
    for a, p in dummy_policy(GameState()):
        assert node._children[a]._P == p


def test_update_arithmetic():
    node = TreeNode(None, 1.0)
    node.expand(dummy_policy(GameState()))
    child = node._children[(18, 18)]
    node.update(1.0, 5.0)
    child.update(1.0, 5.0)
    assert child.get_value() == 1.0 + 5.0 * dummy_distribution[-1] * 0.5
    node.update(0.0, 5.0)
    child.update(0.0, 5.0)
    assert child.get_value() == 0.5 + 5.0 * dummy_distribution[-1] * np.sqrt(2.0) / 3.0


def test_update_recursive_matches():
    node = TreeNode(None, 1.0)
    node.expand(dummy_policy(GameState()))
    child = node._children[(18, 18)]
    child.update_recursive(1.0, 5.0)
    assert child.get_value() == 1.0 + 5.0 * dummy_distribution[-1] / 2.0
    child.update_recursive(0.0, 5.0)
    assert child.get_value() == 0.5 + 5.0 * dummy_distribution[-1] * np.sqrt(2.0) / 3.0


def _expansions(mcts):
    node = mcts._root
    n = 0
    for action, _ in sorted(dummy_policy(GameState()), key=itemgetter(1), reverse=True):
        if action in node._children:
            n += 1
            node = node._children[action]
        else:
            break
    return n


def test_playout_depth():
    m = MCTS(dummy_value, dummy_policy, dummy_policy, n_playout=2)
    m._playout(GameState().copy(), 8)
    assert m._root._children[(18, 18)]._n_visits == 1
    assert _expansions(m) == 8


def test_playout_stops_at_game_end():
    def stop_early(state):
        return dummy_policy(state) if len(state.history) <= 4 else []
    m = MCTS(dummy_value, stop_early, stop_early, n_playout=2)
    m._playout(GameState().copy(), 8)
    assert m._root._children[(18, 18)]._n_visits == 1
    assert _expansions(m) == 5


def test_get_move_and_tree_reuse():
    gs = GameState()
    m = MCTS(dummy_value, dummy_policy, dummy_policy, n_playout=2)
    move = m.get_move(gs)
    gs.do_move(move)
    m.update_with_move(move)
    assert len(m._root._children) > 0
    assert m._root._parent is None
    assert m._root.select()[0] == (18, 17)
