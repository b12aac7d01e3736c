"""Monte Carlo tree search with the reference's exact semantics — reference AlphaGo/mcts.py.

``TreeNode`` / ``MCTS`` reproduce the reference arithmetic (mcts.py:11-216), including its
documented quirks (Q4): the same-signed leaf value is backed up to every ancestor, ``u`` is only
refreshed when a node itself is updated, rollouts are greedy (argmax of the rollout policy), and
the chosen move is the most-visited child. These semantics are pinned by tests/test_mcts.py.

The production search is ``ParallelMCTS`` (search/apv.py): the native multi-threaded APV-MCTS
with virtual loss, negamax backup and batched GPU leaf evaluation.
"""
from operator import itemgetter

import numpy as np


class TreeNode(object):
    """Node with running-mean value Q, prior P and visit-adjusted prior score u."""

    def __init__(self, parent, prior_p):
        self._parent = parent
        self._children = {}
        self._n_visits = 0
        self._Q = 0
        self._u = prior_p
        self._P = prior_p

    def expand(self, action_priors):
        for action, prob in action_priors:
            if action not in self._children:
                self._children[action] = TreeNode(self, prob)

    def select(self):
        """(action, child) maximising Q + u; ties go to the first child in insertion order."""
        return max(self._children.items(), key=lambda act_node: act_node[1].get_value())

    def update(self, leaf_value, c_puct):
        self._n_visits += 1
        self._Q += (leaf_value - self._Q) / self._n_visits
        if not self.is_root():
            self._u = c_puct * self._P * np.sqrt(self._parent._n_visits) / (1 + self._n_visits)

    def update_recursive(self, leaf_value, c_puct):
        """update() applied root-first so parent visit counts are current."""
        if self._parent:
            self._parent.update_recursive(leaf_value, c_puct)
        self.update(leaf_value, c_puct)

    def get_value(self):
        return self._Q + self._u

    def is_leaf(self):
        return self._children == {}

    def is_root(self):
        return self._parent is None


class MCTS(object):
    """Single-threaded MCTS (reference mcts.py:79-216)."""

    def __init__(self, value_fn, policy_fn, rollout_policy_fn, lmbda=0.5, c_puct=5,
                 rollout_limit=500, playout_depth=20, n_playout=10000):
        self._root = TreeNode(None, 1.0)
        self._value = value_fn
        self._policy = policy_fn
        self._rollout = rollout_policy_fn
        self._lmbda = lmbda
        self._c_puct = c_puct
        self._rollout_limit = rollout_limit
        self._L = playout_depth
        self._n_playout = n_playout

    def _playout(self, state, leaf_depth):
        node = self._root
        for i in range(leaf_depth):
            if node.is_leaf():
                action_probs = list(self._policy(state))
                if len(action_probs) == 0:
                    break
                node.expand(action_probs)
            action, node = node.select()
            state.do_move(action)
        v = self._value(state) if self._lmbda < 1 else 0
        z = self._evaluate_rollout(state, self._rollout_limit) if self._lmbda > 0 else 0
        leaf_value = (1 - self._lmbda) * v + self._lmbda * z
        node.update_recursive(leaf_value, self._c_puct)

    def _evaluate_rollout(self, state, limit):
        player = state.get_current_player()
        for i in range(limit):
            action_probs = list(self._rollout(state))
            if len(action_probs) == 0:
                break
            max_action = max(action_probs, key=itemgetter(1))[0]
            state.do_move(max_action)
        else:
            print("WARNING: rollout reached move limit")
        winner = state.get_winner()
        if winner == 0:
            return 0
        return 1 if winner == player else -1

    def get_move(self, state):
        for n in range(self._n_playout):
            state_copy = state.copy()
            self._playout(state_copy, self._L)
        return max(self._root._children.items(), key=lambda act_node: act_node[1]._n_visits)[0]

    def update_with_move(self, last_move):
        if last_move in self._root._children:
            self._root = self._root._children[last_move]
            self._root._parent = None
        else:
            self._root = TreeNode(None, 1.0)
