"""Single-threaded PUCT search with the reference's numeric semantics (its AlphaGo/mcts.py).

This is the oracle the tests pin, not the production search — that is
``ParallelMCTS`` (search/apv.py): the native multi-threaded APV-MCTS with virtual loss, negamax
backup and batched GPU leaf evaluation.

Semantics kept on purpose (reference mcts.py:11-216):
  * a node's score is ``Q + u``; ``Q`` is the running mean of the values backed up through it and
    ``u = c_puct * P * sqrt(N_parent) / (1 + N)`` is refreshed only when the node itself is
    updated (unvisited siblings keep ``u = P``);
  * the same leaf value (no sign flip per ply) is applied to every node on the path, root first;
  * leaves are expanded with the policy's (move, prior) list on their first visit; rollouts play
    the argmax of the rollout policy; the chosen move is the most visited root child.

Layout: one ``_Forest`` holds every node of a search in parallel lists (parent index, prior,
Q, u, visit count, child table). ``TreeNode`` is a two-field handle onto one slot that exposes the
reference attribute names (``_parent``, ``_children``, ``_P``, ``_Q``, ``_u``, ``_n_visits``) as
properties, so the search itself walks integer indices and the tests still see the node API.
"""
import math
import warnings


class _Forest(object):
    """Parallel-list storage of search nodes; a node is an integer slot."""

    __slots__ = ("parent", "prior", "q", "u", "visits", "kids")

    def __init__(self):
        self.parent, self.prior, self.q, self.u, self.visits, self.kids = [], [], [], [], [], []

    def add(self, parent, prior):
        self.parent.append(parent)
        self.prior.append(prior)
        self.q.append(0)
        self.u.append(prior)
        self.visits.append(0)
        self.kids.append({})
        return len(self.prior) - 1

    def best_child(self, i):
        """(action, slot) of the child with the largest Q + u; the first one inserted wins ties."""
        best = None
        top = None
        for action, c in self.kids[i].items():
            score = self.q[c] + self.u[c]
            if top is None or score > top:
                best, top = (action, c), score
        return best

    def visit(self, i, leaf_value, c_puct):
        n = self.visits[i] + 1
        self.visits[i] = n
        self.q[i] += (leaf_value - self.q[i]) / n
        p = self.parent[i]
        if p >= 0:
            self.u[i] = c_puct * self.prior[i] * math.sqrt(self.visits[p]) / (1 + n)

    def backup(self, i, leaf_value, c_puct):
        path = []
        while i >= 0:
            path.append(i)
            i = self.parent[i]
        for j in reversed(path):  # root first: a child's u sees its parent's new count
            self.visit(j, leaf_value, c_puct)


class TreeNode(object):
    """Handle onto one node of a ``_Forest`` (reference TreeNode interface)."""

    __slots__ = ("_f", "_i")

    def __init__(self, parent, prior_p, _forest=None, _slot=None):
        if _forest is not None:
            self._f, self._i = _forest, _slot
            return
        self._f = parent._f if parent is not None else _Forest()
        self._i = self._f.add(parent._i if parent is not None else -1, prior_p)

    @classmethod
    def _at(cls, forest, slot):
        return cls(None, None, forest, slot)

    # ---- reference attribute names -------------------------------------------------------
    @property
    def _parent(self):
        p = self._f.parent[self._i]
        return None if p < 0 else TreeNode._at(self._f, p)

    @_parent.setter
    def _parent(self, node):
        self._f.parent[self._i] = -1 if node is None else node._i

    @property
    def _children(self):
        return {a: TreeNode._at(self._f, c) for a, c in self._f.kids[self._i].items()}

    @property
    def _P(self):
        return self._f.prior[self._i]

    @property
    def _Q(self):
        return self._f.q[self._i]

    @property
    def _u(self):
        return self._f.u[self._i]

    @property
    def _n_visits(self):
        return self._f.visits[self._i]

    def __eq__(self, other):
        return isinstance(other, TreeNode) and other._f is self._f and other._i == self._i

    def __hash__(self):
        return hash((id(self._f), self._i))

    # ---- reference methods -----------------------------------------------------------------
    def expand(self, action_priors):
        kids = self._f.kids[self._i]
        for action, prob in action_priors:
            if action not in kids:
                kids[action] = self._f.add(self._i, prob)

    def select(self):
        action, slot = self._f.best_child(self._i)
        return action, TreeNode._at(self._f, slot)

    def update(self, leaf_value, c_puct):
        self._f.visit(self._i, leaf_value, c_puct)

    def update_recursive(self, leaf_value, c_puct):
        self._f.backup(self._i, leaf_value, c_puct)

    def get_value(self):
        return self._f.q[self._i] + self._f.u[self._i]

    def is_leaf(self):
        return not self._f.kids[self._i]

    def is_root(self):
        return self._f.parent[self._i] < 0


class MCTS(object):
    """Sequential PUCT search over duck-typed functions (reference MCTS interface):
    ``policy_fn(state)`` / ``rollout_policy_fn(state)`` -> [(move, prior)], ``value_fn(state)``
    -> value for the player to move."""

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
        """Descend up to ``leaf_depth`` plies (expanding leaves on the way), evaluate the
        position reached and back the mixed value up the path. Mutates ``state``."""
        forest, node = self._root._f, self._root._i
        for _ in range(leaf_depth):
            if not forest.kids[node]:
                priors = list(self._policy(state))
                if not priors:
                    break  # the policy has no move: evaluate here
                TreeNode._at(forest, node).expand(priors)
            action, node = forest.best_child(node)
            state.do_move(action)
        lm = self._lmbda
        v = self._value(state) if lm < 1 else 0
        z = self._evaluate_rollout(state, self._rollout_limit) if lm > 0 else 0
        forest.backup(node, (1 - lm) * v + lm * z, self._c_puct)

    def _evaluate_rollout(self, state, limit):
        """Greedy rollout: +1 / -1 / 0 for the player to move at the start."""
        me = state.get_current_player()
        moves = 0
        while moves < limit:
            options = list(self._rollout(state))
            if not options:
                break
            best = options[0]
            for cand in options[1:]:
                if cand[1] > best[1]:
                    best = cand
            state.do_move(best[0])
            moves += 1
        else:
            warnings.warn("rollout stopped at the move limit (%d moves)" % limit)
        winner = state.get_winner()
        return 0 if winner == 0 else (1 if winner == me else -1)

    def get_move(self, state):
        for _ in range(self._n_playout):
            self._playout(state.copy(), self._L)
        forest, root = self._root._f, self._root._i
        best, most = None, -1
        for action, c in forest.kids[root].items():
            if forest.visits[c] > most:
                best, most = action, forest.visits[c]
        return best

    def update_with_move(self, last_move):
        """Keep the subtree below ``last_move`` (tree reuse) or start afresh."""
        kids = self._root._f.kids[self._root._i]
        if last_move in kids:
            self._root = TreeNode._at(self._root._f, kids[last_move])
            self._root._parent = None
        else:
            self._root = TreeNode(None, 1.0)
