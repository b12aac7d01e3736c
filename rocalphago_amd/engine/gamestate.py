"""Python facade of the native Go engine with the reference ``AlphaGo.go`` API.

Reference: AlphaGo/go.py:1-585 (GameState, IllegalMove, WHITE/BLACK/EMPTY/PASS_MOVE).
All rules run in C++ (csrc/engine/go_engine.cpp); this class only converts between the
reference's ``(x, y)`` tuples and flat indices and materialises the python-set views
(``group_sets``/``liberty_sets``) lazily, with the same shared-identity semantics the reference
tests rely on (tests/test_gamestate.py:167-178).

Deliberate fixes of reference quirks:
  Q1  ``copy()`` keeps stone ages, pass counts and the end-of-game flag.
  Q2  assigning ``current_player`` invalidates the legal-move cache.
Kept quirks: Q3 (end of game needs WHITE to move after two passes), Q11, Q12, Q15.
"""
import numpy as np

from .._native import engine as _engine

WHITE = -1
BLACK = +1
EMPTY = 0
PASS_MOVE = None

_rg = _engine()
IllegalMove = _rg.IllegalMove

_ZOBRIST = {}


def _zobrist(size):
    """Seed-0 Zobrist tables generated exactly as the reference does (go.py:57-64)."""
    z = _ZOBRIST.get(size)
    if z is None:
        rng = np.random.RandomState(0)
        white = rng.randint(np.iinfo(np.uint64).max, size=(size, size), dtype='uint64')
        black = rng.randint(np.iinfo(np.uint64).max, size=(size, size), dtype='uint64')
        native = _rg.make_zobrist(np.ascontiguousarray(white.ravel()),
                                  np.ascontiguousarray(black.ravel()))
        z = (white, black, native)
        _ZOBRIST[size] = z
    return z


class GameState(object):
    """State of a game of Go (reference go.py:9)."""

    def __init__(self, size=19, komi=7.5, enforce_superko=False):
        white, black, native = _zobrist(size)
        self._b = _rg.Board(size, komi, enforce_superko, native)
        self.size = size
        self._cache = {}
        self.hash_lookup = {WHITE: white, BLACK: black}

    # ------------------------------------------------------------------ index helpers
    def _flat(self, action):
        if action is PASS_MOVE:
            return -1
        x, y = action
        if x < 0 or y < 0 or x >= self.size or y >= self.size:
            return -3  # off board: never legal
        return x * self.size + y

    def _unflat(self, idx):
        if idx < 0:
            return PASS_MOVE
        return divmod(idx, self.size)

    def _invalidate(self):
        self._cache.clear()

    @classmethod
    def _wrap(cls, board, size, hash_lookup):
        st = GameState.__new__(GameState)
        st._b = board
        st.size = size
        st._cache = {}
        st.hash_lookup = hash_lookup
        return st

    # ------------------------------------------------------------------ attribute surface
    @property
    def native(self):
        """The underlying C++ board (used by batched feature extraction and search)."""
        return self._b

    @property
    def board(self):
        b = self._cache.get("board")
        if b is None:
            b = self._b.board()
            self._cache["board"] = b
        return b

    @property
    def current_player(self):
        return self._b.current_player

    @current_player.setter
    def current_player(self, color):
        self._b.current_player = int(color)
        self._invalidate()

    @property
    def ko(self):
        k = self._b.ko
        return None if k < 0 else divmod(k, self.size)

    @ko.setter
    def ko(self, value):
        self._b.ko = -1 if value is None else self._flat(value)
        self._invalidate()

    @property
    def komi(self):
        return self._b.komi

    @komi.setter
    def komi(self, k):
        self._b.komi = float(k)

    @property
    def enforce_superko(self):
        return self._b.enforce_superko

    @enforce_superko.setter
    def enforce_superko(self, v):
        self._b.enforce_superko = bool(v)
        self._invalidate()

    @property
    def is_end_of_game(self):
        return self._b.end_of_game

    @is_end_of_game.setter
    def is_end_of_game(self, v):
        self._b.end_of_game = bool(v)

    @property
    def history(self):
        h = self._cache.get("history")
        if h is None:
            h = [self._unflat(a) for a in self._b.history]
            self._cache["history"] = h
        return h

    @property
    def handicaps(self):
        return [self._unflat(a) for a in self._b.handicaps]

    @property
    def num_black_prisoners(self):
        return self._b.black_prisoners

    @property
    def num_white_prisoners(self):
        return self._b.white_prisoners

    @property
    def passes_black(self):
        return self._b.passes_black

    @property
    def passes_white(self):
        return self._b.passes_white

    @property
    def current_hash(self):
        return np.uint64(self._b.hash)

    @property
    def previous_hashes(self):
        return set(np.uint64(h) for h in self._b.previous_hashes)

    @property
    def liberty_counts(self):
        lc = self._cache.get("libcounts")
        if lc is None:
            lc = self._b.liberty_counts()
            self._cache["libcounts"] = lc
        return lc

    @property
    def stone_ages(self):
        sa = self._cache.get("ages")
        if sa is None:
            sa = self._b.stone_ages()
            self._cache["ages"] = sa
        return sa

    def _set_views(self):
        """Build reference-style 2-D lists of python sets with shared identity per group."""
        S = self.size
        heads = self._b.group_heads()
        groups = {}
        libs = {}
        group_sets = [[None] * S for _ in range(S)]
        liberty_sets = [[None] * S for _ in range(S)]
        for p in range(S * S):
            x, y = divmod(p, S)
            h = int(heads[p])
            if h < 0:
                group_sets[x][y] = set()
                liberty_sets[x][y] = set(divmod(q, S) for q in self._b.liberty_set(p))
            else:
                if h not in groups:
                    groups[h] = set(divmod(q, S) for q in self._b.group(h))
                    libs[h] = set(divmod(q, S) for q in self._b.liberty_set(h))
                group_sets[x][y] = groups[h]
                liberty_sets[x][y] = libs[h]
        self._cache["group_sets"] = group_sets
        self._cache["liberty_sets"] = liberty_sets

    @property
    def group_sets(self):
        if "group_sets" not in self._cache:
            self._set_views()
        return self._cache["group_sets"]

    @property
    def liberty_sets(self):
        if "liberty_sets" not in self._cache:
            self._set_views()
        return self._cache["liberty_sets"]

    # ------------------------------------------------------------------ reference methods
    def get_group(self, position):
        (x, y) = position
        return self.group_sets[x][y]

    def get_groups_around(self, position):
        gs = self.group_sets
        out = []
        for h in self._b.groups_around(self._flat(position)):
            x, y = divmod(h, self.size)
            out.append(gs[x][y])
        return out

    def _on_board(self, position):
        (x, y) = position
        return x >= 0 and y >= 0 and x < self.size and y < self.size

    def _neighbors(self, position):
        (x, y) = position
        return [xy for xy in [(x - 1, y), (x + 1, y), (x, y - 1), (x, y + 1)]
                if self._on_board(xy)]

    def _diagonals(self, position):
        (x, y) = position
        return [xy for xy in [(x - 1, y - 1), (x + 1, y + 1), (x + 1, y - 1), (x - 1, y + 1)]
                if self._on_board(xy)]

    def copy(self):
        """Full copy (fixes reference quirk Q1: ages/passes/end flag are kept)."""
        return GameState._wrap(self._b.copy(), self.size, self.hash_lookup)

    def is_suicide(self, action):
        return self._b.is_suicide(self._flat(action))

    def is_positional_superko(self, action):
        return self._b.is_positional_superko(self._flat(action))

    def is_legal(self, action):
        return self._b.is_legal(self._flat(action))

    def is_eyeish(self, position, owner):
        return self._b.is_eyeish(self._flat(position), int(owner))

    def is_eye(self, position, owner, stack=None):
        st = [self._flat(p) for p in stack] if stack else []
        return self._b.is_eye(self._flat(position), int(owner), st)

    def is_ladder_capture(self, action, prey=None, remaining_attempts=80):
        pr = -1 if prey is None else self._flat(prey)
        return self._b.is_ladder_capture(self._flat(action), pr, remaining_attempts)

    def is_ladder_escape(self, action, prey=None, remaining_attempts=80):
        pr = -1 if prey is None else self._flat(prey)
        return self._b.is_ladder_escape(self._flat(action), pr, remaining_attempts)

    def _legal_lists(self):
        lm = self._cache.get("legal")
        if lm is None:
            non_eye, eyes = self._b.legal_moves()
            S = self.size
            lm = ([divmod(p, S) for p in non_eye], [divmod(p, S) for p in eyes])
            self._cache["legal"] = lm
        return lm

    def get_legal_moves(self, include_eyes=True):
        non_eye, eyes = self._legal_lists()
        if include_eyes:
            return non_eye + eyes
        return list(non_eye)

    def get_winner(self):
        return self._b.get_winner()

    def get_score(self):
        """(score_white, score_black) exactly as get_winner counts them."""
        return self._b.score()

    def place_handicaps(self, actions):
        if len(self._b.history) > 0:
            raise IllegalMove("Cannot place handicap on a started game")
        self._b.place_handicaps([self._flat(a) for a in actions])
        self._invalidate()

    def get_current_player(self):
        return self._b.current_player

    def do_move(self, action, color=None):
        color = color or self._b.current_player
        try:
            end = self._b.do_move(self._flat(action), int(color))
        except IllegalMove:
            raise IllegalMove(str(action)) from None
        self._cache.clear()
        return end

    def __repr__(self):
        return "GameState(size=%d, moves=%d, to_play=%s)" % (
            self.size, self._b.move_count, "B" if self.current_player == BLACK else "W")
