"""Two-player match harness. Behavioural contract: the reference's
``interface/TestPlay.py:15-155`` (and the older ``interface/Play.py:5-35``) — player1 is black,
the game ends at two consecutive passes with WHITE to move, the ASCII board format of
``showboard`` and the area score of ``calculate_score``.

Structure here: the game loop is a generator of moves (``moves()``) that the public
``play`` / ``playover`` methods drain; the board is rendered from a numpy glyph grid
(``render_board``); the score is computed for the whole board at once from a padded
neighbour stack (``area_score``) instead of a per-point eye test.
"""
import numpy as np

from ..engine.gamestate import BLACK, EMPTY, WHITE, GameState

AXIS = "abcdefghijklmnopqrstuvwxy"
RESULT = "DBW"

_OFF = 2           # off-board marker in the padded board
_STARS = (3, 9, 15)  # 19x19 hoshi rows / columns


def eyeish_owner(board):
    """[S, S] int8: BLACK / WHITE where an empty point's on-board neighbours all have that
    colour (the single-point ``is_eyeish`` rule), else 0 — for the whole board at once."""
    board = np.asarray(board, np.int8)
    pad = np.pad(board, 1, constant_values=_OFF)
    nbrs = np.stack([pad[:-2, 1:-1], pad[2:, 1:-1], pad[1:-1, :-2], pad[1:-1, 2:]])
    owner = np.zeros_like(board)
    for c in (BLACK, WHITE):  # black first, as the reference's elif chain
        surrounded = np.all((nbrs == c) | (nbrs == _OFF), axis=0)
        owner[(board == EMPTY) & surrounded & (owner == 0)] = c
    return owner


def area_score(state):
    """(white, black): stones + eyeish empties, komi to white, each side's passes deducted."""
    board = np.asarray(state.board)
    own = np.concatenate([board.ravel(), eyeish_owner(board).ravel()])
    white = float(np.count_nonzero(own == WHITE)) + state.komi - state.passes_white
    black = float(np.count_nonzero(own == BLACK)) - state.passes_black
    return white, black


def render_board(state, finished=False, score=None):
    """The showboard text: axis letters around a grid of x / o stones (B / W marks the last
    move), '+' on 19x19 star points, the last move after the first row and the result after
    the third once the game is finished."""
    S = state.size
    board = np.asarray(state.board)
    glyph = np.full((S, S), ".", dtype="<U1")
    if S == 19:
        glyph[np.ix_(_STARS, _STARS)] = "+"
    glyph[board == BLACK] = "x"
    glyph[board == WHITE] = "o"
    last = state.history[-1] if state.history else None
    if last is not None and glyph[last] in "xo":
        glyph[last] = "B" if glyph[last] == "x" else "W"
    axis = list(AXIS[:S])
    rows = [[" "] + axis + [" "]]
    rows += [[axis[r]] + list(glyph[:, r]) + [axis[r]] for r in range(S)]
    rows.append(rows[0])
    text = [" ".join(r) + " " for r in rows]
    if state.history:
        mover = "W" if state.current_player == BLACK and not finished else "B"
        where = "tt" if last is None else AXIS[last[0]] + AXIS[last[1]]
        text[1] += "    ;%s(%s)" % (mover, where)
    if finished and len(text) > 3:
        winner = state.get_winner()
        sw, sb = score if score is not None else area_score(state)
        verdict = "Winner: %s" % RESULT[winner] if winner else "Draw"
        text[3] += "    %s (W: %s, B: %s)" % (verdict, sw, sb)
    return "\n".join(text)


class PlayMatch(object):
    """Alternating ``get_move`` between two players on one GameState."""

    def __init__(self, player1, player2, save_dir=None, size=19, komi=7.5):
        self.player1, self.player2 = player1, player2
        self.save_dir = save_dir
        self.komi = komi
        self.size = size
        self.clear(showboard=False)

    @property
    def current(self):
        """The player to move (player1 = black)."""
        return self._players[self._turn & 1]

    @property
    def opponent(self):
        return self._players[(self._turn + 1) & 1]

    def clear(self, showboard=True):
        self.state = GameState(size=self.size, komi=self.komi)
        self._players = (self.player1, self.player2)
        self._turn = 0
        self.playout = False
        if showboard:
            self.showboard()

    def _finished_now(self):
        h = self.state.history
        return len(h) >= 2 and h[-1] is None and h[-2] is None and \
            self.state.current_player == WHITE

    def moves(self, limit=None):
        """Generator: plays one move per step (yielding it) until the game is over or
        ``limit`` moves were played."""
        played = 0
        while not self.playout and (limit is None or played < limit):
            mv = self.current.get_move(self.state)
            self.state.do_move(mv)
            played += 1
            if self._finished_now():
                self.playout = True  # the player who ended the game stays "current"
            else:
                self._turn += 1
            yield mv

    def _play(self):
        for _ in self.moves(limit=1):
            pass
        return self.playout

    def play(self, showboard=True):
        """One move by the player to move; True once the game is over."""
        for _ in self.moves(limit=1):
            pass
        if showboard:
            self.showboard()
        return self.playout

    def playover(self, turn=300, showboard=True):
        """Up to ``turn`` moves per side, or until the game ends."""
        for _ in self.moves(limit=2 * turn):
            pass
        if showboard:
            self.showboard()
        return self.playout

    def calculate_score(self):
        """(score_white, score_black) — see ``area_score``."""
        return area_score(self.state)

    def board_string(self):
        return render_board(self.state, self.playout)

    def showboard(self):
        print(self.board_string())


# reference class name
play_match = PlayMatch
