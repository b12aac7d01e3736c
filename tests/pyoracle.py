"""A deliberately naive pure-Python Go rules oracle for differential tests of the C++ engine
("C++ engine vs. a pure-Python oracle (our own)").

Everything is recomputed from the board by flood fill on every query: no incremental group or
liberty state, no hashing (positional superko compares whole board tuples), so it shares no
structure with csrc/engine. It implements the rule set the engine reproduces from the reference
(AlphaGo/go.py, behaviour summarised in SURVEY §2.1 C02-C14 and quirks Q3, Q11, Q12, Q15):

  * legality: on board, empty, not suicide (a move that captures is never suicide), not the ko
    point, and -- with positional superko -- not recreating an earlier position, a check made
    only for points the mover has played before (or handicap points);
  * captures are resolved neighbour by neighbour (W, E, S, N order: (x-1,y), (x+1,y), (x,y-1),
    (x,y+1)); after each single-stone capture, ko is set if the placed stone is a lone stone
    with exactly one liberty at that moment;
  * stone ages count moves (passes included) since the stone was placed;
  * the game ends after two consecutive passes when WHITE is to move;
  * area score: stones plus single-point eyeish empties; komi and pass counts as in the reference.
"""
EMPTY, BLACK, WHITE = 0, 1, -1


class Oracle(object):
    def __init__(self, size, komi=7.5, superko=False):
        self.S = size
        self.komi = komi
        self.superko = superko
        self.board = [EMPTY] * (size * size)
        self.player = BLACK
        self.ko = None
        self.history = []  # flat points, None = pass
        self.handicaps = []
        self.captured = {BLACK: 0, WHITE: 0}  # stones of that colour taken off the board
        self.passes = {BLACK: 0, WHITE: 0}
        self.placed = {}  # point -> clock when its stone was placed
        self.clock = 0
        self.end = False
        self.positions = set()  # boards after every stone placement (superko)

    # ---- geometry
    def nbrs(self, p):
        S = self.S
        x, y = divmod(p, S)
        out = []
        for ax, ay in ((x - 1, y), (x + 1, y), (x, y - 1), (x, y + 1)):
            if 0 <= ax < S and 0 <= ay < S:
                out.append(ax * S + ay)
        return out

    def diags(self, p):
        S = self.S
        x, y = divmod(p, S)
        out = []
        for ax, ay in ((x - 1, y - 1), (x + 1, y + 1), (x + 1, y - 1), (x - 1, y + 1)):
            if 0 <= ax < S and 0 <= ay < S:
                out.append(ax * S + ay)
        return out

    # ---- groups by flood fill
    def group(self, p, board=None):
        board = self.board if board is None else board
        c = board[p]
        seen, todo = {p}, [p]
        while todo:
            q = todo.pop()
            for n in self.nbrs(q):
                if n not in seen and board[n] == c:
                    seen.add(n)
                    todo.append(n)
        return seen

    def libs(self, stones, board=None):
        board = self.board if board is None else board
        return {n for q in stones for n in self.nbrs(q) if board[n] == EMPTY}

    def liberty_counts(self):
        out = [-1] * len(self.board)
        for p, c in enumerate(self.board):
            if c != EMPTY:
                out[p] = len(self.libs(self.group(p)))
        return out

    def stone_ages(self):
        return [self.clock - self.placed[p] if c != EMPTY else -1
                for p, c in enumerate(self.board)]

    # ---- legality
    def _place(self, board, p, c):
        """Board after c plays p (captures resolved); also the list of (captured group) sets."""
        b = list(board)
        b[p] = c
        taken = []
        for n in self.nbrs(p):
            if b[n] == -c:
                g = self.group(n, b)
                if not self.libs(g, b):
                    for q in g:
                        b[q] = EMPTY
                    taken.append(g)
        return b, taken

    def is_suicide(self, p):
        b, taken = self._place(self.board, p, self.player)
        return not taken and not self.libs(self.group(p, b), b)

    def _superko_scope(self, p):
        if p in self.handicaps:
            return True
        has_h = bool(self.handicaps)
        start = 0 if (not has_h and self.player == BLACK) or (has_h and self.player == WHITE) \
            else 1
        return p in self.history[start::2]

    def is_legal(self, p):
        if p is None:
            return True
        if self.board[p] != EMPTY or self.is_suicide(p) or p == self.ko:
            return False
        if self.superko and self._superko_scope(p):
            b, _ = self._place(self.board, p, self.player)
            if tuple(b) in self.positions:
                return False
        return True

    # ---- eyes
    def is_eyeish(self, p, owner):
        return self.board[p] == EMPTY and all(self.board[n] == owner for n in self.nbrs(p))

    def is_eye(self, p, owner, stack=()):
        if not self.is_eyeish(p, owner):
            return False
        allow = 1 if len(self.nbrs(p)) == 4 else 0
        bad = 0
        for d in self.diags(p):
            if self.board[d] == -owner:
                bad += 1
            elif self.board[d] == EMPTY and d not in stack:
                if not self.is_eye(d, owner, stack + (p,)):
                    bad += 1
            if bad > allow:
                return False
        return True

    def legal_moves(self):
        """(non-eye legal points, own-eye legal points) in flat order."""
        non_eye, eyes = [], []
        for p in range(len(self.board)):
            if self.is_legal(p):
                (eyes if self.is_eye(p, self.player) else non_eye).append(p)
        return non_eye, eyes

    # ---- playing
    def play(self, p):
        c = self.player
        if not self.is_legal(p):
            raise ValueError("illegal move %r" % (p,))
        self.ko = None
        self.clock += 1
        if p is None:
            self.passes[c] += 1
        else:
            self.board[p] = c
            self.placed[p] = self.clock
            for n in self.nbrs(p):
                if self.board[n] != -c:
                    continue
                g = self.group(n)
                if self.libs(g):
                    continue
                for q in g:
                    self.board[q] = EMPTY
                    self.placed.pop(q, None)
                self.captured[-c] += len(g)
                if len(g) == 1:
                    mine = self.group(p)
                    if len(mine) == 1 and len(self.libs(mine)) == 1:
                        self.ko = n
            self.positions.add(tuple(self.board))
        self.player = -c
        self.history.append(p)
        if len(self.history) > 1 and self.history[-1] is None and self.history[-2] is None \
                and self.player == WHITE:
            self.end = True

    def place_handicaps(self, points):
        """Black stones played in order, then the move history starts afresh."""
        for p in points:
            self.player = BLACK
            self.play(p)
        self.history = []
        self.handicaps = list(points)

    def score(self):
        """(black, white) area scores."""
        sb = sw = 0
        for p, c in enumerate(self.board):
            if c == BLACK:
                sb += 1
            elif c == WHITE:
                sw += 1
            elif self.is_eyeish(p, BLACK):
                sb += 1
            elif self.is_eyeish(p, WHITE):
                sw += 1
        return sb - self.passes[BLACK], sw + self.komi - self.passes[WHITE]

    def winner(self):
        b, w = self.score()
        return BLACK if b > w else (WHITE if w > b else 0)
