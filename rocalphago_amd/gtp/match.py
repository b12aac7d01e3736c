"""Two-player match harness (reference ``interface/TestPlay.py:15-155`` and the
older ``interface/Play.py:5-35``).

``PlayMatch(player1, player2, size)`` alternates ``get_move`` between the players (player1 is
black) until two consecutive passes with WHITE to move (the engine's end-of-game rule),
renders the board as ASCII (``showboard``) and scores it with the same area counting as
``GameState.get_winner`` (``calculate_score``).
"""
import numpy as np

from ..engine.gamestate import BLACK, EMPTY, WHITE, GameState

AXIS = "abcdefghijklmnopqrstuvwxy"
RESULT = "DBW"


class PlayMatch(object):
    def __init__(self, player1, player2, save_dir=None, size=19, komi=7.5):
        self.player1 = player1
        self.player2 = player2
        self.save_dir = save_dir
        self.komi = komi
        self.state = GameState(size=size, komi=komi)
        self.current = player1
        self.opponent = player2
        self.playout = False

    def _play(self):
        move = self.current.get_move(self.state)
        self.state.do_move(move)
        h = self.state.history
        end = (len(h) > 1 and h[-1] is None and h[-2] is None and
               self.state.current_player == WHITE)
        if end:
            self.playout = True
        else:
            self.current, self.opponent = self.opponent, self.current
        return end

    def clear(self, showboard=True):
        self.state = GameState(size=self.state.size, komi=self.komi)
        self.current, self.opponent = self.player1, self.player2
        self.playout = False
        if showboard:
            self.showboard()

    def play(self, showboard=True):
        """One move by the player to move; returns True once the game is over."""
        if not self.playout:
            self._play()
        if showboard:
            self.showboard()
        return self.playout

    def playover(self, turn=300, showboard=True):
        """Play up to ``turn`` moves per side or until the game ends."""
        if not self.playout:
            for _ in range(turn * 2):
                self._play()
                if self.playout:
                    break
        if showboard:
            self.showboard()
        return self.playout

    def board_string(self):
        st = self.state
        S = st.size
        last = st.history[-1] if st.history else None
        out = []
        for i in range(S + 2):
            row = []
            for j in range(S + 2):
                if i in (0, S + 1) and j in (0, S + 1):
                    ch = " "
                elif i in (0, S + 1):
                    ch = AXIS[j - 1]
                elif j in (0, S + 1):
                    ch = AXIS[i - 1]
                else:
                    v = st.board[j - 1][i - 1]
                    is_last = last is not None and last == (j - 1, i - 1)
                    if v == BLACK:
                        ch = "B" if is_last else "x"
                    elif v == WHITE:
                        ch = "W" if is_last else "o"
                    elif S == 19 and (i - 1) in (3, 9, 15) and (j - 1) in (3, 9, 15):
                        ch = "+"
                    else:
                        ch = "."
                row.append(ch)
            line = " ".join(row) + " "
            if i == 1 and st.history:
                who = "W" if st.current_player == BLACK and not self.playout else "B"
                mv = "tt" if last is None else AXIS[last[0]] + AXIS[last[1]]
                line += "    ;%s(%s)" % (who, mv)
            if i == 3 and self.playout:
                sw, sb = self.calculate_score()
                w = st.get_winner()
                line += "    " + ("Draw" if not w else "Winner: %s" % RESULT[w])
                line += " (W: %s, B: %s)" % (sw, sb)
            out.append(line)
        return "\n".join(out)

    def showboard(self):
        print(self.board_string())

    def calculate_score(self):
        """(score_white, score_black): stones + single-point eyeish empties, komi to white,
        minus passes (reference ``TestPlay.py:136-155``)."""
        st = self.state
        board = np.asarray(st.board)
        sw = float(np.sum(board == WHITE))
        sb = float(np.sum(board == BLACK))
        for x, y in zip(*np.where(board == EMPTY)):
            if st.is_eyeish((int(x), int(y)), BLACK):
                sb += 1
            elif st.is_eyeish((int(x), int(y)), WHITE):
                sw += 1
        sw += st.komi - st.passes_white
        sb -= st.passes_black
        return sw, sb


# reference class name
play_match = PlayMatch
