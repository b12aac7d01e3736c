"""Go Text Protocol (GTP v2) engine — SURVEY C45 / §2.4.

The reference builds on the external ``pygtp`` package (``interface/gtp_wrapper.py:1-154``); that
package is not available here, so the protocol layer is implemented from the GTP v2 rules:

  * a command line is ``[id] command_name [arguments]``; ``#`` starts a comment; control
    characters other than tab/newline are dropped and tabs become spaces
  * success: ``= [id] result\\n\\n``, failure: ``? [id] message\\n\\n``
  * vertices are letter+number with column letters skipping ``I`` (``A1`` .. ``T19``); the engine
    hands the game object 1-indexed ``(x, y)`` tuples, ``PASS = (0, 0)``

``GtpEngine`` provides the base command set (protocol_version, name, version, known_command,
list_commands, quit, boardsize, clear_board, komi, play, genmove, showboard);
``ExtendedGtpEngine`` adds the reference's extras (time_left, place_free_handicap,
set_free_handicap, final_score, final_status_list, load_sgf / save_sgf) plus the standard
``loadsgf`` / ``printsgf``. Scoring uses GNU Go when it is installed (as the reference does, with
a 10 s timeout) and otherwise the engine's own area scorer instead of returning nothing.
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

PASS = (0, 0)
RESIGN = "resign"
BLACK, WHITE = 1, -1
COLUMNS = "ABCDEFGHJKLMNOPQRSTUVWXYZ"
MAX_BOARD = 25

_CTRL = re.compile(r"[\x00-\x08\x0b-\x1f\x7f]")


class GtpError(ValueError):
    pass


def parse_vertex(s):
    """'D4' -> (4, 4); 'pass' -> PASS; None if malformed."""
    s = s.strip().upper()
    if s == "PASS":
        return PASS
    if len(s) < 2 or s[0] not in COLUMNS:
        return None
    try:
        y = int(s[1:])
    except ValueError:
        return None
    x = COLUMNS.index(s[0]) + 1
    if not (1 <= x <= MAX_BOARD and 1 <= y <= MAX_BOARD):
        return None
    return (x, y)


def format_vertex(v):
    if v == PASS or v is None:
        return "pass"
    if v == RESIGN:
        return RESIGN
    x, y = v
    return "%s%d" % (COLUMNS[x - 1], y)


def parse_color(s):
    s = s.strip().lower()
    if s in ("b", "black"):
        return BLACK
    if s in ("w", "white"):
        return WHITE
    return None


def parse_move(args):
    """'black D4' -> (BLACK, (4, 4))."""
    parts = args.split()
    if len(parts) != 2:
        return None
    c, v = parse_color(parts[0]), parse_vertex(parts[1])
    if c is None or v is None:
        return None
    return c, v


def preprocess_line(line):
    line = _CTRL.sub("", line).replace("\t", " ")
    hash_at = line.find("#")
    if hash_at >= 0:
        line = line[:hash_at]
    return line.strip()


class GtpEngine(object):
    """Protocol core. ``game`` must provide: clear(), make_move(color, vertex) -> bool,
    set_size(n), set_komi(k), get_move(color) -> vertex (1-indexed tuple, PASS or 'resign')."""

    protocol = 2

    def __init__(self, game, name="gtp (python library)", version="0.2"):
        self.size = 19
        self.komi = 6.5
        self._game = game
        self._game.clear()
        self._name = name
        self._version = version
        self.disconnect = False
        self.known_commands = sorted(a[4:] for a in dir(self) if a.startswith("cmd_"))

    # ------------------------------------------------------------------ transport
    def send(self, message):
        """Process one command line; returns the full response ('' for empty lines)."""
        line = preprocess_line(message)
        if not line:
            return ""
        parts = line.split(None, 1)
        cid = ""
        if parts[0].isdigit():
            cid = parts[0]
            parts = parts[1].split(None, 1) if len(parts) > 1 else []
            if not parts:
                return self._reply(cid, False, "empty command")
        name = parts[0].lower()
        args = parts[1] if len(parts) > 1 else ""
        fn = getattr(self, "cmd_" + name, None)
        if fn is None:
            return self._reply(cid, False, "unknown command")
        try:
            out = fn(args)
        except (GtpError, ValueError) as e:
            return self._reply(cid, False, str(e))
        return self._reply(cid, True, "" if out is None else out)

    @staticmethod
    def _reply(cid, ok, text):
        head = ("=" if ok else "?") + cid
        return (head + " " + text if text else head) + "\n\n"

    # ------------------------------------------------------------------ base commands
    def cmd_protocol_version(self, args):
        return str(self.protocol)

    def cmd_name(self, args):
        return self._name

    def cmd_version(self, args):
        return self._version

    def cmd_known_command(self, args):
        return "true" if args.strip() in self.known_commands else "false"

    def cmd_list_commands(self, args):
        return "\n".join(self.known_commands)

    def cmd_quit(self, args):
        self.disconnect = True

    def cmd_boardsize(self, args):
        try:
            n = int(args)
        except ValueError:
            raise GtpError("boardsize is not an integer")
        if not 2 <= n <= MAX_BOARD:
            raise GtpError("unacceptable size")
        self.size = n
        self._game.set_size(n)

    def cmd_clear_board(self, args):
        self._game.clear()

    def cmd_komi(self, args):
        try:
            k = float(args)
        except ValueError:
            raise GtpError("syntax error")
        self.komi = k
        self._game.set_komi(k)

    def cmd_play(self, args):
        mv = parse_move(args)
        if mv is None:
            raise GtpError("syntax error")
        if not self._game.make_move(*mv):
            raise GtpError("illegal move")

    def cmd_genmove(self, args):
        c = parse_color(args)
        if c is None:
            raise GtpError("syntax error")
        v = self._game.get_move(c)
        if v != RESIGN:
            self._game.make_move(c, v)
        return format_vertex(v)


def _gnugo(sgf_path, command, timeout=10.0):
    exe = shutil.which("gnugo")
    if exe is None:
        return None
    try:
        p = subprocess.run([exe, "--chinese-rules", "--mode", "gtp", "-l", sgf_path],
                           input=command.encode(), stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, timeout=timeout)
    except (subprocess.TimeoutExpired, OSError):
        return ""
    return p.stdout.decode("utf-8", "replace")[2:].strip()


class ExtendedGtpEngine(GtpEngine):
    """Reference extras (``interface/gtp_wrapper.py:20-82``)."""

    recommended_handicaps = {
        2: "D4 Q16",
        3: "D4 Q16 D16",
        4: "D4 Q16 D16 Q4",
        5: "D4 Q16 D16 Q4 K10",
        6: "D4 Q16 D16 Q4 D10 Q10",
        7: "D4 Q16 D16 Q4 D10 Q10 K10",
        8: "D4 Q16 D16 Q4 D10 Q10 K4 K16",
        9: "D4 Q16 D16 Q4 D10 Q10 K4 K16 K10",
    }

    def cmd_time_left(self, args):
        pass

    def cmd_time_settings(self, args):
        pass

    def cmd_place_free_handicap(self, args):
        try:
            n = int(args)
        except Exception:
            raise GtpError("Number of handicaps could not be parsed: {}".format(args))
        if n < 2 or n > 9:
            raise GtpError("Invalid number of handicap stones: {}".format(n))
        vs = self.recommended_handicaps[n]
        self.cmd_set_free_handicap(vs)
        return vs

    def cmd_set_free_handicap(self, args):
        vs = [parse_vertex(v) for v in args.split()]
        if any(v is None or v == PASS for v in vs):
            raise GtpError("bad vertex list")
        self._game.place_handicaps(vs)

    def cmd_final_score(self, args):
        path = self._game.get_current_state_as_sgf()
        try:
            out = _gnugo(path, "final_score\n")
        finally:
            os.unlink(path)
        return out if out is not None else self._game.final_score()

    def cmd_final_status_list(self, args):
        path = self._game.get_current_state_as_sgf()
        try:
            out = _gnugo(path, "final_status_list {}\n".format(args))
        finally:
            os.unlink(path)
        return out if out is not None else self._game.final_status_list(args.strip())

    def cmd_load_sgf(self, args):
        return self.cmd_loadsgf(args)

    def cmd_save_sgf(self, args):
        name = args.strip()
        if name:
            with open(name, "w") as f:
                f.write(self._game.sgf_string())

    def cmd_loadsgf(self, args):
        parts = args.split()
        if not parts:
            raise GtpError("missing filename")
        upto = int(parts[1]) if len(parts) > 1 else None
        try:
            with open(parts[0]) as f:
                self._game.load_sgf(f.read(), upto)
        except (OSError, IOError):
            raise GtpError("cannot load file")

    def cmd_printsgf(self, args):
        s = self._game.sgf_string()
        name = args.strip()
        if name:
            with open(name, "w") as f:
                f.write(s)
            return None
        return s

    def cmd_showboard(self, args):
        return "\n" + self._game.ascii_board()

    def cmd_undo(self, args):
        if not self._game.undo():
            raise GtpError("cannot undo")


class GTPGameConnector(object):
    """Adapts a GameState (superko on) + player to the engine's game interface
    (``interface/gtp_wrapper.py:85-135``); GTP vertices are 1-indexed."""

    def __init__(self, player):
        from ..engine.gamestate import GameState
        self._GameState = GameState
        self._state = GameState(enforce_superko=True)
        self._player = player
        self._moves = []

    def clear(self):
        self._state = self._GameState(self._state.size, komi=self._state.komi,
                                      enforce_superko=True)
        self._moves = []

    def make_move(self, color, vertex):
        from ..engine.gamestate import IllegalMove, PASS_MOVE
        try:
            if vertex == PASS:
                self._state.do_move(PASS_MOVE, color)
                self._moves.append((color, None))
            else:
                x, y = vertex
                if not (1 <= x <= self._state.size and 1 <= y <= self._state.size):
                    return False
                self._state.do_move((x - 1, y - 1), color)
                self._moves.append((color, (x - 1, y - 1)))
            return True
        except IllegalMove:
            return False

    def set_size(self, n):
        self._state = self._GameState(n, komi=self._state.komi, enforce_superko=True)
        self._moves = []

    def set_komi(self, k):
        self._state.komi = k

    def get_move(self, color):
        from ..engine.gamestate import PASS_MOVE
        self._state.current_player = color
        move = self._player.get_move(self._state)
        if move == PASS_MOVE:
            return PASS
        x, y = move
        return (x + 1, y + 1)

    def place_handicaps(self, vertices):
        self._state.place_handicaps([(x - 1, y - 1) for (x, y) in vertices])
        self._handicaps = list(vertices)

    # ---------------------------------------------------------------- extras
    def sgf_string(self):
        from ..utils.go_util import gamestate_to_sgf_string
        return gamestate_to_sgf_string(self._state, size=self._state.size,
                                       komi=self._state.komi)

    def get_current_state_as_sgf(self):
        fd, path = tempfile.mkstemp(suffix=".sgf")
        with os.fdopen(fd, "w") as f:
            f.write(self.sgf_string())
        return path

    def load_sgf(self, text, upto=None):
        from ..utils.go_util import sgf_iter_states
        state, moves = None, []
        for i, (gs, move, player) in enumerate(sgf_iter_states(text, include_end=True)):
            state = gs
            if upto is not None and i + 1 >= upto:
                break
        if state is None:
            raise GtpError("empty sgf")
        st = state.copy()
        st.enforce_superko = True
        self._state = st
        self._moves = moves

    def undo(self):
        if not self._moves:
            return False
        moves = self._moves[:-1]
        size, komi = self._state.size, self._state.komi
        handicaps = list(self._state.handicaps)
        self._state = self._GameState(size, komi=komi, enforce_superko=True)
        if handicaps:
            self._state.place_handicaps(handicaps)
        self._moves = []
        for color, mv in moves:
            self.make_move(color, PASS if mv is None else (mv[0] + 1, mv[1] + 1))
        return True

    def final_score(self):
        sw, sb = self._state.get_score()
        d = sb - sw
        if d == 0:
            return "0"
        return ("B+%g" if d > 0 else "W+%g") % abs(d)

    def final_status_list(self, status):
        """Without a life-and-death reader every stone counts as alive (consistent with the
        area scorer used by final_score)."""
        if status not in ("alive", "dead", "seki"):
            raise GtpError("invalid status")
        if status != "alive":
            return ""
        b = self._state.board
        S = self._state.size
        return " ".join(format_vertex((x + 1, y + 1)) for x in range(S) for y in range(S)
                        if b[x][y] != 0)

    def ascii_board(self):
        b = self._state.board
        S = self._state.size
        cols = "   " + " ".join(COLUMNS[:S])
        rows = [cols]
        for y in range(S, 0, -1):
            cells = []
            for x in range(1, S + 1):
                v = b[x - 1][y - 1]
                cells.append("X" if v == BLACK else ("O" if v == WHITE else "."))
            rows.append("%2d %s %d" % (y, " ".join(cells), y))
        rows.append(cols)
        return "\n".join(rows)


def run_gtp(player_obj, inpt_fn=None, name="Gtp Player", version="0.0", out=None):
    """REPL: read commands with ``inpt_fn`` (default: stdin lines), write replies to ``out``.
    A single input may carry several newline-separated commands (reference behaviour)."""
    game = GTPGameConnector(player_obj)
    engine = ExtendedGtpEngine(game, name, version)
    out = out or sys.stdout
    if inpt_fn is None:
        def inpt_fn():
            line = sys.stdin.readline()
            if not line:
                raise EOFError
            return line
    sys.stderr.write("GTP engine ready\n")
    sys.stderr.flush()
    while not engine.disconnect:
        try:
            inpt = inpt_fn()
        except EOFError:
            break
        for cmd in str(inpt).split("\n"):
            reply = engine.send(cmd)
            if reply:
                out.write(reply)
                out.flush()
            if engine.disconnect:
                break
    return engine


def main(argv=None):
    """Serve a policy network (or MCTS over it) on stdin/stdout:

    python -m rocalphago_amd.gtp.engine model.json [--weights W] \
        [--player greedy|probabilistic|mcts]
    """
    import argparse
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("model", nargs="?", help="policy JSON (CNNPolicy.save_model); omit for a"
                                             " passing engine")
    ap.add_argument("--weights", default=None)
    ap.add_argument("--player", default="greedy", choices=["greedy", "probabilistic", "mcts"])
    ap.add_argument("--temperature", type=float, default=0.67)
    ap.add_argument("--playouts", type=int, default=800)
    ap.add_argument("--name", default="RocAlphaGo-MI355X")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16",
                    help="GPU compute precision of the networks (bf16 = fused HIP kernels)")
    ap.add_argument("--value", default=None, help="value network JSON (mcts player)")
    ap.add_argument("--value-weights", default=None)
    ap.add_argument("--lmbda", type=float, default=None,
                    help="value/rollout mix (default 0.5 with a value net, else 1 = rollouts)")
    ap.add_argument("--c-puct", type=float, default=5.0)
    ap.add_argument("--mcts-threads", type=int, default=8,
                    help="host threads of the parallel tree descent / leaf featurisation")
    ap.add_argument("--leaf-batch", type=int, default=512,
                    help="leaves evaluated per GPU batch (one search wave)")
    ap.add_argument("--virtual-loss", type=int, default=3,
                    help="virtual visits added along a pending descent path")
    ap.add_argument("--rollout-limit", type=int, default=500)
    args = ap.parse_args(argv)
    if args.model is None:
        class _Pass(object):
            def get_move(self, state):
                return None
        player = _Pass()
    else:
        from ..models.nn_util import NeuralNetBase
        from ..players import ai
        policy = NeuralNetBase.load_model(args.model).set_dtype(args.dtype)
        if args.weights:
            policy.model.load_weights(args.weights)
        if args.player == "greedy":
            player = ai.GreedyPolicyPlayer(policy)
        elif args.player == "probabilistic":
            player = ai.ProbabilisticPolicyPlayer(policy, temperature=args.temperature)
        else:
            from ..search.apv import ParallelMCTSPlayer
            value = None
            if args.value:
                value = NeuralNetBase.load_model(args.value).set_dtype(args.dtype)
                if args.value_weights:
                    value.model.load_weights(args.value_weights)
            lmbda = args.lmbda if args.lmbda is not None else (0.5 if value is not None else 1.0)
            player = ParallelMCTSPlayer(policy, value, lmbda=lmbda, c_puct=args.c_puct,
                                        n_playout=args.playouts, batch=args.leaf_batch,
                                        virtual_loss=args.virtual_loss,
                                        nthreads=args.mcts_threads,
                                        rollout_limit=args.rollout_limit)
    run_gtp(player, name=args.name, version="1.0")


if __name__ == "__main__":
    main()
