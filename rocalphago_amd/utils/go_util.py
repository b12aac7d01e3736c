"""Board/SGF utilities with the reference's AlphaGo/util.py interface (util.py:1-231).

flatten_idx/unflatten_idx (util.py:11-18), SGF move parsing and game-state reconstruction on our
own SGF parser (util.py:21-63,100-128), a main-line SGF writer (util.py:66-97 file contract) and
an optional matplotlib heat map of a network's move distribution (util.py:131-231 signature).
"""
import os

import numpy as np

from ..engine import gamestate as go
from ..io import sgf

# for board location indexing
LETTERS = 'ABCDEFGHIJKLMNOPQRSTUVWXYZ'


def flatten_idx(position, size):
    (x, y) = position
    return x * size + y


def unflatten_idx(idx, size):
    x, y = divmod(idx, size)
    return (x, y)


def _parse_sgf_move(node_value):
    """'' or 'tt' → pass; otherwise (col, row) from the two letters."""
    if node_value == '' or node_value == 'tt':
        return go.PASS_MOVE
    col = LETTERS.index(node_value[0].upper())
    row = LETTERS.index(node_value[1].upper())
    return (col, row)


def _expand_point_list(values):
    """AB/AW may use compressed point lists 'aa:cc' (FF[4]); expand them."""
    out = []
    for v in values:
        if ':' in v:
            a, b = v.split(':', 1)
            (x0, y0), (x1, y1) = _parse_sgf_move(a), _parse_sgf_move(b)
            for x in range(min(x0, x1), max(x0, x1) + 1):
                for y in range(min(y0, y1), max(y0, y1) + 1):
                    out.append((x, y))
        else:
            out.append(_parse_sgf_move(v))
    return out


def _sgf_init_gamestate(sgf_root):
    props = sgf_root.properties
    s_size = props.get('SZ', ['19'])[0]
    s_player = props.get('PL', ['B'])[0]
    gs = go.GameState(int(s_size.split(':')[0]))
    if 'AB' in props:
        for stone in _expand_point_list(props['AB']):
            gs.do_move(stone, go.BLACK)
    if 'AW' in props:
        for stone in _expand_point_list(props['AW']):
            gs.do_move(stone, go.WHITE)
    gs.current_player = go.BLACK if s_player == 'B' else go.WHITE
    return gs


def sgf_iter_states(sgf_string, include_end=True):
    """Yield (GameState, move, player) along the main line; the state is mutated in place."""
    collection = sgf.parse(sgf_string)
    game = collection[0]
    gs = _sgf_init_gamestate(game.root)
    rest = game.rest
    if rest is not None:
        for node in rest:
            props = node.properties
            if 'W' in props:
                move = _parse_sgf_move(props['W'][0])
                player = go.WHITE
            elif 'B' in props:
                move = _parse_sgf_move(props['B'][0])
                player = go.BLACK
            else:
                # setup node (e.g. the ';AB[..]' handicap node our own writer emits, like the
                # reference's save_gamestate_to_sgf): AB before any move = handicap stones
                if 'AB' in props and len(gs.history) == 0 and 'AW' not in props:
                    gs.place_handicaps(_expand_point_list(props['AB']))
                else:
                    for key, color in (('AB', go.BLACK), ('AW', go.WHITE)):
                        for stone in _expand_point_list(props.get(key, [])):
                            gs.do_move(stone, color)
                continue
            yield (gs, move, player)
            gs.do_move(move, player)
    if include_end:
        yield (gs, None, None)


def sgf_to_gamestate(sgf_string):
    gs = None
    for (gs, move, player) in sgf_iter_states(sgf_string, True):
        pass
    return gs


def _sgf_point(move):
    """SGF coordinate of a move: two lower-case letters (column, row) or 'tt' for a pass."""
    if move is None:
        return "tt"
    return LETTERS[move[0]].lower() + LETTERS[move[1]].lower()


def gamestate_to_sgf_string(gamestate, black_player_name='Unknown', white_player_name='Unknown',
                            size=19, komi=7.5):
    """Main-line SGF of a game: a root node with the game info, one AB setup node for handicap
    stones (then white moves first), and one node per history move. Same file contract as the
    reference writer (util.py:66-97); read back by sgf_iter_states."""
    info = [("GM", 1), ("FF", 4), ("CA", "UTF-8"), ("SZ", size), ("KM", komi),
            ("PB", black_player_name), ("PW", white_player_name)]
    handicaps = list(gamestate.handicaps)
    if handicaps:
        info.append(("HA", len(handicaps)))
    nodes = [";" + "".join("%s[%s]" % kv for kv in info)]
    if handicaps:
        nodes.append(";AB" + "".join("[%s]" % _sgf_point(h) for h in handicaps))
    colours = "WB" if handicaps else "BW"
    nodes.extend(";%s[%s]" % (colours[k % 2], _sgf_point(mv))
                 for k, mv in enumerate(gamestate.history))
    return "(" + "".join(nodes) + ")"


def save_gamestate_to_sgf(gamestate, path, filename, black_player_name='Unknown',
                          white_player_name='Unknown', size=19, komi=7.5):
    """Write gamestate_to_sgf_string to path/filename (reference util.py:66-97 signature)."""
    text = gamestate_to_sgf_string(gamestate, black_player_name, white_player_name, size, komi)
    with open(os.path.join(path, filename), "w") as f:
        f.write(text)


def _axis_labels(size, western_column_notation):
    """(x tick labels, y tick labels, x ticks on top) for a size x size board."""
    numbers = list(range(1, size + 1))
    if western_column_notation:
        return numbers, numbers[::-1], False
    columns = [c for c in LETTERS if c != 'I'][:size]
    return columns, numbers, True


def plot_network_output(scores, board, history, out_directory, output_file,
                        should_plot=False, western_column_notation=True):
    """Heat map of a network's move distribution over the board (reference util.py:131-231
    signature; matplotlib is an optional dependency, imported on use).

    Points holding at least 0.1 % of the probability mass are drawn as discs coloured by their
    probability and labelled in percent; stones are drawn on top (black / white) and the last
    move, if any, is marked with a small red square. The figure is saved to
    out_directory/output_file (if given) and shown when should_plot is set."""
    try:
        import matplotlib
        if not should_plot:
            matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        print("plot_network_output needs matplotlib (an optional dependency)")
        raise
    size = board.shape[0]
    probs = np.asarray(scores, dtype=np.float64).reshape(size, size)
    fig, ax = plt.subplots(figsize=(10, 10))
    ax.set_xlim(0, size + 1)
    ax.set_ylim(size + 1, 0)  # row 1 at the top
    ax.set_facecolor("#e8b96a")
    ax.tick_params(length=0)
    xl, yl, top = _axis_labels(size, western_column_notation)
    ax.set_xticks(range(1, size + 1))
    ax.set_xticklabels(xl)
    ax.set_yticks(range(1, size + 1))
    ax.set_yticklabels(yl)
    if top:
        ax.xaxis.tick_top()
    grid = np.arange(1, size + 1)
    for g in grid:
        ax.plot([1, size], [g, g], color="black", linewidth=0.8, zorder=0)
        ax.plot([g, g], [1, size], color="black", linewidth=0.8, zorder=0)
    xi, yi = np.nonzero(probs >= 1e-3)
    if len(xi):
        val = probs[xi, yi]
        ax.scatter(xi + 1, yi + 1, s=650, c=val, cmap="cool", vmin=probs.min(), vmax=probs.max(),
                   edgecolors="black", zorder=1)
        for x, y, v in zip(xi, yi, val):
            ax.text(x + 1, y + 1, "%.1f" % (100 * v), ha="center", va="center", fontsize=9,
                    zorder=3)
    stones = np.asarray(board)
    for colour, face in ((go.BLACK, "black"), (go.WHITE, "white")):
        sx, sy = np.nonzero(stones == colour)
        if len(sx):
            ax.scatter(sx + 1, sy + 1, s=650, c=face, edgecolors="black", zorder=4)
    if len(history) and history[-1] is not go.PASS_MOVE:
        lx, ly = history[-1]
        ax.scatter([lx + 1], [ly + 1], marker="s", s=90, c="red", edgecolors="black", zorder=5)
    if output_file is not None:
        fig.savefig(os.path.join(out_directory, output_file), bbox_inches="tight")
    if should_plot:
        plt.show()
    plt.close(fig)
