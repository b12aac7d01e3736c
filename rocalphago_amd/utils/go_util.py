"""Board/SGF utilities — reference AlphaGo/util.py:1-231.

flatten_idx/unflatten_idx (util.py:11-18), SGF move parsing and game-state reconstruction
(util.py:21-63,100-128), the simplified SGF writer (util.py:66-97) and the optional matplotlib
heat-map (util.py:131-231).
"""
import itertools
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


def gamestate_to_sgf_string(gamestate, black_player_name='Unknown', white_player_name='Unknown',
                            size=19, komi=7.5):
    str_list = ['(;GM[1]FF[4]CA[UTF-8]', 'SZ[{}]'.format(size), 'KM[{}]'.format(komi),
                'PB[{}]'.format(black_player_name), 'PW[{}]'.format(white_player_name)]
    cycle_string = 'BW'
    if len(gamestate.handicaps) > 0:
        cycle_string = 'WB'
        str_list.append('HA[{}]'.format(len(gamestate.handicaps)))
        str_list.append(';AB')
        for handicap in gamestate.handicaps:
            str_list.append('[{}{}]'.format(LETTERS[handicap[0]].lower(),
                                            LETTERS[handicap[1]].lower()))
    for move, color in zip(gamestate.history, itertools.cycle(cycle_string)):
        str_list.append(';{}'.format(color))
        if move is None:
            str_list.append('[tt]')
        else:
            str_list.append('[{}{}]'.format(LETTERS[move[0]].lower(), LETTERS[move[1]].lower()))
    str_list.append(')')
    return ''.join(str_list)


def save_gamestate_to_sgf(gamestate, path, filename, black_player_name='Unknown',
                          white_player_name='Unknown', size=19, komi=7.5):
    """Simplified SGF writer (reference util.py:66-97)."""
    with open(os.path.join(path, filename), "w") as f:
        f.write(gamestate_to_sgf_string(gamestate, black_player_name, white_player_name, size,
                                        komi))


def plot_network_output(scores, board, history, out_directory, output_file,
                        should_plot=False, western_column_notation=True):
    """Heat-map of network output over the board (optional matplotlib dependency)."""
    try:
        import matplotlib
        matplotlib.use("Agg") if not should_plot else None
        import matplotlib.pyplot as plt
        import matplotlib.cm as cm
    except ImportError as e:
        print('Failed to import matplotlib. This is an optional dependency; install it to use '
              'the plotting functions.')
        raise e
    size = board.shape[0]
    fig, ax = plt.subplots(figsize=(10, 10))
    plt.xlim([0, size + 1])
    plt.ylim([0, size + 1])
    ax.set_facecolor('#fec97b')
    plt.gca().invert_yaxis()
    ax.tick_params(axis='both', length=0, width=0)
    if western_column_notation:
        plt.xticks(range(1, size + 1), range(1, size + 1))
        plt.yticks(range(1, size + 1), reversed(range(1, size + 1)))
    else:
        ax.xaxis.tick_top()
        plt.xticks(range(1, size + 1), [x for x in LETTERS[:size + 1] if x != 'I'])
        plt.yticks(range(1, size + 1), range(1, size + 1))
    for i in range(size):
        plt.plot([1, size], [i + 1, i + 1], lw=1, color='k', zorder=0)
        plt.plot([i + 1, i + 1], [1, size], lw=1, color='k', zorder=0)
    reshaped = np.reshape(scores, (size, size))
    xs, ys, vals = [], [], []
    for i in range(size):
        for j in range(size):
            if reshaped[i][j] * 100 >= 0.1:
                xs.append(i + 1)
                ys.append(j + 1)
                vals.append(reshaped[i][j])
    norm = matplotlib.colors.Normalize(vmin=np.amin(scores), vmax=np.amax(scores))
    coloring = cm.ScalarMappable(norm=norm, cmap=cm.cool).to_rgba(vals)
    plt.scatter(xs, ys, marker='o', s=700, c=coloring, edgecolor='k', zorder=1)
    for i, txt in enumerate(vals):
        ax.annotate('{0:.1f}'.format(txt * 100), (xs[i], ys[i]), color='k', ha='center',
                    va='center', size=10, zorder=3)
    sx, sy, sc = [], [], []
    for i in range(size):
        for j in range(size):
            if board[i][j] != go.EMPTY:
                sx.append(i + 1)
                sy.append(j + 1)
                sc.append((0, 0, 0) if board[i][j] == go.BLACK else (1, 1, 1))
    plt.scatter(sx, sy, marker='o', edgecolors='k', s=700, c=sc, zorder=4)
    if len(history) != 0 and history[-1] != go.PASS_MOVE:
        last = history[-1]
        plt.scatter(last[0] + 1, last[1] + 1, marker='s', color='r', edgecolors='k', s=100,
                    zorder=5)
    if output_file is not None:
        plt.savefig(os.path.join(out_directory, output_file), bbox_inches='tight')
    if should_plot:
        plt.show()
    plt.close()
