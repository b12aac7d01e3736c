"""ASCII board builder used by the rules/feature tests.

Rows are separated by '|', spaces ignored; X/B/# = black, O/W = white, '.' = empty, any other
character marks a named point returned in the dict (row, col). Stones are placed with explicit
colours in reading order, as in the reference's tests/parseboard.py:4-31.
"""
from rocalphago_amd.engine import BLACK, WHITE, GameState


def parse(diagram):
    rows = diagram.replace(' ', '').split('|')
    rows = [r for r in rows if r]
    size = max(len(rows), max(len(r) for r in rows))
    state = GameState(size=size)
    marks = {}
    for r, line in enumerate(rows):
        for c, ch in enumerate(line):
            if ch == '.':
                continue
            if ch in 'XB#':
                state.do_move((r, c), color=BLACK)
            elif ch in 'OW':
                state.do_move((r, c), color=WHITE)
            else:
                assert ch not in marks, "duplicate marker %s" % ch
                marks[ch] = (r, c)
    return state, marks


def random_games(n, size, seed, lo, hi):
    """n positions from rollout-policy games of lo..hi moves (ladder-rich mid/late game)."""
    import numpy as np
    from rocalphago_amd._native import engine
    rp = engine().RolloutPolicy()
    rs = np.random.RandomState(seed)
    out = []
    for _ in range(n):
        st = GameState(size=size)
        for _k in range(int(rs.randint(lo, hi))):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            st.do_move(None if mv < 0 else divmod(mv, size))
            if st.is_end_of_game:
                break
        out.append(st)
    return out


def ladder_scenarios():
    """The reference ladder scenarios (its tests/test_ladders.py) at each step, both colours."""
    boards = [
        ("d b c . . . .|B W a . . . .|. B . . . . .|. . . . . . .|. . . . . . .|"
         ". . . . . W .|", ["a", "b"]),
        (". B . . . . .|B W a . . W .|B b . . . . .|. c . . . . .|. . . . . . .|"
         ". . . . . W .|", ["a", "b"]),
        (". B . . . . .|B W B . . W .|B a c . . . .|. b . . . . .|. . . . . . .|"
         ". W . . . . .|. . . . . . .|", ["a"]),
    ]
    out = []
    for text, moves in boards:
        for first in (BLACK, WHITE):
            st, m = parse(text)
            st.current_player = first
            out.append(st.copy())
            for mv in moves:
                if not st.is_legal(m[mv]):
                    break
                st.do_move(m[mv])
                out.append(st.copy())
    return out
