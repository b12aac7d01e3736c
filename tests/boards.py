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
