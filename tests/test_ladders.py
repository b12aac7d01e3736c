"""Ladder reading (spec: reference tests/test_ladders.py scenarios, go.py:329-463)."""
from rocalphago_amd.engine import BLACK, WHITE

from boards import parse


def test_simple_capture_then_escape_fails():
    st, m = parse("d b c . . . .|"
                  "B W a . . . .|"
                  ". B . . . . .|"
                  ". . . . . . .|"
                  ". . . . . . .|"
                  ". . . . . W .|")
    st.current_player = BLACK
    assert st.is_ladder_capture(m['a'])
    assert not st.is_ladder_capture(m['b'])
    st.do_move(m['a'])
    assert not st.is_ladder_escape(m['b'])
    st.do_move(m['b'])
    assert st.is_ladder_capture(m['c'])
    assert not st.is_ladder_capture(m['d'])  # self-atari


def test_breaker_turns_ladder_into_escape():
    st, m = parse(". B . . . . .|"
                  "B W a . . W .|"
                  "B b . . . . .|"
                  ". c . . . . .|"
                  ". . . . . . .|"
                  ". . . . . W .|"
                  ". . . . . . .|")
    st.current_player = BLACK
    assert not st.is_ladder_capture(m['a'])
    assert not st.is_ladder_capture(m['b'])
    st.do_move(m['a'])
    assert st.is_ladder_escape(m['b'])
    st.do_move(m['b'])
    assert not st.is_ladder_capture(m['c'])


def test_missing_breaker():
    st, m = parse(". B . . . . .|"
                  "B W B . . W .|"
                  "B a c . . . .|"
                  ". b . . . . .|"
                  ". . . . . . .|"
                  ". W . . . . .|"
                  ". . . . . . .|")
    st.current_player = WHITE
    assert not st.is_ladder_escape(m['a'])
    st.do_move(m['a'])
    assert st.is_ladder_capture(m['b'])
    assert not st.is_ladder_capture(m['c'])


def test_capturing_hunters_escapes():
    st, m = parse(". O X . . .|"
                  ". X O X . .|"
                  ". . O X . .|"
                  ". . a . . .|"
                  ". O . . . .|"
                  ". . . . . .|")
    st.current_player = BLACK
    assert not st.is_ladder_capture(m['a'])


def test_throw_in():
    st, m = parse("X a O X . .|"
                  "b O O X . .|"
                  "O O X X . .|"
                  "X X . . . .|"
                  ". . . . . .|"
                  ". . . O . .|")
    st.current_player = BLACK
    assert st.is_ladder_capture(m['a'])
    assert st.is_ladder_capture(m['b'])
    st.do_move(m['a'])
    assert not st.is_ladder_escape(m['b'])


def test_snapback_is_no_escape():
    st, m = parse(". . . . . . . . .|"
                  ". . . . . . . . .|"
                  ". . X X X . . . .|"
                  ". . O . . . . . .|"
                  ". . O X . . . . .|"
                  ". . X O a . . . .|"
                  ". . X O X . . . .|"
                  ". . . X . . . . .|"
                  ". . . . . . . . .|")
    st.current_player = WHITE
    assert not st.is_ladder_escape(m['a'])


def test_two_capturing_moves():
    st, m = parse(". . . . . .|"
                  ". . . . . .|"
                  ". . a b . .|"
                  ". X O O X .|"
                  ". . X X . .|"
                  ". . . . . .|")
    st.current_player = BLACK
    assert st.is_ladder_capture(m['a'])
    assert st.is_ladder_capture(m['b'])


def test_two_escaping_moves():
    st, m = parse(". . X . . .|"
                  ". X O a . .|"
                  ". X c X . .|"
                  ". O X b . .|"
                  ". . O . . .|"
                  ". . . . . .|")
    st.do_move(m['c'], color=WHITE)
    st.current_player = WHITE
    assert st.is_ladder_escape(m['a'])
    assert st.is_ladder_escape(m['b'], prey=m['c'])


def test_depth_limit():
    st, m = parse("d b c . . . .|"
                  "B W a . . . .|"
                  ". B . . . . .|"
                  ". . . . . . .|"
                  ". . . . . . .|"
                  ". . . . . W .|")
    st.current_player = BLACK
    # with no reading budget the capture is assumed and the escape is given up
    assert st.is_ladder_capture(m['a'], remaining_attempts=0)
    st.do_move(m['a'])
    assert not st.is_ladder_escape(m['b'], remaining_attempts=0)
