"""Rules engine behaviour (spec: reference tests/test_gamestate.py, test_liberties.py, go.py)."""
import numpy as np
import pytest

from rocalphago_amd.engine import BLACK, EMPTY, PASS_MOVE, WHITE, GameState, IllegalMove


def play(gs, moves):
    for m in moves:
        gs.do_move(m)
    return gs


class TestKo:
    def test_ko_blocks_immediate_recapture(self):
        gs = play(GameState(size=9), [(1, 0), (2, 0), (0, 1), (3, 1), (1, 2), (2, 2), (2, 1)])
        gs.do_move((1, 1))  # white captures the lone black stone at (2,1)
        assert gs.num_black_prisoners == 1 and gs.num_white_prisoners == 0
        assert gs.ko == (2, 1)
        assert not gs.is_legal((2, 1))
        play(gs, [(5, 5), (5, 6)])  # ko threat exchange
        assert gs.is_legal((2, 1))

    def test_snapback_is_not_ko(self):
        gs = GameState(size=5)
        for b, w in zip([(0, 0), (2, 1), (3, 0)], [(0, 1), (1, 1), (2, 0)]):
            gs.do_move(b)
            gs.do_move(w)
        gs.do_move((1, 0))  # black captures one white stone, but its own pair is in atari
        assert gs.ko is None
        assert gs.is_legal((2, 0))
        gs.do_move((2, 0))  # snapback captures two black stones
        assert gs.num_black_prisoners == 2
        assert gs.num_white_prisoners == 1

    def test_positional_superko_only_when_enforced(self):
        seq = [(0, 3), (0, 4), (1, 3), (1, 4), (2, 3), (2, 4), (2, 2), (3, 4), (2, 1), (3, 3),
               (3, 1), (3, 2), (3, 0), (4, 2), (1, 1), (4, 1), (8, 0), (4, 0), (8, 1), (0, 2),
               (8, 2), (0, 1), (8, 3), (1, 0), (8, 4), (2, 0), (0, 0)]
        assert play(GameState(size=9), seq).is_legal((1, 0))
        assert not play(GameState(size=9, enforce_superko=True), seq).is_legal((1, 0))

    def test_illegal_move_raises_and_keeps_player(self):
        gs = GameState(size=5)
        gs.do_move((2, 2))
        with pytest.raises(IllegalMove):
            gs.do_move((2, 2))
        assert gs.current_player == WHITE
        with pytest.raises(IllegalMove):
            gs.do_move((7, 7))


class TestEyes:
    def test_eyeish(self):
        gs = play(GameState(size=7), [(1, 0), (5, 4), (2, 1), (6, 5), (1, 2), (5, 6), (0, 1),
                                      (4, 5)])
        assert gs.is_eyeish((1, 1), BLACK) and not gs.is_eyeish((1, 1), WHITE)
        assert gs.is_eyeish((5, 5), WHITE) and not gs.is_eyeish((5, 5), BLACK)
        for p in [(1, 0), (2, 2)]:
            assert not gs.is_eyeish(p, BLACK) and not gs.is_eyeish(p, WHITE)

    def test_false_then_true_corner_eye(self):
        gs = GameState(size=7)
        gs.do_move((1, 0), BLACK)
        gs.do_move((0, 1), BLACK)
        assert gs.is_eyeish((0, 0), BLACK)
        assert not gs.is_eye((0, 0), BLACK)
        for p in [(1, 2), (2, 1), (2, 2), (0, 2)]:
            gs.do_move(p, BLACK)
        assert gs.is_eye((0, 0), BLACK)
        assert gs.is_eye((1, 1), BLACK)

    def test_mutually_supporting_eyes(self):
        gs = GameState(7)
        for x in range(7):
            for y in range(7):
                if (x + y) % 2 == 1:
                    gs.do_move((x, y), BLACK)
        assert gs.is_eye((0, 0), BLACK)


class TestGroupsAndLiberties:
    def test_liberties_after_capture_match_fresh_board(self):
        cap, ref = GameState(7), GameState(7)
        for x in range(2, 5):
            for y in range(2, 5):
                cap.do_move((x, y), BLACK)
        walls = [(x, 1) for x in range(2, 5)] + [(x, 5) for x in range(2, 5)] + [(1, 1)] + \
                [(1, y) for y in range(2, 5)] + [(5, y) for y in range(2, 5)]
        for p in walls:
            cap.do_move(p, WHITE)
            ref.do_move(p, WHITE)
        assert np.all(ref.board == cap.board)
        assert np.all(ref.liberty_counts == cap.liberty_counts)
        assert cap.num_black_prisoners == 9

    def test_shared_set_identity_survives_copy(self):
        gs = GameState(7)
        gs.do_move((4, 4), BLACK)
        gs.do_move((4, 5), BLACK)
        assert gs.group_sets[4][5] is gs.group_sets[4][4]
        assert gs.liberty_sets[4][5] is gs.liberty_sets[4][4]
        cp = gs.copy()
        assert cp.group_sets[4][5] is cp.group_sets[4][4]
        assert cp.liberty_sets[4][5] is cp.liberty_sets[4][4]
        assert cp.group_sets[4][4] == {(4, 4), (4, 5)}

    def test_liberty_counts(self):
        gs = play(GameState(), [(4, 5), (5, 5), (5, 6), (10, 10), (4, 6), (10, 11), (6, 6),
                                (9, 10)])
        assert gs.liberty_counts[5][5] == 2
        assert gs.liberty_counts[4][5] == 8
        assert gs.liberty_counts[5][6] == 8
        assert gs.liberty_counts[0][0] == -1

    def test_group_sizes(self):
        gs = play(GameState(), [(0, 0), (5, 5), (0, 1), (6, 6), (1, 0), (1, 1)])
        assert len(gs.get_group((0, 0))) == 3
        assert len(gs.get_group((4, 4))) == 0
        assert len(gs.get_group((5, 5))) == 1

    def test_groups_around_unique(self):
        gs = GameState(5)
        for p in [(1, 2), (2, 1), (2, 2)]:
            gs.do_move(p, WHITE)
        groups = gs.get_groups_around((1, 1))
        assert len(groups) == 1 and groups[0] == {(1, 2), (2, 1), (2, 2)}

    def test_empty_point_liberty_set_is_empty_neighbours(self):
        gs = GameState(5)
        gs.do_move((0, 1), BLACK)
        assert gs.liberty_sets[0][0] == {(1, 0)}


class TestGameFlow:
    def test_stone_ages_and_copy_keeps_them(self):
        gs = play(GameState(9), [(0, 0), (1, 1), PASS_MOVE, (2, 2)])
        assert gs.stone_ages[0][0] == 3 and gs.stone_ages[1][1] == 2 and gs.stone_ages[2][2] == 0
        assert gs.stone_ages[4][4] == -1
        assert np.all(gs.copy().stone_ages == gs.stone_ages)  # quirk Q1 fixed

    def test_end_of_game_needs_white_to_move(self):
        gs = GameState(9)
        gs.do_move(PASS_MOVE)            # B passes
        assert not gs.do_move(PASS_MOVE)  # W passes: black to move -> not over (quirk Q3)
        assert gs.do_move(PASS_MOVE)      # B passes again: white to move -> over
        assert gs.is_end_of_game

    def test_winner_area_scoring(self):
        gs = GameState(5, komi=0.5)
        for y in range(5):
            gs.do_move((2, y), BLACK)
        # black owns column 2 (5 stones); eyeish singles only: none -> black 5, white 0.5
        assert gs.get_winner() == BLACK
        gs2 = GameState(5, komi=7.5)
        gs2.do_move((2, 2), BLACK)
        assert gs2.get_winner() == WHITE

    def test_handicaps(self):
        gs = GameState(19)
        gs.place_handicaps([(3, 3), (15, 15)])
        assert gs.current_player == WHITE and gs.history == []
        assert gs.handicaps == [(3, 3), (15, 15)]
        assert gs.board[3][3] == BLACK
        gs.do_move((10, 10))
        with pytest.raises(IllegalMove):
            gs.place_handicaps([(4, 4)])

    def test_current_player_assignment_invalidates_cache(self):
        gs = GameState(5)
        for p in [(0, 1), (1, 0), (1, 1)]:
            gs.do_move(p, BLACK)
        gs.current_player = BLACK
        assert (0, 0) in gs.get_legal_moves(include_eyes=True)
        assert (0, 0) not in gs.get_legal_moves(include_eyes=False)
        gs.current_player = WHITE  # for white (0,0) is suicide
        assert (0, 0) not in gs.get_legal_moves(include_eyes=True)

    def test_legal_move_order_is_x_major(self):
        moves = GameState(5).get_legal_moves()
        assert moves == [(x, y) for x in range(5) for y in range(5)]

    def test_zobrist_matches_seed0_tables(self):
        gs = GameState(9)
        gs.do_move((3, 4))
        assert gs.current_hash == gs.hash_lookup[BLACK][3][4]
        gs.do_move((4, 4))
        assert gs.current_hash == np.bitwise_xor(gs.hash_lookup[BLACK][3][4],
                                                 gs.hash_lookup[WHITE][4][4])
        assert gs.board[4][4] == WHITE and gs.board[0][0] == EMPTY
