"""APV-MCTS (native tree, virtual loss, negamax backup, batched evaluation) and the fast
rollout policy. CPU only; the GPU rollout kernel is checked in tests/test_gpu_search.py."""
import numpy as np
import pytest

from rocalphago_amd._native import engine
from rocalphago_amd.engine.gamestate import BLACK, WHITE, GameState
from rocalphago_amd.search.apv import ParallelMCTS, ParallelMCTSPlayer

from boards import parse

rg = engine()


class UniformEval(object):
    """Evaluator stub: uniform priors, optional value function of the native board."""

    def __init__(self, value=None):
        self.value = value
        self.calls = []

    def __call__(self, boards):
        self.calls.append(len(boards))
        n = len(boards)
        P = boards[0].size ** 2
        priors = np.full((n, P), 1.0 / P, np.float32)
        values = None
        if self.value is not None:
            values = np.array([self.value(b) for b in boards], np.float32)
        return priors, values


# ---------------------------------------------------------------------------- rollout policy
def test_rollout_candidates_features():
    st, m = parse(". . . . .|"
                  ". X O . .|"
                  ". O a . .|"
                  ". . O . .|"
                  ". . . . .|")
    st.current_player = BLACK
    rp = rg.RolloutPolicy()
    mv, fb, pat = rp.candidates(st.native)
    S = st.size
    feats = dict(zip(mv.tolist(), fb.tolist()))
    # black X at (1,1) has liberties (0,1),(1,0): not in atari; 'a' is surrounded by white on
    # two sides: playing there is self-atari-ish only if libs <= 1 -> (2,2) has 2 empty nbrs
    a = m['a'][0] * S + m['a'][1]
    assert a in feats
    RESP, SAVE, CAP, SELF, NEAR2, OWN, EDGE = range(7)
    assert not feats[a] >> CAP & 1
    # corner (0,0) is on the edge
    assert feats[0] >> EDGE & 1
    # every candidate is empty
    assert all(st.native.color_at(int(p)) == 0 for p in mv)
    assert len(mv) == len(pat)


def test_rollout_capture_and_save_atari_features():
    st, m = parse(". X . . .|"
                  "X O c . .|"
                  ". X . . .|"
                  ". . . . .|"
                  ". . . . .|")
    S = st.size
    st.current_player = BLACK
    rp = rg.RolloutPolicy()
    mv, fb, _ = rp.candidates(st.native)
    feats = dict(zip(mv.tolist(), fb.tolist()))
    c = m['c'][0] * S + m['c'][1]
    assert feats[c] >> 2 & 1, "capture feature at the last liberty of the white stone"
    st.current_player = WHITE
    mv, fb, _ = rp.candidates(st.native)
    feats = dict(zip(mv.tolist(), fb.tolist()))
    assert feats[c] >> 1 & 1, "save-atari feature for white"


def test_rollouts_reach_the_end_and_are_seeded():
    st = GameState(size=9)
    rp = rg.RolloutPolicy()
    w1, n1 = rp.rollout(st.native, seed=5, limit=1000)
    w2, n2 = rp.rollout(st.native, seed=5, limit=1000)
    assert (w1, n1) == (w2, n2)
    assert w1 in (BLACK, WHITE, 0) and 40 < n1 < 1000
    ws = rp.rollouts([st.native] * 64, seed=3, limit=1000, nthreads=4)
    assert set(np.unique(ws)).issubset({-1, 0, 1})
    # the original state is untouched
    assert st.native.move_count == 0


def test_rollout_weights_roundtrip():
    rp = rg.RolloutPolicy()
    w = rp.weights
    w[0] = 7.0
    rp.weights = w
    assert rp.weights[0] == 7.0
    p = np.zeros(rg.ROLLOUT_PATTERNS, np.float32)
    p[5] = 1.5
    rp.pattern = p
    assert rp.pattern[5] == 1.5


# ---------------------------------------------------------------------------- native tree
def test_virtual_loss_spreads_a_wave():
    st = GameState(size=7)
    s = rg.Search(st.native, 2)
    s.lmbda = 0.0
    wid, n = s.select(1)
    assert n == 1
    s.backup_value(wid, np.full((1, 49), 1 / 49.0, np.float32), np.zeros(1, np.float32))
    wid, n = s.select(16)
    assert n == 16
    firsts = set()
    for b in s.leaf_boards(wid):
        firsts.add(b.last_moves[0])
    assert len(firsts) == 16, "virtual loss must send the 16 descents to different children"
    s.backup_value(wid, np.full((n, 49), 1 / 49.0, np.float32), np.zeros(n, np.float32))
    assert s.root_visits == 17
    assert s.pending_waves == 0


def test_async_rollout_waves_keep_virtual_loss():
    """With lambda > 0 a wave holds its virtual losses until its rollouts are backed up, and
    later waves can be selected and value-backed-up meanwhile (the APV pipeline)."""
    st = GameState(size=7)
    s = rg.Search(st.native, 2)
    s.lmbda = 0.5
    pri = np.full((64, 49), 1 / 49.0, np.float32)
    w0, n0 = s.select(1)
    s.backup_value(w0, pri, np.zeros(n0, np.float32))
    s.backup_rollout(w0, np.zeros(n0, np.float32))
    w1, n1 = s.select(8)
    s.backup_value(w1, pri, np.zeros(n1, np.float32))
    w2, n2 = s.select(8)  # w1's rollouts still in flight
    firsts = {b.last_moves[0] for b in s.leaf_boards(w1)} | \
        {b.last_moves[0] for b in s.leaf_boards(w2)}
    assert len(firsts) == 16, "in-flight waves must repel new descents"
    assert s.pending_waves == 2
    with pytest.raises(RuntimeError):
        s.backup_rollout(w2, np.zeros(n2, np.float32))  # value backup must come first
    s.backup_value(w2, pri, np.zeros(n2, np.float32))
    s.backup_rollout(w2, np.ones(n2, np.float32))  # black wins every rollout
    s.backup_rollout(w1, np.ones(n1, np.float32))
    assert s.pending_waves == 0
    mv, vis, q, _ = s.root_stats()
    # black (to move at the root) wins the rollouts: mixed Q of explored children > 0
    assert (q[vis > 0] > 0).all()
    assert s.rollouts == 17


def test_negamax_sign_prefers_good_moves_for_the_mover():
    # value net stub: +1 for the player to move if it is WHITE and black played corner (0,0),
    # i.e. black's move (0,0) is terrible for black -> black must avoid it
    st = GameState(size=5)

    def value(b):
        bad = b.color_at(0) == BLACK
        return (1.0 if b.current_player == WHITE else -1.0) if bad else 0.0

    ev = UniformEval(value)
    m = ParallelMCTS(evaluator=ev, lmbda=0.0, n_playout=400, batch=8, c_puct=1.0)
    # a value net is given through the evaluator, so keep lmbda at 0
    m.lmbda = 0.0
    m.get_move(st)
    mv, vis, q, pr = m.root_statistics()
    corner = int(np.where(mv == 0)[0][0])
    assert q[corner] < -0.9
    assert vis[corner] <= np.sort(vis)[len(vis) // 2]
    assert m.get_move(st) != (0, 0)


def test_search_finds_capture_with_rollouts():
    # black to play can capture 3 white stones at 'c'; with rollouts only MCTS should find it
    st, m = parse("O O O c .|"
                  "X X X X .|"
                  ". . . . .|"
                  ". . . . .|"
                  ". . . . .|")
    st.current_player = BLACK
    mc = ParallelMCTS(evaluator=UniformEval(), lmbda=1.0, n_playout=1500, batch=32,
                      rollout_limit=200, seed=3)
    mc.get_move(st)
    mv, vis, q, _ = mc.root_statistics()
    assert q[list(mv).index(m['c'][0] * 5 + m['c'][1])] > 0.5
    assert q[np.argmax(vis)] > 0.5


def test_tree_reuse_keeps_visits():
    st = GameState(size=7)
    mc = ParallelMCTS(evaluator=UniformEval(lambda b: 0.0), lmbda=0.0, n_playout=200, batch=16)
    mv = mc.get_move(st)
    mvs, vis, _, _ = mc.root_statistics()
    kept = int(vis[np.where(mvs == mv[0] * 7 + mv[1])[0][0]])
    mc.update_with_move(mv)
    assert mc._search.root_visits == kept
    st.do_move(mv)
    mc.search(st, 50)
    assert mc._search.root_visits >= kept + 50 - 1


def test_terminal_positions_are_scored_exactly():
    st = GameState(size=5)
    st.do_move(None)
    st.do_move(None)  # black, white pass -> black to move; game not over (quirk Q3)
    mc = ParallelMCTS(evaluator=UniformEval(lambda b: 0.0), lmbda=0.0, n_playout=64, batch=8)
    mc.get_move(st)
    assert mc._search.terminal >= 0


def test_player_plays_legal_moves_and_passes():
    ev = UniformEval(lambda b: 0.0)
    p = ParallelMCTSPlayer(evaluator=ev, lmbda=0.0, n_playout=32, batch=8)
    st = GameState(size=7)
    for _ in range(8):
        mv = p.get_move(st)
        assert mv is None or st.is_legal(mv)
        st.do_move(mv)
    # only own eyes left -> pass
    st2, _ = parse("X X X|X . X|X X X|")
    st2.current_player = BLACK
    assert ParallelMCTSPlayer(evaluator=ev, lmbda=0.0, n_playout=8, batch=4).get_move(st2) \
        is None


@pytest.mark.parametrize("lmbda", [0.0, 0.5, 1.0])
def test_network_evaluator_cpu(lmbda):
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.models.value import CNNValue
    feats = ["board", "ones", "sensibleness"]
    pol = CNNPolicy(feats, board=7, filters_per_layer=8, layers=2, device="cpu", seed=1)
    val = CNNValue(feats + ["color"], board=7, filters_per_layer=8, layers=2, device="cpu",
                   seed=2)
    mc = ParallelMCTS(pol, val, lmbda=lmbda, n_playout=96, batch=16, rollout_limit=150)
    st = GameState(size=7)
    mv = mc.get_move(st)
    assert st.is_legal(mv)
    assert mc.stats["sims"] >= 90


def test_parallel_select_claims_distinct_leaves():
    """Waves of B >= parallel_select_min descend on the pool (atomic virtual loss + leaf claim):
    exactly B distinct leaves, virtual loss returned on backup."""
    st = GameState(size=9)
    s = rg.Search(st.native, 4)
    s.lmbda = 0.5
    s.parallel_select_min = 16
    rs = np.random.RandomState(0)
    total = 0
    for _ in range(12):
        wid, n = s.select(64)
        if n == 0:
            continue
        nodes = s.leaf_nodes(wid)
        assert len(nodes) == n == len(set(nodes))
        pri = rs.dirichlet(np.ones(81), size=n).astype(np.float32)
        s.backup_value(wid, pri, rs.uniform(-1, 1, n).astype(np.float32))
        s.backup_rollout(wid, rs.uniform(-1, 1, n).astype(np.float32))
        total += n
    assert s.pending_waves == 0
    assert s.root_visits == total > 600
    mv, vis, _, _ = s.root_stats()
    assert vis.sum() == total - 1


def test_slot_pool_restarts_rotation_when_reallocated(monkeypatch):
    """After a shape change empties the pool, the rotation restarts at the oldest slot: with
    two waves in flight a stale odd counter would hand out the slot of the wave still in flight
    (_Slots.take)."""
    from types import SimpleNamespace

    from rocalphago_amd.search import apv

    def fake_slot(B, S, F, PW, device, host_ladders):
        return SimpleNamespace(B=B, S=S, planes=np.zeros((1, F)), o_pri=np.zeros((1, PW)),
                               h={"ladders": 1} if host_ladders else {})
    monkeypatch.setattr(apv, "_Slot", fake_slot)
    slots = apv._Slots("cpu", 2)
    a, b = slots.take(64, 19, 48, 362, False), slots.take(64, 19, 48, 362, False)
    assert slots.take(64, 19, 48, 362, False) is a  # next = 1 (odd) now
    c = slots.take(64, 9, 48, 82, False)  # new board size: pool reallocated
    d = slots.take(64, 9, 48, 82, False)
    assert c is not d
    assert slots.take(64, 9, 48, 82, False) is c  # the oldest wave's slot, not d (in flight)
    assert slots.take(64, 9, 48, 82, False) is d


def test_tree_arena_cache_is_bounded_and_trimmable():
    """The warm tree arenas a finished Search leaves for the next one are capped and can be
    released (MapCache kept up to 6 GiB resident for the life of the process)."""
    s = rg.Search(GameState().native, 2)
    s.select(8)
    del s
    assert 0 < rg.tree_cache_bytes() <= (2560 << 20)
    assert rg.trim_tree_cache() > 0
    assert rg.tree_cache_bytes() == 0
