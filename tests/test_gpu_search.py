"""GPU rollout kernel (csrc/hip/rollout.hip) vs the native rollout policy, and APV-MCTS with
GPU rollouts + GPU network evaluation."""
import numpy as np
import pytest
import torch

from rocalphago_amd._native import engine
from rocalphago_amd.engine.gamestate import BLACK, GameState

pytestmark = pytest.mark.gpu
rg = engine()


@pytest.fixture(scope="module")
def gro():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rocalphago_amd.search.gpu_rollout import GpuRollouts
    rp = rg.RolloutPolicy()
    pat = np.random.RandomState(0).randn(rg.ROLLOUT_PATTERNS).astype(np.float32) * 0.3
    rp.pattern = pat
    return rp, GpuRollouts(rp)


def _random_positions(n, size, seed):
    rs = np.random.RandomState(seed)
    out = []
    rp = rg.RolloutPolicy()
    for i in range(n):
        st = GameState(size=size)
        for k in range(int(rs.randint(0, size * size * 1.2))):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            if mv < 0:
                st.do_move(None)
            else:
                st.do_move(divmod(mv, size))
            if st.is_end_of_game:
                break
        out.append(st)
    return out


@pytest.mark.parametrize("size", [9, 19])
def test_initial_logits_match_native_policy(gro, size):
    rp, g = gro
    states = _random_positions(24, size, 1 + size)
    lg = g.initial_logits(states)
    w = rp.weights
    pat = rp.pattern
    for i, st in enumerate(states):
        mv, fb, pt = rp.candidates(st.native)
        want = np.full(size * size, -np.inf, np.float32)
        for a, f, p in zip(mv, fb, pt):
            if not st.native.is_legal(int(a)):
                continue
            want[a] = pat[p] + sum(w[k] for k in range(rg.ROLLOUT_FEATURES) if f >> k & 1)
        fin = np.isfinite(want)
        assert np.array_equal(np.isfinite(lg[i]), fin), "candidate set differs at state %d" % i
        np.testing.assert_allclose(lg[i][fin], want[fin], rtol=1e-5, atol=1e-5)


def test_rollout_outcomes_match_native_statistics(gro):
    rp, g = gro
    st = GameState(size=9)
    wg, lg = g.run([st], R=4096, limit=1000, seed=7)
    assert (lg < 1000).all(), "GPU rollouts must end by two passes"
    wc = rp.rollouts([st.native] * 1024, seed=11, limit=1000, nthreads=8)
    pg = (wg == BLACK).mean()
    pc = (wc == BLACK).mean()
    assert abs(pg - pc) < 0.06, (pg, pc)
    lens = [rp.rollout(st.native, seed=s, limit=1000)[1] for s in range(200)]
    assert abs(lg.mean() - np.mean(lens)) < 0.1 * np.mean(lens)


def test_rollouts_bit_exact_vs_recorded_run():
    """Winners, lengths and initial logits of fixed positions + seed equal a run recorded on an
    MI355X before the kernel's latency rewrites (scripts/dbg/rollout_ref.py; 384 positions x 4
    playouts): the rewrites must not change a single game."""
    import os
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "scripts", "dbg"))
    from rollout_ref import states
    from rocalphago_amd.search.gpu_rollout import GpuRollouts
    sts, rp = states()
    gr = GpuRollouts(rp, torch.device("cuda"))
    w, ln = gr.run(sts, R=4, limit=500, seed=123)
    lg = gr.initial_logits(sts[:64])
    ref = np.load(os.path.join(root, "tests", "data", "rollout_ref.npz"))
    assert np.array_equal(ref["w"], w)
    assert np.array_equal(ref["ln"], ln)
    assert np.array_equal(ref["lg"], lg)


@pytest.mark.parametrize("size,slice_moves", [(19, 64), (19, 7), (9, 16)])
def test_sliced_rollouts_equal_one_launch(size, slice_moves):
    """Sliced playouts (the games parked in HBM between launches of at most ``slice_moves``
    moves) play exactly the games of one launch per playout: same winners, same lengths."""
    from rocalphago_amd.search.gpu_rollout import GpuRollouts
    rp = rg.RolloutPolicy()
    rp.pattern = np.random.RandomState(2).randn(rg.ROLLOUT_PATTERNS).astype(np.float32) * 0.3
    sts = _random_positions(40, size, 5 + size)
    one = GpuRollouts(rp, torch.device("cuda"), slice_moves=0)
    sl = GpuRollouts(rp, torch.device("cuda"), slice_moves=slice_moves)
    w0, l0 = one.run(sts, R=3, limit=500, seed=77)
    w1, l1 = sl.run(sts, R=3, limit=500, seed=77)
    assert np.array_equal(w0, w1)
    assert np.array_equal(l0, l1)
    assert l0.max() > slice_moves  # the games did span several launches


def test_gpu_rollouts_in_search_find_capture(gro):
    from rocalphago_amd.search.apv import ParallelMCTS
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from boards import parse
    from test_apv import UniformEval
    st, m = parse("O O O c .|X X X X .|. . . . .|. . . . .|. . . . .|")
    st.current_player = BLACK
    mc = ParallelMCTS(evaluator=UniformEval(), lmbda=1.0, n_playout=1024, batch=64,
                      rollout_limit=200, rollout_device="gpu", rollouts_per_leaf=8, seed=3)
    mv = mc.get_move(st)
    # black is winning here whatever it plays: every explored move must look good for black,
    # and most of all the capture (a sign error in the GPU result plumbing flips these)
    mvs, vis, q, _ = mc.root_statistics()
    c = m["c"][0] * 5 + m["c"][1]
    assert q[list(mvs).index(c)] > 0.5
    assert q[np.argmax(vis)] > 0.5
    assert mv is not None


def test_apv_with_gpu_networks(gro):
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.models.value import CNNValue
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.search.apv import ParallelMCTS
    dev = torch.device("cuda")
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=64, layers=4, device=dev,
                    seed=1)
    val = CNNValue(DEFAULT_FEATURES + ["color"], board=19, filters_per_layer=64, layers=4,
                   device=dev, seed=2)
    mc = ParallelMCTS(pol, val, lmbda=0.5, n_playout=512, batch=128, rollout_device="gpu",
                      rollouts_per_leaf=4)
    st = GameState()
    mv = mc.get_move(st)
    assert st.is_legal(mv)
    assert mc.stats["sims"] >= 500


def test_graph_replayed_evaluation_matches_eager(monkeypatch):
    """NetworkEvaluator.submit replays a captured HIP graph from the second wave of a size on;
    its priors / values / sensibleness equal the eager pass, also after a weight update."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.models.value import CNNValue
    from rocalphago_amd.search.apv import NetworkEvaluator
    dev = torch.device("cuda")
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=64, layers=4, device=dev,
                    seed=3)
    val = CNNValue(DEFAULT_FEATURES + ["color"], board=19, filters_per_layer=64, layers=4,
                   device=dev, seed=4)
    boards = [s.native for s in _random_positions(40, 19, 7)]
    other = [s.native for s in _random_positions(40, 19, 8)]
    eager = NetworkEvaluator(pol, val)
    ref = [eager.submit(b).result() for b in (boards, other)]
    ev = NetworkEvaluator(pol, val, graph=True)
    for rep in range(3):  # eager, capture + replay, replay
        for b, r in zip((boards, other), ref):
            got = ev.submit(b).result()
            for g, e in zip(got, r):
                assert np.array_equal(g, e), rep
    assert len(ev._graphs) == 1
    # a larger wave reallocates the activations: graphs of the smaller size must be re-captured
    small = boards[:20]
    ref_small = NetworkEvaluator(pol, val).submit(small).result()
    ev2 = NetworkEvaluator(pol, val, graph=True)
    for b in (small, small, small, boards + other, small, small):
        got = ev2.submit(b).result()
        if len(b) == 20:
            for g, e in zip(got, ref_small):
                assert np.array_equal(g, e)
    # a weight update reaches the replayed graph through the packed-weight refresh
    w = pol.model.get_weights()
    w[0] = w[0] * 0.5
    pol.model.set_weights(w)
    ref2 = NetworkEvaluator(pol, val).submit(boards).result()
    got2 = ev.submit(boards).result()
    assert not np.array_equal(ref2[0], ref[0][0])
    for g, e in zip(got2, ref2):
        assert np.array_equal(g, e)


def test_two_stream_evaluation_matches_one_stream(monkeypatch):
    """two_streams=True runs the value trunk on a second stream; priors / values /
    sensibleness equal the single-stream pass for repeated waves of two sizes."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.models.value import CNNValue
    from rocalphago_amd.search.apv import NetworkEvaluator
    dev = torch.device("cuda")
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=4, device=dev,
                    seed=3)
    val = CNNValue(DEFAULT_FEATURES + ["color"], board=19, filters_per_layer=192, layers=4,
                   device=dev, seed=4)
    waves = [[s.native for s in _random_positions(n, 19, 11 + n)] for n in (64, 33)]
    one = NetworkEvaluator(pol, val, two_streams=False)
    ref = [one.submit(b).result() for b in waves]
    two = NetworkEvaluator(pol, val)
    assert two.two_streams
    for rep in range(3):
        pend = [two.submit(b) for b in waves]  # both waves in flight before reading either
        for p, r in zip(pend, ref):
            for g, e in zip(p.result(), r):
                assert np.array_equal(g, e), rep


@pytest.mark.parametrize("superko,graph", [(False, "0"), (False, "1"), (True, "0")])
def test_packed_wave_matches_board_path(monkeypatch, superko, graph):
    """submit_wave (leaves packed natively into pinned slots, one GPU pass per wave, optionally
    graph-replayed) gives the same priors / values / sensible masks as evaluating the wave's
    board objects (NetworkEvaluator.submit), for a mid-game root, also with positional superko."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.models.value import CNNValue
    from rocalphago_amd.search.apv import NetworkEvaluator, _Slots
    dev = torch.device("cuda")
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=64, layers=4, device=dev,
                    seed=5)
    val = CNNValue(DEFAULT_FEATURES + ["color"], board=19, filters_per_layer=64, layers=4,
                   device=dev, seed=6)
    st = _random_positions(1, 19, 21)[0]
    root = GameState(size=19, enforce_superko=superko)
    for mv in st.history:
        root.do_move(mv)
    ev = NetworkEvaluator(pol, val, graph=graph == "1")
    assert ev.wave_capable(19)
    slots = _Slots(dev, 2)
    s = rg.Search(root.native, 4)
    s.lmbda = 0.0
    s.parallel_select_min = 1 << 20  # serial, deterministic descents
    rs = np.random.RandomState(0)
    wid, n = s.select(1)  # expand the root first
    r0 = ev.submit(s.leaf_boards(wid)).result()
    s.backup_value(wid, np.ascontiguousarray(r0[0]), r0[1], r0[2])
    for rep in range(4):  # eager, eager (graph: capture), replay, replay
        wid, n = s.select(48)
        assert n == 48
        ref = ev.submit(s.leaf_boards(wid)).result()
        got = ev.submit_wave(s, wid, n, slots, 48).result()
        for g, e in zip(got, ref):
            assert g.shape == e.shape
            assert np.array_equal(g, e), rep
        s.backup_value(wid, np.ascontiguousarray(got[0]), rs.uniform(-1, 1, n).astype(np.float32),
                       got[2])
