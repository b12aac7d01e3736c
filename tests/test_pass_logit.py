"""Optional pass logit (reference policy head policy.py:124-136 has none): a
``PassLogit`` layer appends W . z + b to the S*S position logits, softmax over S*S + 1 classes.
Off by default; on: JSON/HDF5 round trip, players and both searches may pass, and the fused HIP
head matches the fp32 torch reference (GPU tests)."""

import numpy as np
import pytest

from rocalphago_amd._native import engine
from rocalphago_amd.engine.gamestate import PASS_MOVE, GameState
from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
from rocalphago_amd.models import kerasish as K
from rocalphago_amd.models.nn_util import NeuralNetBase
from rocalphago_amd.models.policy import CNNPolicy, has_pass_logit
from rocalphago_amd.players.ai import GreedyPolicyPlayer

FEATS = ["board", "ones", "turns_since", "liberties", "sensibleness"]
rg = engine()


def _policy(device="cpu", board=7, **kw):
    return CNNPolicy(FEATS, board=board, filters_per_layer=8, layers=2, device=device, seed=5,
                     pass_logit=True, **kw)


def test_default_has_no_pass():
    p = CNNPolicy(FEATS, board=7, filters_per_layer=8, layers=2, device="cpu", seed=5)
    assert not has_pass_logit(p)
    assert p.forward(p.preprocessor.state_to_tensor(GameState(7))).shape == (1, 49)


def test_pass_logit_forward_and_roundtrip(tmp_path):
    p = _policy()
    assert has_pass_logit(p)
    W, b = p.model.get_weights()[-2:]
    assert W.shape == (49,) and b.shape == (1,)
    rs = np.random.RandomState(0)
    w = p.model.get_weights()
    w[-2] = rs.randn(49).astype(np.float32) * 0.1
    w[-1] = np.array([0.7], np.float32)
    p.model.set_weights(w)
    x = p.preprocessor.state_to_tensor(GameState(7))
    out = p.forward(x)
    assert out.shape == (1, 50) and abs(out.sum() - 1) < 1e-5
    probs = dict(p.eval_state(GameState(7)))
    assert PASS_MOVE in probs and abs(sum(probs.values()) - 1) < 1e-5
    js, h5 = str(tmp_path / "p.json"), str(tmp_path / "p.h5")
    p.save_model(js, h5)
    q = NeuralNetBase.load_model(js, device="cpu")  # the same (fp32) executor as p
    assert has_pass_logit(q)
    np.testing.assert_allclose(q.forward(x), out, rtol=1e-6, atol=1e-7)


def test_pass_logit_trains_and_greedy_player_passes():
    p = _policy()
    p.model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.5))
    x = np.stack([p.preprocessor.state_to_tensor(GameState(7))[0]] * 4)
    y = np.zeros((4, 50), np.float32)
    y[:, 49] = 1  # always pass
    before = p.model.get_weights()[-1].copy()
    for _ in range(30):
        p.model.train_on_batch(x, y)
    assert p.model.get_weights()[-1][0] > before[0]
    assert GreedyPolicyPlayer(p).get_move(GameState(7)) is PASS_MOVE


def test_native_search_expands_a_pass_child():
    st = GameState(size=5)
    s = rg.Search(st.native, 1)
    s.lmbda = 0.0
    s.pass_prior = True
    wid, n = s.select(1)
    pri = np.full((1, 26), 0.5 / 25, np.float32)
    pri[0, 25] = 0.5  # pass gets half the prior mass
    s.backup_value(wid, pri, np.zeros(1, np.float32))
    mv, vis, q, prior = s.root_stats()
    assert mv[-1] == -1 and len(mv) == 26
    assert abs(prior[-1] - 0.5) < 1e-6


@pytest.mark.gpu
def test_hip_pass_head_matches_torch(cuda):
    g = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=32, layers=3, device="cuda",
                  seed=3, pass_logit=True)
    c = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=32, layers=3, device="cpu",
                  seed=3, pass_logit=True)
    rs = np.random.RandomState(1)
    w = g.model.get_weights()
    w[-2] = rs.randn(361).astype(np.float32) * 0.05
    w[-1] = np.array([0.3], np.float32)
    g.model.set_weights(w)
    c.model.set_weights(w)
    assert g.model._plan_for() is not None
    X = (rs.rand(8, 48, 19, 19) > 0.6).astype(np.float32)
    pg, pc = g.forward(X), c.forward(X)
    assert pg.shape == (8, 362)
    assert np.abs(pg - pc).max() < 2e-3 * max(1.0, np.abs(pc).max() * 362)
    for m in (g, c):
        m.model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.1))
    Y = np.zeros((8, 362), np.float32)
    Y[np.arange(8), [361, 3, 361, 50, 7, 361, 200, 100]] = 1
    w0 = c.model.get_weights()
    lg, lc = g.model.train_on_batch(X, Y), c.model.train_on_batch(X, Y)
    assert abs(lg - lc) < 1e-2 * abs(lc)
    rel = []
    for a, b, b0 in zip(g.model.get_weights(), c.model.get_weights(), w0):
        rel.append(float(np.abs(a - b).max() / max(np.abs(b - b0).max(), 1e-6)))
    # the head-level parameters (position Bias, PassLogit W and b: fp32 logits on both sides)
    # match to 2 % of their update; the conv tensors carry the bf16 trunk's rounding (<= 20 %
    # of a tensor's largest update, which is ~1e-3 here)
    assert max(rel[-3:]) < 2e-2, rel
    assert max(rel) < 0.2, rel
    dWg = g.model.get_weights()[-2] - w0[-2]
    dWc = c.model.get_weights()[-2] - w0[-2]
    assert np.abs(dWc).max() > 1e-4
    assert np.abs(dWg - dWc).max() < 2e-2 * np.abs(dWc).max()


@pytest.mark.gpu
def test_gpu_players_and_search_can_pass(cuda):
    """Device move selection (sample.hip over S*S + 1 classes) and APV-MCTS with a pass child."""
    from rocalphago_amd.players.ai import ProbabilisticPolicyPlayer
    from rocalphago_amd.search.apv import ParallelMCTS
    g = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=32, layers=3, device="cuda",
                  seed=3, pass_logit=True)
    w = g.model.get_weights()
    w[-1] = np.array([40.0], np.float32)  # pass dominates
    g.model.set_weights(w)
    states = [GameState() for _ in range(4)]
    assert GreedyPolicyPlayer(g).get_moves(states) == [PASS_MOVE] * 4
    assert ProbabilisticPolicyPlayer(g).get_moves(states) == [PASS_MOVE] * 4
    mc = ParallelMCTS(g, None, lmbda=1.0, n_playout=256, batch=64, rollout_device="gpu")
    mc.get_move(GameState())
    mv, vis, _, prior = mc.root_statistics()
    assert -1 in list(mv) and prior[list(mv).index(-1)] > 0.99
