"""Models: construction, evaluation, JSON/HDF5 save-load (spec: reference tests/test_policy.py)."""
import json
import os

import numpy as np
import pytest
import torch

from rocalphago_amd.engine import BLACK, GameState
from rocalphago_amd.models import kerasish as K
from rocalphago_amd.models.nn_util import NeuralNetBase
from rocalphago_amd.models.policy import CNNPolicy, ResnetPolicy
from rocalphago_amd.models.value import CNNValue, value_trainer

FEATS = ["board", "liberties", "sensibleness", "capture_size"]


def small(cls=CNNPolicy, **kw):
    args = dict(layers=3, filters_per_layer=8, device="cpu")
    args.update(kw)
    return cls(FEATS, **args)


def test_default_policy_evaluates():
    p = CNNPolicy(FEATS, device="cpu")
    out = p.eval_state(GameState())
    assert len(out) == 361
    assert abs(sum(pr for _, pr in out) - 1.0) < 1e-4


def test_batch_eval_state():
    res = small().batch_eval_state([GameState(), GameState()])
    assert len(res) == 2 and len(res[0]) == 361


@pytest.mark.parametrize("board", [19, 13, 9])
def test_output_shape(board):
    p = small(board=board)
    out = p.forward(p.preprocessor.state_to_tensor(GameState(board)))
    assert out.shape == (1, board * board)


def test_eval_state_renormalises_over_given_moves():
    p = small()
    moves = [(3, 3), (15, 15), (9, 9)]
    out = p.eval_state(GameState(), moves)
    assert [m for m, _ in out] == moves
    assert abs(sum(pr for _, pr in out) - 1.0) < 1e-5
    assert p.eval_state(GameState(), []) != []  # empty list -> all legal moves (quirk Q5)


@pytest.mark.parametrize("cls", [CNNPolicy, ResnetPolicy])
def test_save_load_separate_and_combined(tmp_path, cls):
    p = small(cls)
    m1, w1 = str(tmp_path / "p.json"), str(tmp_path / "w.h5")
    m2, w2 = str(tmp_path / "p2.json"), str(tmp_path / "w2.h5")
    p.save_model(m1)
    p.model.save_weights(w1, overwrite=True)
    p.save_model(m2, w2)
    a = NeuralNetBase.load_model(m1)
    a.model.load_weights(w1)
    b = NeuralNetBase.load_model(m2)
    assert type(a) is cls and type(b) is cls
    for x, y, z in zip(a.model.get_weights(), b.model.get_weights(), p.model.get_weights()):
        assert np.array_equal(x, y) and np.array_equal(x, z)
    spec = json.load(open(m2))
    assert spec["class"] == cls.__name__ and spec["feature_list"] == FEATS
    assert json.loads(spec["keras_model"])["class_name"] in ("Sequential", "Model")


def test_keras_weight_names_and_layer_order(tmp_path):
    from rocalphago_amd.io import h5lite
    p = small()
    path = str(tmp_path / "w.h5")
    p.model.save_weights(path)
    f = h5lite.File(path)
    names = [n.decode() for n in f.attrs["layer_names"]]
    assert names[0].startswith("convolution2d_") and names[-1].startswith("activation_")
    bias = [n for n in names if n.startswith("bias_")][0]
    assert [w.decode() for w in f[bias].attrs["weight_names"]] == ["param_0"]
    assert f[bias]["param_0"].shape == (361,)


def test_loads_reference_minimodel(ref_data):
    mm = CNNPolicy.load_model(os.path.join(ref_data, "minimodel.json"), device="cpu")
    assert mm.model.input_shape == (None, 12, 19, 19)
    w = mm.model.get_weights()
    assert [a.shape for a in w[:2]] == [(16, 12, 5, 5), (16,)] and w[-1].shape == (361,)
    assert np.abs(w[0]).max() <= 0.05 + 1e-6  # 'uniform' init
    out = mm.eval_state(GameState())
    assert len(out) == 361


def test_set_weights_validates_shapes():
    p = small()
    w = p.model.get_weights()
    with pytest.raises(ValueError):
        p.model.set_weights(w[:-1])
    w[0] = np.zeros((1, 1, 1, 1), np.float32)
    with pytest.raises(ValueError):
        p.model.set_weights(w)


def test_uniform_init_and_bias_zero():
    p = small()
    w = p.model.get_weights()
    assert all(np.abs(a).max() <= 0.05 + 1e-6 for a in w)
    assert np.all(w[-1] == 0)


def test_train_on_batch_reduces_loss_cpu():
    torch.manual_seed(0)
    p = small(seed=1)
    m = p.model
    m.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.5), metrics=["accuracy"])
    x = p.preprocessor.state_to_tensor(GameState())
    X = np.repeat(x, 4, axis=0)
    Y = np.zeros((4, 361), np.float32)
    Y[:, 60] = 1
    first = m.train_on_batch(X, Y)[0]
    for _ in range(30):
        last = m.train_on_batch(X, Y)[0]
    assert last < first


def test_sgd_decay_schedule():
    opt = K.SGD(lr=0.1, decay=0.5)
    assert opt.current_lr() == pytest.approx(0.1)
    opt.iterations = 2
    assert opt.current_lr() == pytest.approx(0.05)


def test_value_network():
    v = CNNValue(layers=3, filters_per_layer=8, device="cpu")
    assert v.preprocessor.output_dim == 49
    val = v.eval_state(GameState())
    assert -1 <= val <= 1
    vals = v.batch_eval_state([GameState(), GameState(9 + 10)])
    assert vals.shape == (2,)
    v.model.compile(loss="mse", optimizer=K.SGD(lr=0.1))
    X = v.preprocessor.states_to_tensor([GameState()] * 4)
    loss = v.model.train_on_batch(X, np.ones((4, 1), np.float32))
    assert np.isfinite(loss)


def test_value_trainer_reference_class():
    vt = value_trainer(filters_per_layer=8, layers=2, device="cpu")
    st = [GameState(), GameState()]
    st[1].do_move((3, 3))
    X, y = vt.get_samples(st, [BLACK, BLACK])
    assert X.shape == (2, 49, 19, 19) and list(y[:, 0]) == [1.0, -1.0]
    assert np.isfinite(vt.train(X, y, batch_size=2))


def test_resnet_batchnorm_learning_phase():
    r = small(ResnetPolicy, layers=4)
    assert r.model.uses_learning_phase
    out1 = r.forward(r.preprocessor.state_to_tensor(GameState()))
    assert np.isfinite(out1).all() and abs(out1.sum() - 1) < 1e-4


def test_resnet_generic_training_updates_running_stats():
    """Training-phase BN (batch statistics) through the generic executor: the running averages
    move with momentum and the loss decreases (regression: in-place running-stat updates used
    to invalidate tensors autograd saved)."""
    r = small(ResnetPolicy, layers=3)
    m = r.model
    m.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.05))
    S = m.input_shape[-1]
    X = (np.random.RandomState(0).rand(8, m.input_shape[1], S, S) > 0.5).astype(np.uint8)
    Y = np.eye(S * S, dtype=np.float32)[:8]
    names = [w for (_, w, _) in m.net.weight_names]
    i = names.index([n for n in names if n.endswith("_running_mean")][0])
    before = m.get_weights()[i].copy()
    l0 = m.train_on_batch(X, Y)
    for _ in range(5):
        l1 = m.train_on_batch(X, Y)
    assert l1 < l0
    assert np.abs(m.get_weights()[i] - before).max() > 0


def test_flat_buffer_complement_ranges():
    """engine.complement: the parts of the flat parameter buffer that the folded SGD step does
    not cover (stepped by the plain kernel), in order; the fold is skipped when they are too
    many (fused._TrunkPlan.SGD_FOLD_MAX_GAPS)."""
    from rocalphago_amd.models.engine import complement
    assert complement([(2, 5), (7, 9)], 12) == [(0, 2), (5, 7), (9, 12)]
    assert complement([(0, 12)], 12) == []
    assert complement([(5, 8), (0, 5)], 8) == []
    assert complement([], 4) == [(0, 4)]
