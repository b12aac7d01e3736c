"""Substrate CLI flags: --dtype on the trainers/GTP engine, --mcts-threads /
--leaf-batch / --virtual-loss on the GTP engine's MCTS player."""
import os

import pytest
import torch

from rocalphago_amd.gtp import engine as gtp_engine
from rocalphago_amd.models.kerasish import default_precision
from rocalphago_amd.models.policy import CNNPolicy
from rocalphago_amd.models.value import CNNValue


def _save(tmp_path, net, name):
    p = str(tmp_path / name)
    net.save_model(p)
    return p


def _main_player(monkeypatch, argv):
    got = {}
    monkeypatch.setattr(gtp_engine, "run_gtp", lambda player, **kw: got.setdefault("p", player))
    gtp_engine.main(argv)
    return got["p"]


def test_gtp_mcts_flags(tmp_path, monkeypatch):
    pol = CNNPolicy(["board", "ones", "sensibleness"], board=9, layers=2, filters_per_layer=8)
    val = CNNValue(["board", "ones", "sensibleness", "color"], board=9, layers=2,
                   filters_per_layer=8, dense=16)
    pj, vj = _save(tmp_path, pol, "p.json"), _save(tmp_path, val, "v.json")
    player = _main_player(monkeypatch, [pj, "--player", "mcts", "--value", vj, "--playouts",
                                        "32", "--mcts-threads", "3", "--leaf-batch", "16",
                                        "--virtual-loss", "5", "--c-puct", "2.5",
                                        "--dtype", "fp32"])
    m = player.mcts
    assert (m.nthreads, m.batch, m.virtual_loss, m.n_playout) == (3, 16, 5, 32)
    assert m.c_puct == 2.5 and m.lmbda == 0.5
    assert m.evaluator.policy.model.precision == "fp32"
    assert m.evaluator.value.model.precision == "fp32"
    # no value net: rollouts only
    player = _main_player(monkeypatch, [pj, "--player", "mcts", "--playouts", "8"])
    assert player.mcts.lmbda == 1.0 and player.mcts.evaluator.policy.model.precision == "bf16"


def test_precision_switch():
    pol = CNNPolicy(["board", "ones"], board=9, layers=2, filters_per_layer=8)
    m = pol.model
    assert m.precision == default_precision() == "bf16"
    x = torch.rand(2, 4, 9, 9)
    y16 = pol.forward(x)
    assert pol.set_dtype("fp32") is pol and m.precision == "fp32"
    assert m._plan_for() is None
    assert torch.allclose(torch.as_tensor(pol.forward(x)), torch.as_tensor(y16))
    with pytest.raises(ValueError):
        m.set_precision("fp16")


def test_rag_dtype_env(monkeypatch):
    monkeypatch.setenv("RAG_DTYPE", "fp32")
    assert CNNPolicy(["board"], board=9, layers=1, filters_per_layer=4).model.precision == "fp32"
    monkeypatch.setenv("RAG_DTYPE", "int4")
    with pytest.raises(ValueError):
        default_precision()


@pytest.mark.parametrize("mod", ["supervised", "value_trainer", "reinforcement"])
def test_trainer_dtype_flag(mod):
    import importlib
    src = open(importlib.import_module("rocalphago_amd.training." + mod).__file__).read()
    assert '"--dtype"' in src and ".set_dtype(args.dtype)" in src


@pytest.mark.gpu
def test_fp32_matches_bf16_plan(cuda):
    """fp32 (reference precision) and the bf16 fused plan agree to bf16 accuracy on the GPU."""
    pol = CNNPolicy(["board", "ones", "turns_since"], board=19, layers=4, filters_per_layer=64)
    pol.model.to(cuda)
    x = (torch.rand(8, 12, 19, 19, device=cuda) > 0.7).float()
    y16 = torch.as_tensor(pol.forward_device(x)).float()
    pol.set_dtype("fp32")
    y32 = torch.as_tensor(pol.forward_device(x)).float()
    assert pol.model._plan_for() is None
    assert torch.allclose(y16.sum(-1), torch.ones(8, device=cuda), atol=1e-3)
    assert (y16 - y32).abs().max().item() < 2e-2 * y32.max().item() + 1e-4
    assert os.environ.get("RAG_ALLOW_TORCH_FALLBACK", "0") != "1"
