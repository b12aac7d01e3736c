"""The reference's command-line flows run on the GPU (HIP plans active): SL and RL policy
training on the reference fixtures, the value pipeline, and a GTP session with APV-MCTS."""
import io
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


FEATS = ["board", "ones", "turns_since"]  # 12 planes, like the reference's minimodel


@pytest.fixture(scope="module")
def cuda_only():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def fixtures(tmp_path_factory, cuda_only):
    """Self-made stand-ins for the reference fixtures (the GPU box has no reference tree):
    SGF records of rollout-policy games, the converter's HDF5 dataset, a small CNNPolicy spec
    and a weights file."""
    from rocalphago_amd._native import engine
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.features import converter
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.utils.go_util import save_gamestate_to_sgf
    d = tmp_path_factory.mktemp("fx")
    games = d / "games"
    games.mkdir()
    rp = engine().RolloutPolicy()
    for g in range(6):
        st = GameState()
        for k in range(120):
            mv = rp.sample(st.native, g * 1000 + k)
            st.do_move(None if mv < 0 else divmod(mv, 19))
        save_gamestate_to_sgf(st, str(games), "g%d.sgf" % g)
    data = str(d / "data.h5")
    converter.run_game_converter(["--features", ",".join(FEATS), "--outfile", data,
                                  "--directory", str(games)])
    pol = CNNPolicy(FEATS, filters_per_layer=16, layers=5, device="cpu", seed=5)
    spec = str(d / "model.json")
    pol.save_model(spec)
    weights = str(d / "weights.hdf5")
    pol.model.save_weights(weights)
    return {"data": data, "model": spec, "weights": weights}


def test_sl_cli_on_gpu(fixtures, tmp_path):
    from rocalphago_amd.training import supervised as sl
    out = str(tmp_path / "sl")
    sl.run_training([fixtures["model"], fixtures["data"], out, "--epochs", "2", "--seed", "3",
                     "-B", "32"])
    m = json.load(open(os.path.join(out, "metadata.json")))
    assert len(m["epochs"]) == 2
    assert m["epochs"][1]["loss"] < m["epochs"][0]["loss"] + 0.5
    assert np.isfinite(m["epochs"][1]["val_loss"])


def test_rl_cli_on_gpu(fixtures, tmp_path):
    from rocalphago_amd.training import reinforcement as rl
    out = str(tmp_path / "rl") + "/"
    rl.run_training([fixtures["model"], fixtures["weights"], out,
                     "--game-batch", "4", "--iterations", "2", "--move-limit", "30"])
    assert os.path.exists(os.path.join(out, "weights.00002.hdf5"))


def test_value_pipeline_on_gpu(cuda_only, tmp_path):
    import test_value_pipeline as tv
    tv.test_generate_dataset_and_train(tmp_path, device="cuda")


def test_gtp_with_apv_mcts_on_gpu(cuda_only):
    from rocalphago_amd.gtp.engine import run_gtp
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.models.value import CNNValue
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.search.apv import ParallelMCTSPlayer
    pol = CNNPolicy(DEFAULT_FEATURES, board=9, filters_per_layer=32, layers=3, device="cuda")
    val = CNNValue(DEFAULT_FEATURES + ["color"], board=9, filters_per_layer=32, layers=3,
                   device="cuda")
    player = ParallelMCTSPlayer(pol, val, n_playout=128, batch=32, rollout_device="gpu",
                                rollouts_per_leaf=2)
    cmds = iter(["1 boardsize 9", "2 clear_board", "3 genmove b", "4 play w E5",
                 "5 genmove b", "6 genmove w", "7 showboard", "8 quit"])
    out = io.StringIO()
    run_gtp(player, lambda: next(cmds), out=out)
    replies = out.getvalue().split("\n\n")
    assert replies[2].startswith("=3 ") and replies[2] != "=3 pass"
    assert replies[4].startswith("=5 ")
    assert "?" not in "".join(r[:1] for r in replies if r)
