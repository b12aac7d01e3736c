"""Value-network pipeline (C37/C59): self-play position dataset -> HDF5 -> value training CLI."""
import json
import os

import numpy as np

from rocalphago_amd.features.preprocessing import VALUE_FEATURES
from rocalphago_amd.io import h5lite
from rocalphago_amd.models.policy import CNNPolicy
from rocalphago_amd.models.value import CNNValue
from rocalphago_amd.players.ai import ProbabilisticPolicyPlayer
from rocalphago_amd.training import value_trainer as vt


def test_generate_dataset_and_train(tmp_path, device="cpu"):
    pol = CNNPolicy(["board", "ones", "sensibleness"], board=7, filters_per_layer=8, layers=2,
                    device=device, seed=1)
    player = ProbabilisticPolicyPlayer(pol, move_limit=60)
    data = str(tmp_path / "values.h5")
    X, y = vt.generate_value_dataset(player, 24, out_file=data, board=7, move_limit=60,
                                     rng=np.random.RandomState(1), batch_games=8)
    assert X.shape == (24, 49, 7, 7) and X.dtype == np.uint8
    assert set(np.unique(y)).issubset({-1.0, 0.0, 1.0})
    with h5lite.File(data) as f:
        assert f["states"].shape == (24, 49, 7, 7)
        assert np.array_equal(f["values"][()], y)
    val = CNNValue(VALUE_FEATURES, board=7, filters_per_layer=8, layers=2, device=device, seed=2)
    spec = str(tmp_path / "value.json")
    val.save_model(spec)
    out = str(tmp_path / "vout")
    meta = vt.run_training([spec, data, out, "--epochs", "2", "--minibatch", "4",
                            "--train-val-test", "0.75", "0.25", "0.0"])
    assert len(meta["epochs"]) == 2 and "val_loss" in meta["epochs"][0]
    assert os.path.exists(os.path.join(out, "weights.00001.hdf5"))
    assert json.load(open(os.path.join(out, "metadata.json")))["epochs"][1]["loss"] >= 0
    # resume
    vt.run_training([spec, data, out, "--epochs", "1", "--minibatch", "4",
                     "--weights", "weights.00001.hdf5"])
