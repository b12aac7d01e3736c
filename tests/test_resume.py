"""Checkpoint / resume with fault injection: a run killed mid-epoch and
resumed from its last checkpoint (weights + optimizer/cursor sidecar) ends bit-identical to an
uninterrupted run."""
import json
import os

import numpy as np
import pytest

from rocalphago_amd.models.policy import CNNPolicy
from rocalphago_amd.training import supervised as sl


def _args(ref_data, out, epochs, extra=()):
    return [os.path.join(ref_data, "minimodel.json"),
            os.path.join(ref_data, "hdf5", "alphago-vs-lee-sedol-features.hdf5"), out,
            "--epochs", str(epochs), "--seed", "7", "-B", "16", "--epoch-length", "128",
            "--symmetries", "noop", "--learning-rate", "0.05", "--decay", "0.01"] + list(extra)


def _weights(ref_data, path):
    p = CNNPolicy.load_model(os.path.join(ref_data, "minimodel.json"), device="cpu")
    p.model.load_weights(path)
    return p.model.get_weights()


def test_fault_and_resume_matches_uninterrupted(ref_data, tmp_path, monkeypatch):
    full = str(tmp_path / "full")
    sl.run_training(_args(ref_data, full, 2))
    cut = str(tmp_path / "cut")
    monkeypatch.setenv("RAG_FAULT_AT_STEP", "12")  # epoch 1 covers steps 8..15
    with pytest.raises(RuntimeError, match="injected fault"):
        sl.run_training(_args(ref_data, cut, 2))
    monkeypatch.delenv("RAG_FAULT_AT_STEP")
    assert os.path.exists(os.path.join(cut, "weights.00000.hdf5"))
    assert not os.path.exists(os.path.join(cut, "weights.00001.hdf5"))
    side = json.load(open(os.path.join(cut, "weights.00000.opt.json")))
    assert side["iterations"] == 8 and side["epoch"] == 0
    sl.run_training(_args(ref_data, cut, 1, ["--weights", "weights.00000.hdf5"]))
    a = _weights(ref_data, os.path.join(full, "weights.00001.hdf5"))
    b = _weights(ref_data, os.path.join(cut, "weights.00001.hdf5"))
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=0, atol=1e-6)
    meta = json.load(open(os.path.join(cut, "metadata.json")))
    assert len(meta["epochs"]) == 2
    lines = open(os.path.join(cut, "metrics.jsonl")).read().strip().splitlines()
    assert [json.loads(l)["epoch"] for l in lines] == [0, 1]
    assert json.loads(lines[-1])["step"] == 16
