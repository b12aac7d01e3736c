"""Supervised restart: a training job killed by an injected fault is relaunched
by the supervisor — as a child process — from its newest checkpoint and ends with the same
weights as an uninterrupted run; a hung job is killed by the progress watchdog."""
import json
import os
import sys

import numpy as np

from rocalphago_amd.models.policy import CNNPolicy
from rocalphago_amd.parallel import supervisor
from rocalphago_amd.training import supervised as sl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _args(ref_data, out, epochs):
    return [os.path.join(ref_data, "minimodel.json"),
            os.path.join(ref_data, "hdf5", "alphago-vs-lee-sedol-features.hdf5"), out,
            "--epochs", str(epochs), "--seed", "7", "-B", "16", "--epoch-length", "128",
            "--symmetries", "noop", "--learning-rate", "0.05", "--decay", "0.01"]


def _weights(ref_data, path):
    p = CNNPolicy.load_model(os.path.join(ref_data, "minimodel.json"), device="cpu")
    p.model.load_weights(path)
    return p.model.get_weights()


def test_resume_command_rewrites_weights_and_epochs(tmp_path):
    cmd = ["python", "train.py", "m.json", "d.h5", str(tmp_path), "--epochs", "5"]
    assert supervisor.resume_command(cmd, str(tmp_path), 5) == cmd  # nothing checkpointed yet
    for e in (0, 1, 2):
        open(tmp_path / ("weights.%05d.hdf5" % e), "w").close()
    got = supervisor.resume_command(cmd, str(tmp_path), 5)
    assert got[-4:] == ["--epochs", "2", "--weights", "weights.00002.hdf5"]
    assert supervisor.resume_command(cmd + ["--weights", "x"], str(tmp_path), 3) is None


def test_supervisor_restarts_failed_job_from_checkpoint(ref_data, tmp_path, monkeypatch):
    full = str(tmp_path / "full")
    sl.run_training(_args(ref_data, full, 3))
    cut = str(tmp_path / "cut")
    cmd = [sys.executable, "-m", "rocalphago_amd.training.supervised"] + _args(ref_data, cut, 3)
    monkeypatch.setenv("RAG_FAULT_AT_STEP", "12")  # dies in epoch 1 (steps 8..15)
    monkeypatch.setenv("PYTHONPATH", ROOT)
    logs = []
    rc = supervisor.run(cmd, cut, max_restarts=2, log=logs.append)
    assert rc == 0, logs
    assert sum("attempt" in l for l in logs) == 2
    a = _weights(ref_data, os.path.join(full, "weights.00002.hdf5"))
    b = _weights(ref_data, os.path.join(cut, "weights.00002.hdf5"))
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=0, atol=1e-6)
    meta = json.load(open(os.path.join(cut, "metadata.json")))
    assert len(meta["epochs"]) == 3


def test_supervisor_watchdog_kills_hung_job(tmp_path):
    script = tmp_path / "hang.py"
    script.write_text("import time\ntime.sleep(120)\n")
    logs = []
    rc = supervisor.run([sys.executable, str(script)], str(tmp_path), max_restarts=0,
                        hang_timeout=2, poll_s=0.2, log=logs.append)
    assert rc != 0
    assert any("no progress" in l for l in logs)


def test_resume_skips_incomplete_checkpoints(tmp_path):
    """A job killed while saving epoch 2 (weights without sidecar, or a sidecar whose weights
    never landed) resumes from epoch 1; the metadata's epoch log is cut back to the checkpoint
    so the lost epoch is re-run rather than skipped (supervisor resume)."""
    from rocalphago_amd.parallel.supervisor import latest_checkpoint
    from rocalphago_amd.training.supervised import resume_epoch_base
    d = tmp_path
    for e in (0, 1):
        (d / ("weights.%05d.hdf5" % e)).write_bytes(b"x")
        (d / ("weights.%05d.opt.json" % e)).write_text('{"epoch": %d, "iterations": 5}' % e)
    (d / "weights.00002.hdf5").write_bytes(b"trunc")  # killed before its sidecar... (legacy order)
    (d / "weights.00003.opt.json").write_text('{"epoch": 3}')  # ...or before its weights
    assert latest_checkpoint(str(d)) == (1, "weights.00001.hdf5")
    meta = {"epochs": [{"loss": 3.0}, {"loss": 2.0}, {"loss": 1.0}], "best_epoch": 2}
    assert resume_epoch_base(meta, {"epoch": 1, "iterations": 5}) == 2
    # best_epoch is recomputed from the entries kept (epoch 1's loss 2.0 beats epoch 0's 3.0)
    assert len(meta["epochs"]) == 2 and meta["best_epoch"] == 1
    # killed between the checkpoint of epoch 2 and metadata.json: the sidecar's logs restore
    # the missing entry, so entry i keeps describing weights.<i>.hdf5
    meta = {"epochs": [{"loss": 3.0}, {"loss": 2.0}], "best_epoch": 1}
    assert resume_epoch_base(meta, {"epoch": 2, "logs": {"loss": 0.5}}) == 3
    assert meta["epochs"][2] == {"loss": 0.5} and meta["best_epoch"] == 2
    # RL-style directories (no sidecars at all): newest weights file
    rl = tmp_path / "rl"
    rl.mkdir()
    for e in (0, 4, 2):
        (rl / ("weights.%05d.hdf5" % e)).write_bytes(b"x")
    assert latest_checkpoint(str(rl)) == (4, "weights.00004.hdf5")
