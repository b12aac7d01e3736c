"""Trainers and converter (spec: reference tests/test_supervised_policy_trainer.py,
test_reinforcement_policy_trainer.py, test_game_converter.py)."""
import json
import os

import numpy as np
import numpy.testing as npt
import pytest

from rocalphago_amd.engine import BLACK, PASS_MOVE, WHITE, GameState
from rocalphago_amd.features.converter import run_game_converter
from rocalphago_amd.io import h5lite
from rocalphago_amd.models import kerasish as K
from rocalphago_amd.models.policy import CNNPolicy
from rocalphago_amd.training import reinforcement as rl
from rocalphago_amd.training import supervised as sl
from rocalphago_amd.training.data import TRANSFORM_NAMES, apply_transform_np, label_transform_table
from rocalphago_amd.utils.go_util import sgf_iter_states


def test_label_table_matches_plane_transform():
    table = label_transform_table(7)
    for t in range(8):
        for p in (0, 5, 24, 48):
            one = np.zeros((1, 7, 7))
            one[0][divmod(p, 7)] = 1
            assert np.argmax(apply_transform_np(one, t)[0]) == table[t, p], TRANSFORM_NAMES[t]


def test_supervised_one_epoch(ref_data, tmp_path):
    out = str(tmp_path / "sl")
    meta = sl.run_training([os.path.join(ref_data, "minimodel.json"),
                            os.path.join(ref_data, "hdf5", "alphago-vs-lee-sedol-features.hdf5"),
                            out, "--epochs", "1", "--seed", "3"])
    for f in ("metadata.json", "shuffle.npz", "weights.00000.hdf5"):
        assert os.path.exists(os.path.join(out, f))
    m = json.load(open(os.path.join(out, "metadata.json")))
    assert len(m["epochs"]) == 1 and {"loss", "acc", "val_loss", "val_acc"} <= set(m["epochs"][0])
    assert np.load(os.path.join(out, "shuffle.npz")).shape == (1033,)
    # resume appends an epoch
    sl.run_training([os.path.join(ref_data, "minimodel.json"),
                     os.path.join(ref_data, "hdf5", "alphago-vs-lee-sedol-features.hdf5"),
                     out, "--epochs", "1", "--weights", "weights.00000.hdf5"])
    assert len(json.load(open(os.path.join(out, "metadata.json")))["epochs"]) == 2


def test_supervised_rejects_feature_mismatch(ref_data, tmp_path):
    p = CNNPolicy(["board", "ones"], layers=2, filters_per_layer=8, device="cpu")
    mj = str(tmp_path / "m.json")
    p.save_model(mj)
    with pytest.raises(ValueError):
        sl.run_training([mj, os.path.join(ref_data, "hdf5", "alphago-vs-lee-sedol-features.hdf5"),
                         str(tmp_path / "o"), "--epochs", "1"])


def test_game_converter_cli(ref_data, tmp_path):
    out = str(tmp_path / "conv.h5")
    run_game_converter(["--features", "board,ones,turns_since", "--outfile", out,
                        "--directory", os.path.join(ref_data, "sgf")])
    f = h5lite.File(out)
    assert f["states"].shape == (1033, 12, 19, 19)
    assert f["features"][()] == b"board,ones,turns_since"
    assert len(f["file_offsets"].keys()) == 5
    ref = h5lite.File(os.path.join(ref_data, "hdf5", "alphago-vs-lee-sedol-features.hdf5"))
    # same positions, same order within each game
    for key in f["file_offsets"].keys():
        s, n = f["file_offsets"][key][()]
        rkey = [k for k in ref["file_offsets"].keys() if k.endswith(key.split(":")[-1])][0]
        rs, rn = ref["file_offsets"][rkey][()]
        assert n == rn
        assert np.array_equal(f["states"][s:s + n], ref["states"][rs:rs + rn])
    out2 = str(tmp_path / "conv2.h5")
    run_game_converter(["--features", "board,ones,turns_since", "--outfile", out2,
                        "--directory", ref_data, "--recurse"])
    assert len(h5lite.File(out2)["file_offsets"].keys()) >= 6


# ----------------------------------------------------------------------------- RL
class MockPlayer(object):
    def __init__(self, policy, sgf_path):
        with open(sgf_path) as fh:
            self.moves = [m for (_, m, _) in sgf_iter_states(fh.read())]
        self.policy = policy

    def get_moves(self, states):
        return [self.moves[len(s.history)] if len(s.history) < len(self.moves) else PASS_MOVE
                for s in states]


class MockState(GameState):
    def __init__(self, winner, length, *a, **kw):
        super(MockState, self).__init__(*a, **kw)
        self.predetermined_winner = winner
        self.length = length

    def do_move(self, *a, **kw):
        super(MockState, self).do_move(*a, **kw)
        if len(self.history) > self.length:
            self.is_end_of_game = True

    def get_winner(self):
        return self.predetermined_winner


def _games(ref_data):
    d = os.path.join(ref_data, "sgf")
    return [os.path.join(d, f) for f in sorted(os.listdir(d))[:2]]


def _policy(ref_data):
    return CNNPolicy.load_model(os.path.join(ref_data, "minimodel.json"), device="cpu")


def test_rl_gradient_direction_flips_with_result(ref_data):
    for game in _games(ref_data):
        base = _policy(ref_data).model.get_weights()

        def run(winners):
            states = [MockState(w, 2, size=19) for w in winners]
            p1, p2 = _policy(ref_data), _policy(ref_data)
            p1.model.set_weights(base)
            opt = K.SGD(lr=0.001)
            p1.model.compile(loss=rl.log_loss, optimizer=opt)
            rl.run_n_games(opt, MockPlayer(p1, game), MockPlayer(p2, game), 2, mock_states=states)
            return p1.model.get_weights()

        a = run([BLACK, WHITE])
        b = run([WHITE, BLACK])
        assert any(not np.array_equal(i, x) for i, x in zip(base, a))
        for i, x, y in zip(base, a, b):
            npt.assert_allclose(x - i, -(y - i), rtol=1e-3, atol=1e-11)


@pytest.mark.parametrize("winner,sign", [(BLACK, 1), (WHITE, -1)])
def test_rl_win_raises_loss_lowers_move_probs(ref_data, winner, sign):
    game = _games(ref_data)[0]
    p1, p2 = _policy(ref_data), _policy(ref_data)
    opt = K.SGD()
    p1.model.compile(loss=rl.log_loss, optimizer=opt)
    with open(game) as fh:
        txt = fh.read()

    def probs():
        out = []
        for (st, mv, pl) in sgf_iter_states(txt):
            if pl == BLACK:
                d = dict(p1.eval_state(st))
                out.append(d.get(mv, 0))
        return out[:10]

    before = probs()
    rl.run_n_games(opt, MockPlayer(p1, game), MockPlayer(p2, game), 1,
                   mock_states=[MockState(winner, 20, size=19)])
    after = probs()
    assert sign * sum(a - b for a, b in zip(after, before)) > 0


def test_rl_batched_update_matches_direction(ref_data):
    game = _games(ref_data)[0]
    p1, p2 = _policy(ref_data), _policy(ref_data)
    base = p1.model.get_weights()
    opt = K.SGD(lr=0.01)
    p1.model.compile(loss=rl.log_loss, optimizer=opt)
    rl.run_n_games(opt, MockPlayer(p1, game), MockPlayer(p2, game), 1,
                   mock_states=[MockState(BLACK, 20, size=19)], mode="batched")
    assert any(not np.array_equal(i, x) for i, x in zip(base, p1.model.get_weights()))


def test_rl_cli_one_iteration(ref_data, tmp_path):
    out = str(tmp_path / "rl") + "/"
    meta = rl.run_training([os.path.join(ref_data, "minimodel.json"),
                            os.path.join(ref_data, "hdf5", "random_minimodel_weights.hdf5"), out,
                            "--game-batch", "2", "--iterations", "1", "--move-limit", "12"])
    for f in ("metadata.json", "weights.00000.hdf5", "weights.00001.hdf5"):
        assert os.path.exists(os.path.join(out, f))
    m = json.load(open(os.path.join(out, "metadata.json")))
    assert m["opponents"] == ["weights.00000.hdf5"] and "weights.00000.hdf5" in m["win_ratio"]
    rl.run_training([os.path.join(ref_data, "minimodel.json"), "weights.00001.hdf5", out,
                     "--game-batch", "2", "--iterations", "1", "--move-limit", "12",
                     "--resume"])
    assert os.path.exists(os.path.join(out, "weights.00002.hdf5"))


def test_comm_timer_resolves_events_as_it_goes():
    """CommTimer keeps a bounded number of event pairs alive (one pair per step used
    to pile up until the per-epoch pop); host mode counts every start/stop pair."""
    import torch
    from rocalphago_amd.utils.metrics import CommTimer
    t = CommTimer("cpu")
    for _ in range(50):
        t.start()
        t.stop()
    ms, n = t.pop()
    assert n == 50 and ms >= 0.0
    assert t.pop() == (0.0, 0)
    if torch.cuda.is_available():
        g = CommTimer("cuda", ring=8)
        for _ in range(100):
            g.start()
            g.stop()
            assert g.pending() <= 9
        ms, n = g.pop()
        assert n == 100 and g.pending() == 0
