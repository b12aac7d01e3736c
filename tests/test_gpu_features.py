"""GPU feature kernel (csrc/hip/features.hip) == native extractor, plane for plane."""
import numpy as np
import pytest
import torch

from rocalphago_amd._native import engine
from rocalphago_amd.engine.gamestate import GameState
from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES, Preprocess

pytestmark = pytest.mark.gpu
rg = engine()


def _positions(n, size, seed, superko=False):
    rs = np.random.RandomState(seed)
    rp = rg.RolloutPolicy()
    out = []
    for i in range(n):
        st = GameState(size=size, enforce_superko=superko)
        target = int(rs.randint(0, int(size * size * 1.6)))
        for k in range(target):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            st.do_move(None if mv < 0 else divmod(mv, size))
            if st.is_end_of_game:
                break
        out.append(st)
    return out


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


@pytest.mark.parametrize("ladders", ["host", "gpu"])
@pytest.mark.parametrize("size,seed", [(19, 1), (19, 2), (9, 3), (13, 4), (7, 5)])
def test_gpu_features_match_native(dev, size, seed, ladders):
    from rocalphago_amd.ops.features import GpuFeatures
    feats = DEFAULT_FEATURES + ["color", "legal"]
    states = _positions(48, size, seed)
    gf = GpuFeatures(feats, dev, ladders=ladders)
    got = gf([s.native for s in states]).cpu().numpy()
    want = rg.batch_features([s.native for s in states], Preprocess(feats).feature_ids, 4)
    assert got.shape == want.shape
    if not np.array_equal(got, want):
        bad = np.argwhere(got != want)
        b, f, x, y = bad[0]
        raise AssertionError("first mismatch state %d plane %d at (%d,%d): gpu %d native %d "
                             "(%d mismatches)" % (b, f, x, y, got[b, f, x, y], want[b, f, x, y],
                                                  len(bad)))


def test_gpu_features_superko_and_subsets(dev):
    from rocalphago_amd.ops.features import GpuFeatures
    states = _positions(24, 9, 7, superko=True)
    for feats in (["legal", "sensibleness"], ["liberties_after", "board", "zeros"],
                  ["ladder_escape", "capture_size", "ones"]):
        gf = GpuFeatures(feats, dev, ladders="gpu")  # superko boards: native ladders anyway
        got = gf([s.native for s in states]).cpu().numpy()
        want = rg.batch_features([s.native for s in states], Preprocess(feats).feature_ids, 4)
        assert np.array_equal(got, want), feats


def test_gpu_sensibleness_late_game(dev):
    """The true-eye DFS (pruned frames: a frame fails once its bad diagonals exceed the allowance
    and succeeds once its remaining eyeish diagonals cannot) on late-game 19x19 positions, where
    large eyeish regions make the recursion deep: the same planes as the native extractor."""
    from rocalphago_amd.ops.features import GpuFeatures
    rs = np.random.RandomState(11)
    rp = rg.RolloutPolicy()
    states = []
    for _ in range(96):
        st = GameState()
        for _ in range(int(rs.randint(250, 450))):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            st.do_move(None if mv < 0 else divmod(mv, 19))
            if st.is_end_of_game:
                break
        states.append(st)
    feats = ["sensibleness", "legal", "board"]
    gf = GpuFeatures(feats, dev, ladders="host")
    got = gf([s.native for s in states]).cpu().numpy()
    want = rg.batch_features([s.native for s in states], Preprocess(feats).feature_ids, 4)
    assert np.array_equal(got, want), int((got != want).sum())
