"""GPU ladder reading (csrc/hip/ladder.hip) == the native is_ladder_capture / is_ladder_escape
(csrc/engine/go_engine.cpp, pinned to the reference scenarios by tests/test_ladders.py), for
every point of every position."""
import numpy as np
import pytest
import torch

from rocalphago_amd._native import engine

from boards import ladder_scenarios, random_games

pytestmark = pytest.mark.gpu
rg = engine()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


_games = random_games


def _compare(dev, states):
    from rocalphago_amd.ops.features import gpu_ladders
    boards = [s.native for s in states]
    S = boards[0].size
    colors, _, meta, _, want = rg.gpu_feature_inputs(boards, True, 8)
    c = torch.from_numpy(colors).to(dev)
    m = torch.from_numpy(meta).to(dev)
    got, work = gpu_ladders(c, m, S)
    got = got.cpu().numpy()
    overflow = int(work[8:12].view(torch.int32).item())
    assert overflow == 0
    if not np.array_equal(got, want):
        bad = np.argwhere(got != want)
        b, k, p = bad[0]
        raise AssertionError("state %d %s at %s: gpu %d native %d (%d mismatches)" % (
            b, ("capture", "escape")[k], divmod(int(p), S), got[b, k, p], want[b, k, p],
            len(bad)))
    return int(want.sum())


@pytest.mark.parametrize("size,seed,lo,hi", [(19, 11, 40, 250), (19, 12, 150, 400),
                                             (13, 13, 20, 200), (9, 14, 10, 120)])
def test_gpu_ladders_match_native(dev, size, seed, lo, hi):
    states = _games(192, size, seed, lo, hi)
    n = _compare(dev, states)
    assert n > 0, "no ladder in the sample: the comparison would be vacuous"


_reference_scenarios = ladder_scenarios


def test_gpu_ladders_reference_scenarios(dev):
    states = _reference_scenarios()
    assert _compare(dev, states) > 0


def test_gpu_features_use_gpu_ladders(dev):
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES, Preprocess
    from rocalphago_amd.ops.features import GpuFeatures
    states = _games(64, 19, 21, 60, 300)
    gf = GpuFeatures(DEFAULT_FEATURES, dev, ladders="gpu")
    got = gf([s.native for s in states]).cpu().numpy()
    want = rg.batch_features([s.native for s in states], Preprocess(DEFAULT_FEATURES).feature_ids,
                             4)
    assert np.array_equal(got, want)
