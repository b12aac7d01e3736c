"""Feature planes — reference AlphaGo/preprocessing/preprocessing.py:1-294.

Every plane is computed by the native engine (csrc/engine/features.cpp) in one pass per state;
``Preprocess.states_to_tensor`` extracts a whole batch with native threads (the GPU-resident
feature kernel for search lives in rocalphago_amd/ops/features.py).

The reference registry (preprocessing.py:209-258, 12 entries, DEFAULT_FEATURES = 48 planes) is
extended with ``color`` (1 plane: player to move is black), which the reference's value network
expects as its 49th input plane (value.py:16) but never defines.
"""
import numpy as np

from .._native import engine as _engine

_rg = _engine()

_FID = {
    "board": 0, "ones": 1, "turns_since": 2, "liberties": 3, "capture_size": 4,
    "self_atari_size": 5, "liberties_after": 6, "ladder_capture": 7, "ladder_escape": 8,
    "sensibleness": 9, "zeros": 10, "legal": 11, "color": 12,
}


def _planes(name):
    def fn(state, _fid=_FID[name]):
        return _rg.Board.features(state.native, [_fid]).astype(np.float64)
    fn.__name__ = "get_" + name
    return fn


get_board = _planes("board")
get_turns_since = _planes("turns_since")
get_liberties = _planes("liberties")
get_capture_size = _planes("capture_size")
get_self_atari_size = _planes("self_atari_size")
get_liberties_after = _planes("liberties_after")
get_ladder_capture = _planes("ladder_capture")
get_ladder_escape = _planes("ladder_escape")
get_sensibleness = _planes("sensibleness")
get_legal = _planes("legal")
get_color = _planes("color")

FEATURES = {
    "board": {"size": 3, "function": get_board},
    "ones": {"size": 1, "function": _planes("ones")},
    "turns_since": {"size": 8, "function": get_turns_since},
    "liberties": {"size": 8, "function": get_liberties},
    "capture_size": {"size": 8, "function": get_capture_size},
    "self_atari_size": {"size": 8, "function": get_self_atari_size},
    "liberties_after": {"size": 8, "function": get_liberties_after},
    "ladder_capture": {"size": 1, "function": get_ladder_capture},
    "ladder_escape": {"size": 1, "function": get_ladder_escape},
    "sensibleness": {"size": 1, "function": get_sensibleness},
    "zeros": {"size": 1, "function": _planes("zeros")},
    "legal": {"size": 1, "function": get_legal},
    "color": {"size": 1, "function": get_color},
}

DEFAULT_FEATURES = [
    "board", "ones", "turns_since", "liberties", "capture_size",
    "self_atari_size", "liberties_after", "ladder_capture", "ladder_escape",
    "sensibleness", "zeros"]

# value network input = policy features + color (49 planes)
VALUE_FEATURES = DEFAULT_FEATURES + ["color"]


class Preprocess(object):
    """Convert GameStates to one-hot feature tensors (reference preprocessing.py:266-294)."""

    def __init__(self, feature_list=DEFAULT_FEATURES):
        self.output_dim = 0
        self.feature_list = feature_list
        self.processors = [None] * len(feature_list)
        self._fids = []
        for i in range(len(feature_list)):
            feat = feature_list[i].lower()
            if feat in FEATURES:
                self.processors[i] = FEATURES[feat]["function"]
                self.output_dim += FEATURES[feat]["size"]
                self._fids.append(_FID[feat])
            else:
                raise ValueError("uknown feature: %s" % feat)

    @property
    def feature_ids(self):
        return list(self._fids)

    def state_to_tensor(self, state):
        """(1, F, S, S) float32 tensor of the requested planes, in feature_list order."""
        planes = state.native.features(self._fids)
        f, s = self.output_dim, state.size
        return planes.reshape((1, f, s, s)).astype(np.float32)

    def states_to_tensor_u8(self, states, nthreads=8):
        """(B, F, S, S) uint8 for a list of states, extracted by native threads."""
        return _rg.batch_features([st.native for st in states], self._fids, nthreads)

    def states_to_tensor(self, states, nthreads=8):
        return self.states_to_tensor_u8(states, nthreads).astype(np.float32)
