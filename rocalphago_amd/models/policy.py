"""Policy networks — reference AlphaGo/models/policy.py (CNNPolicy :9-138, ResnetPolicy :141-271).

CNNPolicy: 'same' conv K1xK1 (default 5x5) + ReLU, (layers-1) x conv 3x3 + ReLU, 1x1 conv to one
plane (linear, scalar bias), Flatten, per-position Bias, softmax over S*S points (no pass logit,
quirk Q17; ``pass_logit=True`` adds one, softmax over S*S + 1 with pass last). On a GPU the
whole network (forward, fused softmax/loss, backward, SGD) runs on the hand-written gfx950
kernels (models/fused.py). Defaults follow the reference (128 filters, 12
layers); the north-star benchmark model is 48 planes / 192 filters / 12+1 layers.
"""
import warnings

import numpy as np

from ..engine.gamestate import PASS_MOVE
from ..utils.go_util import flatten_idx
from . import kerasish as K
from .nn_util import Bias, NeuralNetBase, neuralnet


@neuralnet
class CNNPolicy(NeuralNetBase):
    """Convolutional policy network: state -> distribution over board points."""

    def batch_eval_state(self, states, moves_lists=None):
        """``[eval_state(s) for s in states]`` through one forward pass (reference
        policy.py:27-48): every state must have the same board size."""
        if not states:
            return []
        sizes = {st.size for st in states}
        if len(sizes) > 1:
            raise ValueError("batch_eval_state: mixed board sizes %s" % sorted(sizes))
        probs = self.forward(self.preprocessor.states_to_tensor_u8(states))
        if moves_lists is None:
            moves_lists = [st.get_legal_moves() for st in states]
        return [_move_distribution(p, mv, st.size)
                for p, mv, st in zip(probs, moves_lists, states)]

    def eval_state(self, state, moves=None):
        """(move, probability) pairs over ``moves`` (default: all legal moves, quirk Q5),
        renormalised over those moves (reference policy.py:50-64)."""
        probs = self.forward(self.preprocessor.state_to_tensor(state))[0]
        return _move_distribution(probs, moves or state.get_legal_moves(), state.size)

    @staticmethod
    def create_network(**kwargs):
        """Keyword args (reference policy.py:66-80): input_dim, board (19), filters_per_layer
        (128), filters_per_layer_K, layers (12), filter_width_K (3; 5 for K=1). Extra: seed,
        pass_logit (False): a learned pass logit, softmax over S*S + 1."""
        defaults = {
            "board": 19,
            "filters_per_layer": 128,
            "layers": 12,
            "filter_width_1": 5
        }
        params = defaults
        params.update(kwargs)
        layers = [K.Convolution2D(
            input_shape=(params["input_dim"], params["board"], params["board"]),
            nb_filter=params.get("filters_per_layer_1", params["filters_per_layer"]),
            nb_row=params["filter_width_1"], nb_col=params["filter_width_1"],
            init='uniform', activation='relu', border_mode='same')]
        for i in range(2, params["layers"] + 1):
            fw = params.get("filter_width_%d" % i, 3)
            nf = params.get("filters_per_layer_%d" % i, params["filters_per_layer"])
            layers.append(K.Convolution2D(nb_filter=nf, nb_row=fw, nb_col=fw, init='uniform',
                                          activation='relu', border_mode='same'))
        layers.append(K.Convolution2D(nb_filter=1, nb_row=1, nb_col=1, init='uniform',
                                      border_mode='same'))
        layers.append(K.Flatten())
        layers.append(Bias())
        if params.get("pass_logit"):
            layers.append(K.PassLogit())
        layers.append(K.Activation('softmax'))
        return K.Sequential(layers, device=params.get("device"), seed=params.get("seed"))


@neuralnet
class ResnetPolicy(CNNPolicy):
    """Residual policy (He et al. 2015) exactly as reference policy.py:141-271: linear input conv,
    units of n_skip_K x (BatchNorm -> ReLU -> conv) with sum-merge, final ReLU, 1x1 conv, Flatten,
    Bias, softmax. Note the reference's BatchNormalization uses Keras' default axis=-1 on 'th'
    tensors; that axis is kept for checkpoint compatibility. ``pass_logit=True`` adds the learned
    pass logit of CNNPolicy (softmax over S*S + 1, pass last)."""

    @staticmethod
    def create_network(**kwargs):
        defaults = {
            "board": 19,
            "filters_per_layer": 128,
            "layers": 20,
            "filter_width_1": 5
        }
        params = defaults
        params.update(kwargs)
        layers = []

        def add(layer, inbound):
            layer.inbound = list(inbound)
            layers.append(layer)
            return layer.name

        inp = K.Layer("InputLayer", {"name": K._auto_name("input"), "batch_input_shape":
                                     [None, params["input_dim"], params["board"],
                                      params["board"]], "input_dtype": "float32",
                                     "sparse": False})
        layers.append(inp)
        path = add(K.Convolution2D(nb_filter=params["filters_per_layer"],
                                   nb_row=params["filter_width_1"],
                                   nb_col=params["filter_width_1"], init='uniform',
                                   activation='linear', border_mode='same'), [inp.name])

        def add_resnet_unit(path, Kidx):
            block_input = path
            n_skip = params.get("n_skip_%d" % Kidx, 1)
            for i in range(n_skip):
                layer = Kidx + i
                path = add(K.BatchNormalization(), [path])
                path = add(K.Activation('relu'), [path])
                fw = params.get("filter_width_%d" % layer, 3)
                path = add(K.Convolution2D(nb_filter=params["filters_per_layer"], nb_row=fw,
                                           nb_col=fw, init='uniform', activation='linear',
                                           border_mode='same'), [path])
            path = add(K.Layer("Merge", {"name": K._auto_name("merge"), "mode": "sum",
                                         "concat_axis": -1, "dot_axes": -1,
                                         "output_shape": None, "output_shape_type": "raw",
                                         "output_mask": None, "arguments": {}}),
                       [block_input, path])
            return path, Kidx + n_skip

        layer = 1
        while layer < params['layers']:
            path, layer = add_resnet_unit(path, layer)
        if layer > params['layers']:  # an n_skip_K ran past the requested depth
            warnings.warn("ResnetPolicy: n_skip settings give %d layers (%d requested)"
                          % (layer, params['layers']))
        path = add(K.Activation('relu'), [path])
        path = add(K.Convolution2D(nb_filter=1, nb_row=1, nb_col=1, init='uniform',
                                   border_mode='same'), [path])
        path = add(K.Flatten(), [path])
        path = add(Bias(), [path])
        if params.get("pass_logit"):
            path = add(K.PassLogit(), [path])
        out = add(K.Activation('softmax'), [path])
        return K.Model(layers, functional=True, inputs=[inp.name], outputs=[out],
                       device=params.get("device"), seed=params.get("seed"))


def has_pass_logit(policy):
    """True for a policy network built with ``pass_logit=True`` (output S*S + 1, pass last)."""
    model = getattr(policy, "model", None)
    return model is not None and any(getattr(ld, "class_name", None) == "PassLogit"
                                     for ld in getattr(model, "layers", []))


def policy_probabilities(policy, states):
    """(B, S*S) probabilities for a list of states (fast path for players / search)."""
    x = policy.preprocessor.states_to_tensor_u8(states)
    return np.asarray(policy.forward(x))


def _move_distribution(probs, moves, size):
    """The network's probabilities of ``moves`` (PASS_MOVE maps to the pass logit of a
    pass-logit network, which also always offers it), renormalised to sum to one."""
    if not moves:
        return []
    moves = list(moves)
    pass_slot = len(probs) > size * size
    if pass_slot and PASS_MOVE not in moves:
        moves.append(PASS_MOVE)
    idx = np.fromiter((size * size if m is PASS_MOVE else flatten_idx(m, size) for m in moves),
                      dtype=np.int64, count=len(moves))
    sel = np.asarray(probs)[idx]
    return list(zip(moves, sel / sel.sum()))
