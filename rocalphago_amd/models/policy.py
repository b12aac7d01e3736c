"""Policy networks — reference AlphaGo/models/policy.py (CNNPolicy :9-138, ResnetPolicy :141-271).

CNNPolicy: 'same' conv K1xK1 (default 5x5) + ReLU, (layers-1) x conv 3x3 + ReLU, 1x1 conv to one
plane (linear, scalar bias), Flatten, per-position Bias, softmax over S*S points (no pass logit,
quirk Q17; ``pass_logit=True`` adds one, softmax over S*S + 1 with pass last). On a GPU the
whole network (forward, fused softmax/loss, backward, SGD) runs on the hand-written gfx950
kernels (models/fused.py). Defaults follow the reference (128 filters, 12
layers); the north-star benchmark model is 48 planes / 192 filters / 12+1 layers.
"""
import numpy as np

from ..engine.gamestate import PASS_MOVE
from ..utils.go_util import flatten_idx
from . import kerasish as K
from .nn_util import Bias, NeuralNetBase, neuralnet


@neuralnet
class CNNPolicy(NeuralNetBase):
    """Convolutional policy network: state -> distribution over board points."""

    def _select_moves_and_normalize(self, nn_output, moves, size):
        if len(moves) == 0:
            return []
        if len(nn_output) > size * size:  # pass-logit network: pass is a move like any other
            moves = list(moves) + ([PASS_MOVE] if PASS_MOVE not in moves else [])
        move_indices = [size * size if m is PASS_MOVE else flatten_idx(m, size) for m in moves]
        distribution = nn_output[move_indices]
        distribution = distribution / distribution.sum()
        return list(zip(moves, distribution))

    def batch_eval_state(self, states, moves_lists=None):
        """Evaluate many states in one network call: [eval_state(s) for s in states]."""
        n_states = len(states)
        if n_states == 0:
            return []
        state_size = states[0].size
        if not all([st.size == state_size for st in states]):
            raise ValueError("all states must have the same size")
        nn_input = self.preprocessor.states_to_tensor_u8(states)
        network_output = self.forward(nn_input)
        moves_lists = moves_lists or [st.get_legal_moves() for st in states]
        return [self._select_moves_and_normalize(network_output[i], moves_lists[i], state_size)
                for i in range(n_states)]

    def eval_state(self, state, moves=None):
        """(move, probability) pairs over ``moves`` (default: all legal moves, quirk Q5)."""
        tensor = self.preprocessor.state_to_tensor(state)
        network_output = self.forward(tensor)
        moves = moves or state.get_legal_moves()
        return self._select_moves_and_normalize(network_output[0], moves, state.size)

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
        if layer > params['layers']:
            print("Due to skipping, ended with {} layers instead of {}"
                  .format(layer, params['layers']))
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
