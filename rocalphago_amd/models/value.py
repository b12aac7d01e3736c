"""Value network — the reference only has a skeleton (AlphaGo/models/value.py:1-44: an
unregistered ``value_trainer`` with TODO get_samples/train).

``CNNValue`` is a registered NeuralNetBase: policy-style conv trunk (default 49 planes = the 48
policy planes + ``color``), a 1x1 conv to one plane, Flatten, Dense(256, ReLU as in the AlphaGo
paper — the reference's linear Dense is available as ``dense_activation='linear'``) and
Dense(1, tanh). Trained with MSE on game outcomes (training/value_trainer.py). On a GPU the conv
trunk and the 1x1 head run on the HIP engine; the two small dense layers are library GEMMs.

``value_trainer`` keeps the reference's class (K=152, LR 0.003, decay 8.66e-8 from the paper)
with working ``get_samples``/``train``.
"""
import numpy as np

from ..features.preprocessing import VALUE_FEATURES
from . import kerasish as KS
from .nn_util import NeuralNetBase, neuralnet

# Parameters obtained from the paper (reference value.py:7-9)
K = 152
LEARNING_RATE = .003
DECAY = 8.664339379294006e-08


@neuralnet
class CNNValue(NeuralNetBase):
    """Convolutional value network: state -> expected outcome in [-1, 1] for the player to move."""

    def __init__(self, feature_list=VALUE_FEATURES, **kwargs):
        super(CNNValue, self).__init__(feature_list, **kwargs)

    def batch_eval_state(self, states):
        if len(states) == 0:
            return np.zeros((0,), np.float32)
        x = self.preprocessor.states_to_tensor_u8(states)
        return np.asarray(self.forward(x)).reshape(-1)

    def eval_state(self, state):
        return float(self.forward(self.preprocessor.state_to_tensor(state)).reshape(-1)[0])

    @staticmethod
    def create_network(**kwargs):
        defaults = {"board": 19, "filters_per_layer": 128, "layers": 12, "filter_width_1": 5,
                    "dense": 256, "dense_activation": "relu"}
        params = defaults
        params.update(kwargs)
        layers = [KS.Convolution2D(
            input_shape=(params["input_dim"], params["board"], params["board"]),
            nb_filter=params.get("filters_per_layer_1", params["filters_per_layer"]),
            nb_row=params["filter_width_1"], nb_col=params["filter_width_1"], init='uniform',
            activation='relu', border_mode='same')]
        for i in range(2, params["layers"] + 1):
            fw = params.get("filter_width_%d" % i, 3)
            nf = params.get("filters_per_layer_%d" % i, params["filters_per_layer"])
            layers.append(KS.Convolution2D(nb_filter=nf, nb_row=fw, nb_col=fw, init='uniform',
                                           activation='relu', border_mode='same'))
        layers.append(KS.Convolution2D(nb_filter=1, nb_row=1, nb_col=1, init='uniform',
                                       activation='linear', border_mode='same'))
        layers.append(KS.Flatten())
        layers.append(KS.Dense(params["dense"], init='uniform',
                               activation=params["dense_activation"]))
        layers.append(KS.Dense(1, init='uniform', activation='tanh'))
        return KS.Sequential(layers, device=params.get("device"), seed=params.get("seed"))


class value_trainer(object):
    """Reference-compatible trainer object (value.py:16-43) around a K=152 CNNValue."""

    def __init__(self, feature_list=VALUE_FEATURES, **kwargs):
        kw = dict(filters_per_layer=K, layers=12, dense_activation="linear")
        kw.update(kwargs)
        self.network = CNNValue(feature_list, **kw)
        self.model = self.network.model
        self.model.compile(loss='mean_squared_error',
                           optimizer=KS.SGD(lr=LEARNING_RATE, decay=DECAY))

    def get_samples(self, states, winners):
        """(X, y): features of the given positions and z = +1/-1 from the mover's view."""
        X = self.network.preprocessor.states_to_tensor_u8(states)
        y = np.array([[1.0 if w == st.current_player else (-1.0 if w != 0 else 0.0)]
                      for st, w in zip(states, winners)], dtype=np.float32)
        return X, y

    def train(self, X, y, batch_size=32, epochs=1):
        n = len(X)
        losses = []
        for _ in range(epochs):
            perm = np.random.permutation(n)
            for i in range(0, n - batch_size + 1, batch_size):
                idx = perm[i:i + batch_size]
                losses.append(self.model.train_on_batch(X[idx], y[idx]))
        return float(np.mean(losses)) if losses else None
