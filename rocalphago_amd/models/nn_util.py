"""NeuralNetBase, the @neuralnet registry and the Bias layer — reference AlphaGo/models/nn_util.py.

``save_model`` writes the reference JSON spec ``{class, keras_model, feature_list[, weights_file]}``
(nn_util.py:85-108) and ``load_model`` reads it back, rebuilding the network from the embedded
Keras-1 JSON through our kerasish interpreter (nn_util.py:60-83).
"""
import json
import os

from ..features.preprocessing import Preprocess
from . import kerasish


class NeuralNetBase(object):
    """Base class: feature preprocessing + a network built by the subclass' create_network."""

    subclasses = {}

    def __init__(self, feature_list, **kwargs):
        self.preprocessor = Preprocess(feature_list)
        kwargs["input_dim"] = self.preprocessor.output_dim
        if kwargs.get('init_network', True):
            self.model = self.__class__.create_network(**kwargs)
            self.forward = self._model_forward()

    def _model_forward(self):
        """np/tensor batch (B, F, S, S) -> network output as numpy (learning phase = test)."""
        model = self.model
        return lambda inpt: model.predict(inpt)

    def forward_device(self, x):
        """Device-resident batch -> device-resident output (no host round trip; used by the GPU
        players and self-play). Learning phase = test, as ``forward``."""
        import torch
        model = self.model
        plan = model._plan_for()
        with torch.no_grad():
            if plan is not None:
                return plan.forward(x)
            return model.net.forward(x.float(), training=False)

    @staticmethod
    def load_model(json_file, device=None):
        """Rebuild a network from its JSON spec (class name, Keras-1 model JSON,
        feature list, optional weights file); reference contract
        /root/reference/AlphaGo/models/nn_util.py:60-83."""
        with open(json_file, 'r') as f:
            spec = json.load(f)
        name = spec.get('class', 'CNNPolicy')
        cls = NeuralNetBase.subclasses.get(name)
        if cls is None:
            known = ", ".join(sorted(NeuralNetBase.subclasses))
            raise ValueError("%s names network class %r, which is not registered (known: %s); "
                             "decorate the class with @neuralnet" % (json_file, name, known))
        net = cls(spec['feature_list'], init_network=False)
        net.model = kerasish.model_from_json(spec['keras_model'], custom_objects={'Bias': Bias},
                                             device=device)
        weights = spec.get('weights_file')
        if weights:
            net.model.load_weights(_resolve(weights, json_file))
        net.forward = net._model_forward()
        return net

    def set_dtype(self, dtype):
        """GPU compute precision: ``"bf16"`` (fused HIP kernels, default) or ``"fp32"``
        (reference precision through the generic executor)."""
        self.model.set_precision(dtype)
        return self

    def save_model(self, json_file, weights_file=None):
        """Write the JSON spec (and the weights, when a file is given) that load_model reads."""
        spec = {'class': type(self).__name__, 'keras_model': self.model.to_json(),
                'feature_list': self.preprocessor.feature_list}
        if weights_file is not None:
            self.model.save_weights(weights_file)
            spec['weights_file'] = weights_file
        with open(json_file, 'w') as f:
            json.dump(spec, f)


def _resolve(path, json_file):
    """Weights paths in specs are relative to the working directory (reference behaviour); if
    that fails, also try relative to the JSON file and its parent directories."""
    if os.path.isabs(path) or os.path.exists(path):
        return path
    d = os.path.dirname(os.path.abspath(json_file))
    while True:
        cand = os.path.join(d, path)
        if os.path.exists(cand):
            return cand
        parent = os.path.dirname(d)
        if parent == d:
            return path
        d = parent


def neuralnet(cls):
    """Class decorator registering NeuralNetBase subclasses for load_model."""
    NeuralNetBase.subclasses[cls.__name__] = cls
    return cls


class Bias(object):
    """Per-position trainable bias added after Flatten (reference nn_util.py:118-133).

    Calling ``Bias()`` yields the kerasish layer description; its single weight ``param_0`` has
    the input's shape minus the batch axis and is initialised to zeros. On the HIP path it is
    fused into the policy-head kernel."""

    def __new__(cls, **kwargs):
        return kerasish.BiasLayer(name=kwargs.get("name"))
