"""AlphaGo.models.nn_util — see rocalphago_amd/models/nn_util.py."""
from rocalphago_amd.models.nn_util import Bias, NeuralNetBase, neuralnet  # noqa: F401
