"""AlphaGo.preprocessing.preprocessing — feature planes. See rocalphago_amd/features."""
from rocalphago_amd.features.preprocessing import *  # noqa: F401,F403
from rocalphago_amd.features.preprocessing import (DEFAULT_FEATURES, FEATURES,  # noqa: F401
                                                   VALUE_FEATURES, Preprocess)
