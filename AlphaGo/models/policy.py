"""AlphaGo.models.policy — see rocalphago_amd/models/policy.py."""
from rocalphago_amd.models.policy import CNNPolicy, ResnetPolicy  # noqa: F401
