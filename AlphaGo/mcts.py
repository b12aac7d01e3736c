"""AlphaGo.mcts — reference-semantics MCTS + the native APV-MCTS (ParallelMCTS)."""
from rocalphago_amd.search.mcts import MCTS, TreeNode  # noqa: F401
try:
    from rocalphago_amd.search.apv import ParallelMCTS  # noqa: F401
except ImportError:  # pragma: no cover
    pass
