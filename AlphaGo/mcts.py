"""AlphaGo.mcts — reference-semantics MCTS (TreeNode, MCTS) and the native APV-MCTS
(ParallelMCTS, the reference's empty stub at AlphaGo/mcts.py:219-220, implemented)."""
from rocalphago_amd.search.apv import ParallelMCTS, ParallelMCTSPlayer  # noqa: F401
from rocalphago_amd.search.mcts import MCTS, TreeNode  # noqa: F401
