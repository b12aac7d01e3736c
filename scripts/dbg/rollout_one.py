"""One GPU rollout launch of N games from the empty 19x19 board (for PMC passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rocalphago_amd._native import engine  # noqa: E402
from rocalphago_amd.engine.gamestate import GameState  # noqa: E402
from rocalphago_amd.search.gpu_rollout import GpuRollouts  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
g = GpuRollouts(engine().RolloutPolicy(), torch.device("cuda"))
st = [GameState() for _ in range(n // 4)]
w, ln = g.run(st, R=4, limit=1000, seed=3)
torch.cuda.synchronize()
print("games", n, "moves", int(ln.sum()))
