"""GPU rollout kernel throughput (games/s, moves/s) on 19x19 from the empty board."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from rocalphago_amd._native import engine
from rocalphago_amd.engine.gamestate import GameState
from rocalphago_amd.search.gpu_rollout import GpuRollouts


def run(games, R, no_pattern=False):
    rg = engine()
    g = GpuRollouts(rg.RolloutPolicy(), torch.device("cuda"), slice_moves=0)  # alone on the GPU
    if no_pattern:
        g.pattern = None
    st = [GameState() for _ in range(games // R)]
    g.run(st, R=R, limit=1000, seed=1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    w, ln = g.run(st, R=R, limit=1000, seed=2)
    dt = time.perf_counter() - t
    return {"games": games, "R": R, "no_pattern": no_pattern, "ms": round(dt * 1e3, 2),
            "games_per_s": round(games / dt), "moves_per_s": round(float(ln.sum()) / dt),
            "mean_len": round(float(ln.mean()), 1)}


if __name__ == "__main__":
    for games, R in [(1024, 4), (4096, 4), (16384, 16)]:
        print(json.dumps(run(games, R)))
    print(json.dumps(run(1024, 4, no_pattern=True)))
