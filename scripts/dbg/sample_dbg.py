import sys; sys.path.insert(0, ".")
import numpy as np, torch
from rocalphago_amd.ops import hipops as ops
P = 361
probs = torch.zeros(3, P, device="cuda")
mask = torch.zeros(3, P, dtype=torch.uint8, device="cuda")
for r in range(3):
    mask[r, [58, 122, 250, 300]] = 1
probs[:, 250] = 0.9
probs[:, 58] = 0.05
probs[1, 300] = 0.95
g = torch.ones(3, dtype=torch.uint8, device="cuda")
print("greedy", ops.sample_moves(probs, mask, 1.0, g, seed=1).cpu().numpy())
print("beta1000", ops.sample_moves(probs, mask, 1000.0, None, seed=1).cpu().numpy())
g[2] = 0
print("mixed", ops.sample_moves(probs, mask, 1000.0, g, seed=1).cpu().numpy())
