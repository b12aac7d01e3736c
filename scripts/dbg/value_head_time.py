"""Time the value-MLP training head: HIP (ops.value_mlp_train) vs the torch autograd tail."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rocalphago_amd.ops import hipops as ops  # noqa: E402


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    dev = torch.device("cuda")
    B, P, H = 256, 361, 256
    z = torch.randn(B, P, device=dev)
    W1 = torch.randn(P, H, device=dev) * 0.05
    b1 = torch.randn(H, device=dev) * 0.1
    W2 = torch.randn(H, 1, device=dev) * 0.1
    b2 = torch.randn(1, device=dev) * 0.1
    y = torch.rand(B, device=dev) * 2 - 1
    g = [torch.empty_like(t) for t in (W1, b1, W2, b2)]
    dz = torch.empty(B, P, device=dev)

    def hip():
        ops.value_mlp_train(z, W1, b1, W2, b2, y, None, "relu", *g, dz=dz)

    def torch_tail():
        ps = [t.detach().requires_grad_() for t in (z, W1, b1, W2, b2)]
        v = torch.tanh(torch.relu(ps[0] @ ps[1] + ps[2]) @ ps[3] + ps[4]).reshape(-1)
        loss = ((v - y) ** 2).mean()
        torch.autograd.grad(loss, ps)

    print(json.dumps({"B": B, "P": P, "H": H, "hip_us": round(timeit(hip), 2),
                      "torch_autograd_us": round(timeit(torch_tail), 2)}))


if __name__ == "__main__":
    main()
