"""Eager PyTorch (MIOpen) reference for the SL policy training step — the bar the HIP kernels beat.

Same architecture as the north-star policy (48 planes, 5x5 + 11x 3x3 convs at 192 filters, 1x1
head, per-position bias, softmax), bf16 autocast, channels_last, SGD. Prints one JSON line.
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Net(nn.Module):
    def __init__(self, planes=48, k=192, layers=12, board=19):
        super().__init__()
        convs = [nn.Conv2d(planes, k, 5, padding=2)]
        for _ in range(layers - 1):
            convs.append(nn.Conv2d(k, k, 3, padding=1))
        self.convs = nn.ModuleList(convs)
        self.head = nn.Conv2d(k, 1, 1)
        self.bias = nn.Parameter(torch.zeros(board * board))

    def forward(self, x):
        for c in self.convs:
            x = F.relu(c(x))
        return self.head(x).flatten(1) + self.bias


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--fp32", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda")
    net = Net().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(net.parameters(), lr=0.01)
    x = (torch.rand(args.batch, 48, 19, 19, device=dev) > 0.5).float().to(
        memory_format=torch.channels_last)
    y = torch.randint(0, 361, (args.batch,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=not args.fp32):
            loss = F.cross_entropy(net(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    print(json.dumps({"what": "torch_eager_policy_train", "batch": args.batch,
                      "ms_per_step": dt * 1e3, "positions_per_s": args.batch / dt,
                      "dtype": "fp32" if args.fp32 else "bf16-autocast"}))


if __name__ == "__main__":
    main()
