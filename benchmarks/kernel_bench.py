"""Per-kernel timing of the HIP conv/head kernels vs torch (MIOpen) at the north-star shape.

Reports us/call and TFLOP/s for a 3x3 192->192 conv on B x 19 x 19 boards (fwd, dgrad, wgrad),
the 5x5 48->192 input layer, and the fused policy head. One JSON line per kernel.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from rocalphago_amd.ops import hipops as ops


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--torch", action="store_true", help="also time torch/MIOpen")
    args = ap.parse_args()
    dev = torch.device("cuda")
    B, S = args.batch, 19
    res = []
    for (cin, cout, ks) in [(192, 192, 3), (48, 192, 5), (128, 128, 3)]:
        cinp, coutp = ops.pad_channels(cin), ops.pad_channels(cout)
        hi = ks // 2
        flops = 2.0 * B * S * S * cin * cout * ks * ks
        x = torch.randn(B, cin, S, S, device=dev).relu()
        w = torch.randn(cout, cin, ks, ks, device=dev) * 0.05
        xp = ops.pack_nchw(x, hi, cinp)
        wf, wb = ops.pack_weights(w, coutp, cinp, wb=torch.empty(ks * ks, cinp, coutp,
                                                                  dtype=torch.bfloat16, device=dev))
        bias = torch.zeros(coutp, device=dev)
        y = ops.alloc_padded(B, S, 1, coutp, dev)
        t = timeit(lambda: ops.conv_igemm(xp, wf, bias, y, B, S, hi, 1, cinp, coutp, ks, True))
        res.append(("fwd", cin, cout, ks, t, flops / t / 1e6))
        g = ops.pack_nchw(torch.randn(B, cout, S, S, device=dev), hi, coutp)
        if ks == 3:
            dx = ops.alloc_padded(B, S, 1, cinp, dev)
            t = timeit(lambda: ops.conv_igemm(g, wb, None, dx, B, S, 1, 1, coutp, cinp, ks, False,
                                              mask=xp))
            res.append(("dgrad", cin, cout, ks, t, flops / t / 1e6))
        dw = torch.zeros(cout, cin, ks, ks, device=dev)
        db = torch.zeros(cout, device=dev)
        work = ops.wgrad_workspace(B, S, coutp, cinp, ks, dev)
        t = timeit(lambda: ops.conv_wgrad(g, xp, dw, db, B, S, hi, cout, coutp, cin, cinp, ks,
                                          work=work))
        res.append(("wgrad", cin, cout, ks, t, flops / t / 1e6))
        if args.torch:
            xt = x.to(torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
            wt = w.to(torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
            t = timeit(lambda: F.conv2d(xt, wt, padding=ks // 2))
            res.append(("torch_fwd", cin, cout, ks, t, flops / t / 1e6))
            yt = F.conv2d(xt, wt, padding=ks // 2)
            gt = torch.randn_like(yt)
            t = timeit(lambda: torch.autograd.grad(yt, (xt, wt), gt, retain_graph=True))
            res.append(("torch_bwd(d+w)", cin, cout, ks, t, 2 * flops / t / 1e6))
    K = 192
    h = ops.pack_nchw(torch.randn(B, K, S, S, device=dev).relu(), 1, K)
    wv = torch.randn(K, device=dev)
    b0 = torch.zeros(1, device=dev)
    pb = torch.zeros(S * S, device=dev)
    probs = torch.empty(B, S * S, device=dev)
    lab = torch.randint(0, S * S, (B,), device=dev)
    loss = torch.empty(B, device=dev)
    dz = torch.empty(B, S * S, device=dev)
    t = timeit(lambda: ops.policy_head_fwd(h, wv, b0, pb, probs, K, labels=lab, loss=loss, dz=dz,
                                           mode=1, gscale=1.0 / B))
    res.append(("policy_head_fwd", K, 1, 1, t, 0.0))
    dh = ops.alloc_padded(B, S, 1, K, dev)
    dwv = torch.zeros(K, device=dev)
    t = timeit(lambda: ops.head_bwd(h, wv, dz, dh, dwv, b0, pb, K))
    res.append(("head_bwd", K, 1, 1, t, 0.0))
    for name, cin, cout, ks, t, tf in res:
        print(json.dumps({"kernel": name, "cin": cin, "cout": cout, "ks": ks, "batch": B,
                          "us": round(t, 2), "tflops": round(tf, 1)}))


if __name__ == "__main__":
    main()
