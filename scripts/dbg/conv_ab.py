"""A/B of the forward/dgrad conv kernels in one process, interleaved rounds (guide rule 24):
variant 0 = conv_pipe tap-major, 1 = conv_pipe channel-chunk-major, 2 = conv_tap (tap-shared
slab, 3x3 only), 3 / 4 = 8-wave 384-pixel conv_tap8 with a 4- / 5-deep weight ring, 6 / 7 = ping-pong
conv_tap_pp with a 4- / 3-deep ring, 8 = conv_tap_pp with a 5-deep ring (variant v selects
rag_conv_tap_mode(v - 1)), 99 = conv_tap with the register epilogue instead of the LDS-staged one. 3x3 192->192 fwd and dgrad and 5x5 48->192 fwd at B=256, plus an output check
of every variant against an fp32 torch reference."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from rocalphago_amd.ops import hipops as ops  # noqa: E402
from rocalphago_amd.ops.hipops import _lib  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


dev = torch.device("cuda")
B, S = int(os.environ.get("B", 256)), 19
cases = {}
for (cin, cout, ks) in [(192, 192, 3), (48, 192, 5)]:
    cinp, coutp = ops.pad_channels(cin), ops.pad_channels(cout)
    hi = ks // 2
    x = torch.randn(B, cin, S, S, device=dev).relu()
    w = torch.randn(cout, cin, ks, ks, device=dev) * 0.05
    xp = ops.pack_nchw(x, hi, cinp)
    wf, wb = ops.pack_weights(w, coutp, cinp, wb=torch.empty(ks * ks, cinp, coutp,
                                                              dtype=torch.bfloat16, device=dev))
    bias = torch.zeros(coutp, device=dev)
    y = ops.alloc_padded(B, S, 1, coutp, dev)
    cases["fwd%d" % ks] = (lambda xp=xp, wf=wf, bias=bias, y=y, hi=hi, cinp=cinp, coutp=coutp,
                           ks=ks: ops.conv_igemm(xp, wf, bias, y, B, S, hi, 1, cinp, coutp, ks,
                                                 True), y)
    if ks == 3:
        g = ops.pack_nchw(torch.randn(B, cout, S, S, device=dev), hi, coutp)
        dx = ops.alloc_padded(B, S, 1, cinp, dev)
        cases["dgrad3"] = (lambda g=g, wb=wb, dx=dx, xp=xp, cinp=cinp, coutp=coutp:
                           ops.conv_igemm(g, wb, None, dx, B, S, 1, 1, coutp, cinp, 3, False,
                                          mask=xp), dx)
VARIANTS = tuple(int(v) for v in os.environ.get("VARIANTS", "1,2,3,4").split(","))


def select(v):
    # v = 99: conv_tap (mode 1) with the round-2 register epilogue (RAG_EP_LDS A/B)
    _lib().rag_conv_tap_mode(1 if v == 99 else max(v - 1, 0))
    _lib().rag_conv_order(1 if v >= 1 else 0)
    _lib().rag_conv_ep_lds(0 if v == 99 else -1)


out = {}
for name, (fn, y) in cases.items():
    ref = None
    for v in VARIANTS:
        select(v)
        y.zero_()
        fn()
        torch.cuda.synchronize()
        if ref is None:
            ref = y.float().clone()
        else:
            out["%s_v%d_maxdiff" % (name, v)] = float((y.float() - ref).abs().max())
            out["%s_v%d_refmax" % (name, v)] = float(ref.abs().max())
rounds = {k: {v: [] for v in VARIANTS} for k in cases}
for r in range(5):
    for name, (fn, _) in cases.items():
        for v in VARIANTS:
            select(v)
            rounds[name][v].append(timeit(fn))
for name in cases:
    for v in VARIANTS:
        t = sorted(rounds[name][v])
        out["%s_v%d_us_median" % (name, v)] = round(t[len(t) // 2], 2)
        out["%s_v%d_us_min" % (name, v)] = round(t[0], 2)
print(json.dumps(out))
