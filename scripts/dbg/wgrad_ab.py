"""Weight-gradient kernels: slab ring depth A/B (rag_wgrad_slab_nbuf 3/4/5, interleaved rounds in
one process) for the 3x3 192->192 layer, plus the taps kernel shapes (5x5 48->192, 3x3 128->128),
each checked against an fp32 torch reference of dW = conv2d weight gradient."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

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
B, S = 256, 19
out = {}
for (cin, cout, ks, variants) in [(192, 192, 3, (3, 4, 5)), (48, 192, 5, (3,)),
                                  (128, 128, 3, (3,))]:
    cinp, coutp = ops.pad_channels(cin), ops.pad_channels(cout)
    hi = ks // 2
    x = torch.randn(B, cin, S, S, device=dev).relu()
    gy = torch.randn(B, cout, S, S, device=dev)
    xp = ops.pack_nchw(x, hi, cinp)
    g = ops.pack_nchw(gy, hi, coutp)
    dw = torch.zeros(cout, cin, ks, ks, device=dev)
    db = torch.zeros(cout, device=dev)
    work = ops.wgrad_workspace(B, S, coutp, cinp, ks, dev)
    fn = lambda: ops.conv_wgrad(g, xp, dw, db, B, S, hi, cout, coutp, cin, cinp, ks, work=work)  # noqa
    xr = x.to(torch.bfloat16).float().requires_grad_()
    wr = torch.zeros(cout, cin, ks, ks, device=dev, requires_grad=True)
    y = F.conv2d(xr, wr, padding=ks // 2)
    ref = torch.autograd.grad(y, wr, gy.to(torch.bfloat16).float())[0]
    name = "w%d_%d" % (ks, cin)
    for v in variants:
        _lib().rag_wgrad_slab_nbuf(v)
        dw.zero_()
        db.zero_()
        fn()
        torch.cuda.synchronize()
        err = float((dw - ref).abs().max() / ref.abs().max())
        out["%s_nbuf%d_relerr" % (name, v)] = round(err, 5)
    ts = {v: [] for v in variants}
    for r in range(5):
        for v in variants:
            _lib().rag_wgrad_slab_nbuf(v)
            ts[v].append(timeit(fn))
    for v in variants:
        t = sorted(ts[v])
        out["%s_nbuf%d_us_median" % (name, v)] = round(t[len(t) // 2], 2)
print(json.dumps(out))
