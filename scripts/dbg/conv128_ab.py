"""Per-kernel timing of the 3x3 conv forms at 128 and 192 channels, B=256: forward (bias+ReLU,
LDS-staged epilogue), forward with residual (register epilogue), dgrad with ReLU mask, wgrad
(slab, reduction standalone). Variants: tap mode 6 (ping-pong) vs 0 (conv_pipe); at 128
channels also the two-K-steps-per-barrier-pair kernel (K2 env list, default "0,1,2")."""
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
out = {"B": B}
for C in (128, 192):
    x = torch.randn(B, C, S, S, device=dev).relu()
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    xp = ops.pack_nchw(x, 1, C)
    rp = ops.pack_nchw(torch.randn(B, C, S, S, device=dev), 1, C)
    wf, wb = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
    bias = torch.zeros(C, device=dev)
    y = ops.alloc_padded(B, S, 1, C, dev)
    g = ops.pack_nchw(torch.randn(B, C, S, S, device=dev), 1, C)
    dw, db = torch.zeros(C, C, 3, 3, device=dev), torch.zeros(C, device=dev)
    work = ops.wgrad_workspace(B, S, C, C, 3, dev)
    cases = {
        "fwd": lambda: ops.conv_igemm(xp, wf, bias, y, B, S, 1, 1, C, C, 3, True),
        "fwd_res": lambda: ops.conv_igemm(xp, wf, None, y, B, S, 1, 1, C, C, 3, False,
                                          residual=rp),
        "dgrad": lambda: ops.conv_igemm(g, wb, None, y, B, S, 1, 1, C, C, 3, False, mask=xp),
    }
    for mode in (6, 0):
        _lib().rag_conv_tap_mode(mode)
        for k, fn in cases.items():
            out["c%d_%s_mode%d_us" % (C, k, mode)] = round(timeit(fn), 2)
    _lib().rag_conv_tap_mode(6)
    out["c%d_wgrad_us" % C] = round(timeit(lambda: ops.conv_wgrad(
        g, xp, dw, db, B, S, 1, C, C, C, C, 3, work=work, hg=1)), 2)
    _lib().rag_conv_tap_mode(12)  # the default mode (the RS variants are mode-12 kernels)
    coef = torch.zeros(3, S, device=dev)
    coef[0] = 1.0
    if C == 128:  # BN prologue forms (ResnetPolicy)
        cases["bn_fwd_res"] = lambda: ops.conv_igemm_bn(
            xp, wf, None, y, B, S, C, C, False, bn_coef=coef, residual=rp)
        cases["bn_dgrad"] = lambda: ops.conv_igemm_bn(
            g, wb, None, y, B, S, C, C, False, mask=xp, mask_coef=coef)
    # variants (interleaved repeats): "k2_<v>" (rag_conv_k2) / "rs_<v>" (rag_conv_rs)
    variants = os.environ.get("VARIANTS", "k2_0,k2_1,rs_1,rs_2").split(",")
    for rep in range(2):
        for var in variants:
            knob, v = var.rsplit("_", 1)
            getattr(_lib(), "rag_conv_" + knob)(int(v))
            for k, fn in cases.items():
                key = "c%d_%s_%s_us" % (C, k, var)
                t = round(timeit(fn), 2)
                out[key] = min(out.get(key, 1e9), t)
            getattr(_lib(), "rag_conv_" + knob)(0)
    if C == 128:
        out["c128_bn_fwd_res_us"] = out.get("c128_bn_fwd_res_k2_0_us")
        out["c128_bn_dgrad_us"] = out.get("c128_bn_dgrad_k2_0_us")
        out["c128_bn_wgrad_us"] = round(timeit(lambda: ops.conv_wgrad(
            g, xp, dw, db, B, S, 1, C, C, C, C, 3, work=work, hg=1, xcoef=coef)), 2)
        h = ops.PendingReduction()

        def pair(bn):
            ops.conv_wgrad(g, xp, dw, db, B, S, 1, C, C, C, C, 3, work=work, hg=1, defer=True,
                           pending=h, xcoef=coef if bn else None)
            if bn:
                ops.conv_igemm_bn(g, wb, None, y, B, S, C, C, False, mask=xp, mask_coef=coef,
                                  pending=h)
            else:
                ops.conv_igemm(g, wb, None, y, B, S, 1, 1, C, C, 3, False, mask=xp, pending=h)
        out["c128_wgrad_dgrad_deferred_us"] = round(timeit(lambda: pair(False)), 2)
        out["c128_bn_wgrad_dgrad_deferred_us"] = round(timeit(lambda: pair(True)), 2)
    print(json.dumps(out), flush=True)
