"""Direct (conv_tap_pp) vs Winograd F(2,3) (conv_wino) 3x3 192->192 kernels, forward and dgrad
(+ ReLU mask), interleaved rounds in one process (guide §5.4 rule 24), on random data.

    python benchmarks/wino_bench.py [--batch 256] [--rounds 5] [--iters 40]

Prints one JSON line: median / min microseconds per launch of every (kernel, pass), the
effective dense-equivalent TFLOP/s (2 * B * 361 * 192 * 1728 FLOP per launch, i.e. what the
direct algorithm would need) and the max relative difference of the two kernels' outputs."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--size", type=int, default=19)
    ap.add_argument("--diag", default="", help="comma list of conv_wino DIAG timing variants "
                    "(wrong results): 1 no transform, 2 no raw staging, 4 no weight staging, "
                    "8 no MFMAs, 16 no fragment reads, 32 no output stores")
    ap.add_argument("--segments", action="store_true",
                    help="s_memtime segment accounting of the Winograd loop (DIAG 64)")
    a = ap.parse_args(argv)
    from rocalphago_amd.ops import hipops as ops
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B, S, C = a.batch, a.size, 192
    x = torch.randn(B, C, S, S, device=dev).relu()
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    g = torch.randn(B, C, S, S, device=dev)
    xp = ops.pack_nchw(x, 1, C)
    gp = ops.pack_nchw(g, 1, C)
    wf, wb = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
    uf, ub = ops.wino_weights(w, C, C)
    bias = torch.randn(C, device=dev) * 0.1
    y = {k: ops.alloc_padded(B, S, 1, C, dev) for k in ("fd", "fw", "dd", "dw")}
    cases = {
        "fwd_direct": lambda: ops.conv_igemm(xp, wf, bias, y["fd"], B, S, 1, 1, C, C, 3, True),
        "fwd_wino": lambda: ops.conv_wino(xp, uf, bias, y["fw"], B, S, C, C, 1, True),
        "dgrad_direct": lambda: ops.conv_igemm(gp, wb, None, y["dd"], B, S, 1, 1, C, C, 3,
                                               False, mask=xp),
        "dgrad_wino": lambda: ops.conv_wino(gp, ub, None, y["dw"], B, S, C, C, 1, False,
                                            mask=xp),
    }
    lib = ops._lib()
    for d in [int(v) for v in a.diag.split(",") if v]:
        yd = ops.alloc_padded(B, S, 1, C, dev)
        cases["fwd_wino_diag%d" % d] = (
            lambda d=d, yd=yd: lib.rag_conv_wino_diag(d, xp.data_ptr(), uf.data_ptr(),
                                                      bias.data_ptr(), yd.data_ptr(), None, B, S,
                                                      C, C, 1, C, 1, 1, ops._stream()))
    times = {k: [] for k in cases}
    s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for k, fn in cases.items():
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            s_ev.record()
            for _ in range(a.iters):
                fn()
            e_ev.record()
            torch.cuda.synchronize()
            times[k].append(s_ev.elapsed_time(e_ev) / a.iters * 1e3)
    flop = 2.0 * B * S * S * C * C * 9
    out = {"batch": B, "size": S}
    for k, ts in times.items():
        med = statistics.median(ts)
        out[k] = {"median_us": round(med, 2), "min_us": round(min(ts), 2),
                  "dense_equiv_tflops": round(flop / med / 1e6, 1)}

    def rel(p, q):
        p, q = ops.unpack(p, C, 1), ops.unpack(q, C, 1)
        return round(((p - q).norm() / q.norm()).item(), 5)

    if a.segments:
        import numpy as np
        yd = ops.alloc_padded(B, S, 1, C, dev)
        for _ in range(3):
            rc = lib.rag_conv_wino_diag(64, xp.data_ptr(), uf.data_ptr(), bias.data_ptr(),
                                        yd.data_ptr(), None, B, S, C, C, 1, C, 1, 1, ops._stream())
            assert rc == 0, rc
        nblk = B  # one board per block at 19x19
        st = np.zeros((nblk, 8, 6), np.int64)
        assert lib.rag_conv_wino_stamps(st.ctypes.data, nblk) == 0
        steps = 6 * 2 * (C // 32)
        out["segments_cycles_per_step"] = {
            "group0 [Xwait, stage, read, Ywait, mfma, post]":
                [round(float(v), 1) for v in st[:, 0:4].mean((0, 1)) / steps],
            "group1 [Xwait, mfma, transform, Ywait, read, stage]":
                [round(float(v), 1) for v in st[:, 4:8].mean((0, 1)) / steps]}
    out["fwd_rel_diff"] = rel(y["fw"], y["fd"])
    out["dgrad_rel_diff"] = rel(y["dw"], y["dd"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
