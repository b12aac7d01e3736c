"""Direct (conv_tap_pp) vs Winograd F(2,3) (conv_wino) 3x3 192->192 kernels, forward and dgrad
(+ ReLU mask), interleaved rounds in one process (guide §5.4 rule 24), on random data.

    python benchmarks/wino_bench.py [--batch 256 [128 64 ...]] [--rounds 5] [--iters 40]
                                    [--wcopies 16] [--xcopies 8]

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
    ap.add_argument("--batch", type=int, nargs="+", default=[256],
                    help="one JSON line per batch (small batches: the self-play tail)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--size", type=int, default=19)
    ap.add_argument("--channels", type=int, default=192, help="192 or 128 (the 128-wide tile)")
    ap.add_argument("--wcopies", type=int, default=1,
                    help="rotate over this many copies of the weights (cold L2, as in the step)")
    ap.add_argument("--xcopies", type=int, default=1,
                    help="rotate over this many copies of the inputs (beyond the 256 MB MALL)")
    a = ap.parse_args(argv)
    for B in a.batch:
        run(a, B)


def run(a, B):
    from rocalphago_amd.ops import hipops as ops
    dev = torch.device("cuda")
    torch.manual_seed(0)
    S, C = a.size, a.channels
    x = torch.randn(B, C, S, S, device=dev).relu()
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    g = torch.randn(B, C, S, S, device=dev)
    xps = [ops.pack_nchw(x, 1, C) for _ in range(a.xcopies)]
    gps = [ops.pack_nchw(g, 1, C) for _ in range(a.xcopies)]
    xp, gp = xps[0], gps[0]
    wf, wb = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
    uf, ub = ops.wino_weights(w, C, C)
    wfs, wbs = [wf] + [wf.clone() for _ in range(a.wcopies - 1)], \
        [wb] + [wb.clone() for _ in range(a.wcopies - 1)]
    ufs, ubs = [uf] + [uf.clone() for _ in range(a.wcopies - 1)], \
        [ub] + [ub.clone() for _ in range(a.wcopies - 1)]
    bias = torch.randn(C, device=dev) * 0.1
    y = {k: ops.alloc_padded(B, S, 1, C, dev) for k in ("fd", "fw", "fh", "dd", "dw")}
    it = {}

    def nxt(v):
        i = it[id(v)] = it.get(id(v), -1) + 1
        return v[i % len(v)]

    cases = {
        "fwd_direct": lambda: ops.conv_igemm(nxt(xps), nxt(wfs), bias, y["fd"], B, S, 1, 1, C,
                                             C, 3, True),
        "fwd_wino": lambda: ops.conv_wino(nxt(xps), nxt(ufs), bias, y["fw"], B, S, C, C, 1,
                                          True),
        # half-board blocks (two per board) at any batch (192-wide tiles)
        "fwd_wino_half": lambda: ops.conv_wino(nxt(xps), nxt(ufs), bias, y["fh"], B, S, C, C, 1,
                                               True, half=True),
        "dgrad_direct": lambda: ops.conv_igemm(nxt(gps), nxt(wbs), None, y["dd"], B, S, 1, 1, C,
                                               C, 3, False, mask=xp),
        "dgrad_wino": lambda: ops.conv_wino(nxt(gps), nxt(ubs), None, y["dw"], B, S, C, C, 1,
                                            False, mask=xp),
    }
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

    out["fwd_rel_diff"] = rel(y["fw"], y["fd"])
    out["fwd_half_rel_diff"] = rel(y["fh"], y["fd"])
    out["dgrad_rel_diff"] = rel(y["dw"], y["dd"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
