"""Direct slab (wgrad_slab.hip) vs Winograd F(2,3) (wgrad_wino.hip) weight gradient of a 3x3
192 -> 192 layer, interleaved rounds in one process, on random data: the wgrad kernel alone
(reduction deferred, then flushed outside the timed region) and with its chunk reduction.

    python benchmarks/wgrad_bench.py [--batch 256] [--rounds 5] [--iters 30] [--copies 8]

Prints one JSON line: median / min microseconds per launch and the relative difference of the
two kernels' dW."""
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
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--copies", type=int, default=8,
                    help="rotate over this many (G, X) copies (cold caches, as in the step)")
    a = ap.parse_args(argv)
    from rocalphago_amd.ops import hipops as ops
    lib = ops._lib()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B, S, C = a.batch, 19, 192
    xs = [ops.pack_nchw(torch.randn(B, C, S, S, device=dev).relu(), 1, C) for _ in range(a.copies)]
    gs = [ops.pack_nchw(torch.randn(B, C, S, S, device=dev), 1, C) for _ in range(a.copies)]
    work = ops.wgrad_workspace(B, S, C, C, 3, dev)
    dw = {m: torch.zeros(C, C, 3, 3, device=dev) for m in (0, 1)}
    db = {m: torch.zeros(C, device=dev) for m in (0, 1)}
    # the kernel alone: every launch leaves its reduction in a handle of its own (a handle's next
    # deferral would launch the previous one), all flushed after the timed region
    hs = [ops.PendingReduction() for _ in range(a.iters + 3)]
    it = [0]

    def run(mode, reduce):
        i = it[0] = it[0] + 1
        lib.rag_wgrad_wino_mode(mode)
        g, x = gs[i % a.copies], xs[i % a.copies]
        if reduce:
            ops.conv_wgrad(g, x, dw[mode], db[mode], B, S, 1, C, C, C, C, 3, work=work, hg=1)
        else:
            ops.conv_wgrad(g, x, dw[mode], db[mode], B, S, 1, C, C, C, C, 3, work=work, hg=1,
                           defer=True, pending=hs[i % len(hs)])

    def flush():
        for h in hs:
            ops.wgrad_flush(h)

    cases = {"direct": (0, False), "wino": (1, False), "direct+reduce": (0, True),
             "wino+reduce": (1, True)}
    times = {k: [] for k in cases}
    s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    prev = lib.rag_wgrad_wino_mode(-1)
    try:
        for _ in range(a.rounds):
            for k, (mode, red) in cases.items():
                for _ in range(3):
                    run(mode, red)
                flush()
                torch.cuda.synchronize()
                s_ev.record()
                for _ in range(a.iters):
                    run(mode, red)
                e_ev.record()
                torch.cuda.synchronize()
                flush()
                times[k].append(s_ev.elapsed_time(e_ev) / a.iters * 1e3)
        # the two kernels' dW on the same inputs
        for m in (0, 1):
            lib.rag_wgrad_wino_mode(m)
            ops.conv_wgrad(gs[0], xs[0], dw[m], db[m], B, S, 1, C, C, C, C, 3, work=work, hg=1)
        torch.cuda.synchronize()
    finally:
        lib.rag_wgrad_wino_mode(prev)
    out = {"batch": B, "size": S}
    for k, ts in times.items():
        out[k] = {"median_us": round(statistics.median(ts), 2), "min_us": round(min(ts), 2)}
    out["dw_rel_diff"] = round(((dw[1] - dw[0]).norm() / dw[0].norm()).item(), 5)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
