"""Where the 3x3 conv time goes: the ping-pong kernel (conv_tap_pp_kernel) and three diagnostic
builds of it (wrong results) — no staging in the loop, no fragment reads, neither — timed in
interleaved rounds, with the in-kernel clock of each (s_memtime / s_memrealtime stamps of wave 0
around the main loop, median over blocks)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rocalphago_amd.ops import hipops as ops  # noqa: E402
from rocalphago_amd.ops.hipops import _lib  # noqa: E402

dev = torch.device("cuda")
B, S, C = int(os.environ.get("B", 256)), 19, int(os.environ.get("C", 192))
N128 = 16 if C == 128 else 0  # diag bit 4: the 128-channel (NT = 4) kernel
RS = int(os.environ.get("RS", 0))  # diag bits 5-6: register staging (timing builds only)
N128 |= RS << 5
x = torch.randn(B, C, S, S, device=dev).relu()
w = torch.randn(C, C, 3, 3, device=dev) * 0.05
xp = ops.pack_nchw(x, 1, C)
wf, _ = ops.pack_weights(w, C, C)
bias = torch.zeros(C, device=dev)
y = ops.alloc_padded(B, S, 1, C, dev)
lib = _lib()
P = ctypes.c_void_p
lib.rag_conv_pp_diag.argtypes = [ctypes.c_int, P, P, P, P, P] + [ctypes.c_int] * 9 + [P]
lib.rag_conv_diag_stamps.argtypes = [P, ctypes.c_int]
nblk = ((B * S * S + 383) // 384)


def run(diag):
    rc = lib.rag_conv_pp_diag(diag | N128, ops._ptr(xp), ops._ptr(wf), ops._ptr(bias), ops._ptr(y), None,
                              B, S, 1, 1, C, C, C, 1, 1, ops._stream())
    assert rc == 0, rc


def timeit(fn, iters=40):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


names = {0: "full", 1: "no_staging", 2: "no_frag_reads", 3: "mfma_only"}
if RS:
    names = {0: "full"}
res = {n: [] for n in names.values()}
clk = {}
for r in range(4):
    for d, n in names.items():
        res[n].append(timeit(lambda: run(d)))
        st = np.zeros(6 * nblk, np.int64)
        lib.rag_conv_diag_stamps(st.ctypes.data_as(P), nblk)
        st = st.reshape(nblk, 6).astype(np.float64)
        cyc, tick = st[:, 0], st[:, 1]
        ok = tick > 0
        clk.setdefault(n, []).append(float(np.median(cyc[ok] / tick[ok] * 0.1)))
        clk.setdefault(n + "_loop_us", []).append(float(np.median(tick[ok] / 100.0)))
        e, l0, l1, x_ = (st[ok, k] for k in (2, 3, 4, 5))
        t0 = e.min()
        prof = {"span_us": (x_.max() - t0) / 100, "entry_skew_us": (e.max() - t0) / 100,
                "prologue_us_med": float(np.median(l0 - e)) / 100,
                "loop_us_min": (l1 - l0).min() / 100, "loop_us_max": (l1 - l0).max() / 100,
                "epilogue_us_med": float(np.median(x_ - l1)) / 100,
                "last_loop_end_us": (l1.max() - t0) / 100}
        clk.setdefault(n + "_prof", []).append(prof)
# segment accounting (diag 8): per-wave cycles summed over the loop, median over blocks
lib.rag_conv_diag_segments.argtypes = [P, ctypes.c_int]
for _ in range(5):
    run(8)
seg = np.zeros(10 * nblk, np.int64)
lib.rag_conv_diag_segments(seg.ctypes.data_as(P), nblk)
seg = np.median(seg.reshape(nblk, 10).astype(np.float64), axis=0)
segments = {"g0_Xwait": seg[0], "g0_slab_read": seg[1], "g0_Ywait": seg[2],
            "g0_mfma_issue": seg[3], "g0_vmwait": seg[4], "g1_Xwait": seg[5], "g1_mfma_issue": seg[6],
            "g1_Ywait": seg[7], "g1_read": seg[8], "g1_stage_vmwait": seg[9]}
out = {"B": B, "C": C, "RS": RS,
       "segments_cycles_per_step": {k: round(v / (9.0 * C / 32), 1) for k, v in segments.items()}}
for n, v in res.items():
    out[n + "_us_min"] = round(min(v), 2)
    out[n + "_GHz"] = round(float(np.median(clk[n])), 3)
    out[n + "_loop_us_med"] = round(float(np.median(clk[n + "_loop_us"])), 2)
    pr = clk[n + "_prof"][-1]
    out[n + "_timeline"] = {k: round(v, 2) for k, v in pr.items()}
flop = 2.0 * B * 361 * C * 9 * C
out["full_TFLOPs"] = round(flop / out["full_us_min"] / 1e6, 1)
print(json.dumps(out))
