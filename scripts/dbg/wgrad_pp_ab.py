"""A/B of the 192-channel wgrad kernels at B=256 (interleaved rounds, one process): the 12-wave
slab kernel vs the ping-pong 8-wave kernel (rag_wgrad_slab_pp), each with its reduction deferred
into a dgrad launch (the trunk's schedule) and the wgrad kernel alone (standalone reduction)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from rocalphago_amd.ops import hipops as ops  # noqa: E402


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
B, S, C = int(os.environ.get("B", 256)), 19, 192
x = torch.randn(B, C, S, S, device=dev).relu()
w = torch.randn(C, C, 3, 3, device=dev) * 0.05
xp = ops.pack_nchw(x, 1, C)
gp = ops.pack_nchw(torch.randn(B, C, S, S, device=dev), 1, C)
_, wb = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
dw, db = torch.zeros(C, C, 3, 3, device=dev), torch.zeros(C, device=dev)
y = ops.alloc_padded(B, S, 1, C, dev)
work = ops.wgrad_workspace(B, S, C, C, 3, dev)
h = ops.PendingReduction()
lib = ops._lib()


def pair():
    ops.conv_wgrad(gp, xp, dw, db, B, S, 1, C, C, C, C, 3, work=work, hg=1, defer=True, pending=h)
    ops.conv_igemm(gp, wb, None, y, B, S, 1, 1, C, C, 3, False, mask=xp, pending=h)


res = {"B": B}
for rnd in range(3):
    for pp in (0, 1):
        lib.rag_wgrad_slab_pp(pp)
        res.setdefault("pp%d_wgrad_dgrad_us" % pp, []).append(round(timeit(pair), 2))
        res.setdefault("pp%d_wgrad_alone_us" % pp, []).append(round(timeit(lambda: ops.conv_wgrad(
            gp, xp, dw, db, B, S, 1, C, C, C, C, 3, work=work, hg=1)), 2))
lib.rag_wgrad_slab_pp(-1)
res["dgrad_alone_us"] = round(timeit(lambda: ops.conv_igemm(gp, wb, None, y, B, S, 1, 1, C, C, 3,
                                                            False, mask=xp)), 2)
print(json.dumps(res))
