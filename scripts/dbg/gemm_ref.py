"""Reference point: hipBLASLt bf16 GEMMs of the conv's implicit-GEMM shape (M = B*19*19 pixels,
N = 192 channels, K = 9*192) and a square one, timed with events."""
import json

import torch


def timeit(fn, iters=50):
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


res = {}
for (M, N, K) in [(256 * 361, 192, 1728), (256 * 361, 192, 192), (8192, 8192, 8192)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    us = timeit(lambda: a @ b)
    res["%dx%dx%d" % (M, N, K)] = {"us": round(us, 2), "tflops": round(2 * M * N * K / us / 1e6, 1)}
    bt = b.t().contiguous()
    us = timeit(lambda: a @ bt.t())
    res["%dx%dx%d_bT" % (M, N, K)] = {"us": round(us, 2),
                                      "tflops": round(2 * M * N * K / us / 1e6, 1)}
print(json.dumps(res))
