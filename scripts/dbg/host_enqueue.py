"""Host-side cost of enqueuing one search wave's network work (policy + value forward, B=256)
vs replaying it from a captured graph."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES  # noqa: E402
from rocalphago_amd.models.policy import CNNPolicy  # noqa: E402
from rocalphago_amd.models.value import CNNValue  # noqa: E402


def main():
    dev = torch.device("cuda")
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=12, device=dev)
    val = CNNValue(DEFAULT_FEATURES + ["color"], board=19, filters_per_layer=192, layers=12,
                   device=dev)
    pp, pv = pol.model._plan_for(), val.model._plan_for()
    x = (torch.rand(256, 49, 19, 19, device=dev) > 0.7).to(torch.uint8)
    xp = x[:, :48].contiguous()

    def wave():
        with torch.no_grad():
            a = pp.forward(xp)
            b = pv.forward(x)
        return a, b

    for _ in range(5):
        wave()
    torch.cuda.synchronize()
    n = 50
    t_enq = 0.0
    t0 = time.perf_counter()
    for i in range(n):
        t = time.perf_counter()
        wave()
        t_enq += time.perf_counter() - t
        torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    res = {"enqueue_ms": round(t_enq / n * 1e3, 3), "wave_ms_synced": round(t_all / n * 1e3, 3)}
    # graph replay of the same work
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        wave()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            out = wave()
    torch.cuda.synchronize()
    a_ref, b_ref = wave()
    g.replay()
    torch.cuda.synchronize()
    res["graph_max_diff"] = max((out[0] - a_ref).abs().max().item(),
                                (out[1] - b_ref).abs().max().item())
    t_enq = 0.0
    t0 = time.perf_counter()
    for i in range(n):
        t = time.perf_counter()
        g.replay()
        t_enq += time.perf_counter() - t
        torch.cuda.synchronize()
    res["graph_enqueue_ms"] = round(t_enq / n * 1e3, 3)
    res["graph_wave_ms_synced"] = round((time.perf_counter() - t0) / n * 1e3, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
