"""Host-side scaling probe: ladder planes (journaled vs copying reader) and feature inputs of
256 mid-game 19x19 positions at 1..16 threads, plus a C++-free Python baseline."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from boards import random_games  # noqa: E402
from rocalphago_amd._native import engine  # noqa: E402

rg = engine()
st = random_games(256, 19, 12, 100, 300)
b = [s.native for s in st]
out = {"cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
t = time.perf_counter()
for x in b:
    rg.ladder_planes(x, True)
out["copying_us_per_pos_1thr"] = (time.perf_counter() - t) / len(b) * 1e6
t = time.perf_counter()
for x in b:
    rg.ladder_planes(x, False)
out["journal_us_per_pos_1thr"] = (time.perf_counter() - t) / len(b) * 1e6
for nt in (1, 2, 4, 8, 16):
    rg.gpu_feature_inputs(b, True, nt)
    t = time.perf_counter()
    for _ in range(10):
        rg.gpu_feature_inputs(b, True, nt)
    out["inputs+ladders_ms_nt%d" % nt] = (time.perf_counter() - t) / 10 * 1e3
    t = time.perf_counter()
    for _ in range(10):
        rg.gpu_feature_inputs(b, False, nt)
    out["inputs_ms_nt%d" % nt] = (time.perf_counter() - t) / 10 * 1e3
print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}))
