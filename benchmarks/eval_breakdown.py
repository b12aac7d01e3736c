"""Time the pieces of one APV-MCTS leaf-evaluation wave (diagnostic)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from rocalphago_amd._native import engine
from rocalphago_amd.engine.gamestate import GameState
from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
from rocalphago_amd.models.policy import CNNPolicy
from rocalphago_amd.models.value import CNNValue
from rocalphago_amd.ops.features import GpuFeatures

rg = engine()


def tm(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3, r


def main():
    dev = torch.device("cuda")
    rp = rg.RolloutPolicy()
    states = []
    rs = np.random.RandomState(0)
    for i in range(256):
        st = GameState()
        for k in range(int(rs.randint(0, 250))):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            st.do_move(None if mv < 0 else divmod(mv, 19))
        states.append(st)
    boards = [s.native for s in states]
    feats = DEFAULT_FEATURES + ["color"]
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=12, device=dev)
    val = CNNValue(feats, board=19, filters_per_layer=192, layers=12, device=dev)
    gf = GpuFeatures(feats, dev, 16)
    for nt in (8, 16):
        print("inputs+ladders nthreads=%d: %.2f ms" % (nt, tm(lambda: rg.gpu_feature_inputs(
            boards, True, nt))[0]))
    print("inputs no ladders: %.2f ms" % tm(lambda: rg.gpu_feature_inputs(boards, False, 16))[0])
    t, x = tm(lambda: gf(boards))
    print("GpuFeatures total (host ladders, 16 threads): %.2f ms" % t)
    gfg = GpuFeatures(feats, dev, 16, ladders="gpu")
    print("GpuFeatures total (GPU ladder kernel): %.2f ms" % tm(lambda: gfg(boards))[0])
    print("native batch_features 16 thr: %.2f ms" % tm(lambda: rg.batch_features(
        boards, gf.fids, 16))[0])
    xp = x[:, :48].contiguous()
    print("policy predict: %.2f ms" % tm(lambda: pol.model.predict(xp))[0])
    print("value predict: %.2f ms" % tm(lambda: val.model.predict(x))[0])
    plan = pol.model._plan_for()
    print("policy plan.forward (no host copy): %.2f ms" % tm(lambda: plan.forward(xp))[0])


if __name__ == "__main__" and "--wave" not in sys.argv:
    main()


def wave_breakdown():
    """Synchronised timing of each step of real search waves."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from mcts_bench import build_search
    dev = torch.device("cuda")
    mc = build_search(dev)
    st = GameState()
    s = mc.search(st, 1024)
    acc = {}

    def mark(k, t0):
        torch.cuda.synchronize()
        t = time.perf_counter()
        acc[k] = acc.get(k, 0.0) + (t - t0) * 1e3
        return t

    for _ in range(10):
        t = time.perf_counter()
        wid, n = s.select(256)
        t = mark("select", t)
        boards = s.leaf_boards(wid)
        t = mark("leaf_boards", t)
        pend = mc._gpu_rollouts(s, wid)
        t = mark("rollout_launch", t)
        ev = mc.evaluator
        x = ev._extract(ev.vfids, "p", boards)
        t = mark("features", t)
        pr = ev.policy.model.predict(x[:, :ev.npol].contiguous())
        t = mark("policy", t)
        v = ev.value.model.predict(x)
        t = mark("value", t)
        z = pend.result()
        t = mark("rollout_wait", t)
        s.backup_value(wid, np.ascontiguousarray(pr, np.float32),
                       np.ascontiguousarray(v, np.float32))
        s.backup_rollout(wid, z)
        t = mark("backup", t)
    print("per wave (ms):", {k: round(v / 10, 2) for k, v in acc.items()}, "n", n)


if __name__ == "__main__" and "--wave" in sys.argv:
    wave_breakdown()
