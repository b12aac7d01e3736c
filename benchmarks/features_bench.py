"""The 48-plane feature kernel (csrc/hip/features.hip) alone, on random mid-game 19x19
positions (rollout-policy games of 0-250 moves, host ladder planes), at the batch sizes of
self-play (128), the search wave (512) and single evaluations.

    python benchmarks/features_bench.py [--batch 1 16 128 512] [--iters 50]

One JSON line per batch: median us per launch."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 16, 128, 512])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--moves", type=int, nargs=2, default=[0, 250],
                    help="game lengths drawn from [lo, hi) rollout-policy moves")
    a = ap.parse_args(argv)
    from rocalphago_amd._native import engine
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.ops.features import GpuFeatures, _h2d
    rg = engine()
    dev = torch.device("cuda")
    rp = rg.RolloutPolicy()
    rs = np.random.RandomState(0)
    states = []
    for _ in range(max(a.batch)):
        st = GameState()
        for _ in range(int(rs.randint(a.moves[0], a.moves[1]))):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            st.do_move(None if mv < 0 else divmod(mv, 19))
        states.append(st.native)
    gf = GpuFeatures(DEFAULT_FEATURES, dev, 16, ladders="host")
    colors, ages, meta, illegal, lad = rg.gpu_feature_inputs(states, True, 16)
    c, ag, m, ld = (_h2d(x, dev) for x in (colors, ages, meta, lad))
    for B in a.batch:
        out = torch.empty((B, gf.F, 19, 19), dtype=torch.uint8, device=dev)
        sens = torch.empty((B, 361), dtype=torch.uint8, device=dev)

        def fn():
            gf.run(c[:B], ag[:B], m[:B], None, ld[:B], B, 19, out=out, sens_out=sens)

        ts = []
        s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            fn()
            torch.cuda.synchronize()
            s_ev.record()
            for _ in range(a.iters):
                fn()
            e_ev.record()
            torch.cuda.synchronize()
            ts.append(s_ev.elapsed_time(e_ev) / a.iters * 1e3)
        print(json.dumps({"batch": B, "moves": a.moves,
                          "median_us": round(statistics.median(ts), 2),
                          "min_us": round(min(ts), 2)}), flush=True)


if __name__ == "__main__":
    main()
