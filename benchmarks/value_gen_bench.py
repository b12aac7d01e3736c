"""Value-dataset generation throughput (the reference's value trainer is an empty
file and value.py only stubs — BASELINE config #4 trains on self-play positions): games/s of
``generate_value_dataset`` with the north-star policy (48 planes, 192 filters, 13 layers,
random-init weights) on 19x19, native lock-step batch vs the Python get_moves loop.

  python benchmarks/value_gen_bench.py [--games N] [--batch-games G] [--move-limit L]
                                       [--loop native|python]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=256)
    ap.add_argument("--batch-games", type=int, default=256)
    ap.add_argument("--move-limit", type=int, default=500)
    ap.add_argument("--loop", default="native", choices=["native", "python"])
    args = ap.parse_args()
    import numpy as np
    import torch
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.players.ai import ProbabilisticPolicyPlayer
    from rocalphago_amd.training import value_trainer as vt
    dev = torch.device("cuda")
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=12, device=dev,
                    seed=1)
    player = ProbabilisticPolicyPlayer(pol, temperature=0.67, move_limit=args.move_limit,
                                       rng=np.random.RandomState(1))
    kw = dict(board=19, features=list(DEFAULT_FEATURES) + ["color"],
              move_limit=args.move_limit, batch_games=args.batch_games,
              native=args.loop == "native")
    vt.generate_value_dataset(player, 8, rng=np.random.RandomState(0), **kw)  # warmup
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    X, y = vt.generate_value_dataset(player, args.games, rng=np.random.RandomState(1), **kw)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "value-dataset self-play games/s", "loop": args.loop,
                      "games": args.games, "batch_games": args.batch_games,
                      "seconds": round(dt, 3), "games_per_s": round(args.games / dt, 3),
                      "rows": int(len(X)), "label_mean": round(float(y.mean()), 3),
                      "config": "19x19 north-star policy (48x192x13, random init), T=0.67, "
                                "move limit %d, one sampled position per game" % args.move_limit}))


if __name__ == "__main__":
    main()
