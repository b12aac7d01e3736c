"""RL policy-training throughput (reference benchmark:
/root/reference/benchmarks/reinforcement_policy_training_benchmark.py:7-29 — a cProfile of
``run_training`` on a 7x7 board, 32 filters, 4 layers, game batch 20, 10 iterations; the reference
publishes no number).

  python benchmarks/rl_bench.py [--config ref7|19] [--iterations N] [--game-batch G]
                                [--selfplay native|python]

ref7: the reference's benchmark shape through the real CLI (``run_training``: opponent sampling,
      self-play, per-game REINFORCE updates, a weights file per iteration).
19:   the north-star policy (48 planes, 192 filters, 13 layers) on 19x19, random-init weights,
      ``run_n_games`` directly (no file I/O), batched REINFORCE update.

One JSON line: games/s, learner positions/s (positions the learner trains on), plies/s of the
self-play and the host share of a ply (native path).
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REF_FEATURES = ["board", "ones", "turns_since", "liberties", "capture_size", "self_atari_size",
                "liberties_after", "sensibleness"]


def bench_ref7(args):
    import torch
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.training import reinforcement as rl
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    d = tempfile.mkdtemp(prefix="rlbench")
    try:
        pol = CNNPolicy(REF_FEATURES, board=7, filters_per_layer=32, layers=4, device=dev,
                        seed=1)
        model_file = os.path.join(d, "mini_rl_model.json")
        weights = os.path.join(d, "init_weights.hdf5")
        pol.model.save_weights(weights)
        pol.save_model(model_file)
        out = os.path.join(d, "rl_output")
        # untimed warmup iteration (compiles / allocates), then the timed run
        rl.run_training([model_file, weights, out + "_w", "--learning-rate", "0.001",
                         "--save-every", "2", "--game-batch", str(args.game_batch or 20),
                         "--iterations", "1"])
        stats = {"positions": 0, "plies": 0, "host_s": 0.0, "gpu_wait_s": 0.0}
        orig = rl.run_n_games

        def counted(*a, **k):
            r = orig(*a, **k)
            for key, v in getattr(orig, "last_stats", {}).items():
                stats[key] = stats.get(key, 0) + v
            return r
        rl.run_n_games = counted
        if dev == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        rl.run_training([model_file, weights, out, "--learning-rate", "0.001", "--save-every",
                         "2", "--game-batch", str(args.game_batch or 20), "--iterations",
                         str(args.iterations or 10)])
        if dev == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rl.run_n_games = orig
    finally:
        shutil.rmtree(d, ignore_errors=True)
    games = (args.game_batch or 20) * (args.iterations or 10)
    return {"config": "ref7: 7x7, %s, 32 filters x 4 layers, game batch %d, %d iterations, "
                      "run_training CLI (per-game REINFORCE steps, a weights file per iteration)"
                      % ("+".join(REF_FEATURES), args.game_batch or 20, args.iterations or 10),
            "games_per_s": games / dt, "seconds": dt, "games": games, "self_play": stats}


def bench_19(args):
    import numpy as np
    import torch
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.players.ai import ProbabilisticPolicyPlayer
    from rocalphago_amd.training import reinforcement as rl
    dev = torch.device("cuda")
    learner_pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=12,
                            device=dev, seed=1)
    opp_pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=12,
                        device=dev, seed=2)
    opt = K.SGD(lr=0.001)
    learner_pol.model.compile(loss=rl.log_loss, optimizer=opt)
    learner = ProbabilisticPolicyPlayer(learner_pol, temperature=0.67, move_limit=500,
                                        rng=np.random.RandomState(1))
    opponent = ProbabilisticPolicyPlayer(opp_pol, temperature=0.67, move_limit=500,
                                         rng=np.random.RandomState(2))
    G = args.game_batch or 128
    rl.run_n_games(opt, learner, opponent, 8, mode="batched")  # warmup
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = {"positions": 0, "plies": 0, "host_s": 0.0, "gpu_wait_s": 0.0}
    wins = []
    for _ in range(args.iterations or 2):
        wins.append(rl.run_n_games(opt, learner, opponent, G, mode="batched"))
        for key, v in getattr(rl.run_n_games, "last_stats", {}).items():
            stats[key] = stats.get(key, 0) + v
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    games = G * (args.iterations or 2)
    return {"config": "19x19 north-star policy (48 planes, 192 filters, 13 layers) vs a second "
                      "random-init policy, T=0.67, move limit 500, game batch %d, batched "
                      "REINFORCE update, %d iterations" % (G, args.iterations or 2),
            "games_per_s": games / dt, "seconds": dt, "games": games, "self_play": stats,
            "win_ratio_mean": float(np.mean(wins))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ref7", choices=["ref7", "19"])
    ap.add_argument("--iterations", type=int, default=None)
    ap.add_argument("--game-batch", type=int, default=None)
    ap.add_argument("--selfplay", default="native", choices=["native", "python"])
    ap.add_argument("--pipeline", type=int, default=None,
                    help="native self-play: pipelined game groups (default 2)")
    args = ap.parse_args()
    from rocalphago_amd.training import reinforcement
    reinforcement.NATIVE_SELFPLAY = args.selfplay == "native"
    if args.pipeline is not None:
        reinforcement.SELFPLAY_PIPELINE = args.pipeline
    r = bench_ref7(args) if args.config == "ref7" else bench_19(args)
    sp = r.pop("self_play")
    r["selfplay"] = args.selfplay
    r["metric"] = "RL policy training games/s"
    if sp.get("plies"):
        tot = sp["host_s"] + sp["gpu_wait_s"]
        r["learner_positions_per_s"] = sp["positions"] / r["seconds"] / 2.0
        r["selfplay_plies"] = sp["plies"]
        r["selfplay_host_share"] = round(sp["host_s"] / tot, 3) if tot else None
        # where a ply's host time goes (s over the run): native pack / GPU launch (graph
        # replay) / native play, and the time waiting on the GPU
        r["selfplay_split_s"] = {k: round(sp[k], 3) for k in ("pack_s", "launch_s", "play_s",
                                                              "host_s", "gpu_wait_s",
                                                              "gpu_pass_s", "wall_s", "rec_s",
                                                              "gather_s")
                                 if k in sp}
        # share of the self-play wall time the GPU spends in ply passes: with the two pipelined
        # groups a busy host overlaps the other group's GPU pass, so this, not the host share,
        # says which side bounds the loop
        if sp.get("wall_s") and "gpu_pass_s" in sp:
            r["selfplay_gpu_busy"] = round(sp["gpu_pass_s"] / sp["wall_s"], 3)
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
