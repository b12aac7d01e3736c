"""APV-MCTS throughput (BASELINE config #5): simulations/s of the full search on 19x19 —
north-star policy (48 planes, 192 filters, 12+1 layers) + value net (49 planes, same trunk, FC256,
tanh) evaluated on the GPU for every wave of leaves, fast rollouts on the GPU (rollout kernel,
``--rollouts-per-leaf`` games per leaf), lambda = 0.5, random-init weights, from the empty board.

  python benchmarks/mcts_bench.py [--playouts 8192] [--batch 256] [--rollout-device gpu|cpu]

One JSON line: sims/s, leaf evals/s, rollouts/s and the per-phase time split.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build_search(device, filters=192, layers=12, batch=512, rollout_device="gpu",
                 rollouts_per_leaf=1, lmbda=0.5, nthreads=16, seed=1, pipeline=3,
                 max_inflight=8, rollout_group=8):
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.models.value import CNNValue
    from rocalphago_amd.search.apv import ParallelMCTS
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=filters, layers=layers,
                    device=device, seed=seed)
    val = CNNValue(DEFAULT_FEATURES + ["color"], board=19, filters_per_layer=filters,
                   layers=layers, device=device, seed=seed + 1)
    return ParallelMCTS(pol, val, lmbda=lmbda, batch=batch, rollout_device=rollout_device,
                        rollouts_per_leaf=rollouts_per_leaf, nthreads=nthreads, seed=seed,
                        pipeline=pipeline, max_inflight=max_inflight,
                        rollout_group=rollout_group)


def measure(device, playouts=8192, warmup=512, moves=1, **kw):
    import torch
    from rocalphago_amd.engine.gamestate import GameState
    mc = build_search(device, **kw)
    mc.n_playout = playouts
    st = GameState()
    mc.search(st, warmup)  # compiles / allocates; discarded tree
    mc._search = None
    mc.stats = {"waves": 0, "sims": 0}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(moves):
        mv = mc.get_move(st)
        st.do_move(mv)
        mc.update_with_move(mv)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    s = mc.stats
    out = {"sims_per_s": s["sims"] / dt, "sims": s["sims"], "seconds": dt,
           "waves": s["waves"], "batch": mc.batch, "rollouts_per_leaf": mc.rollouts_per_leaf,
           "rollout_device": mc.rollout_device}
    if mc.lmbda > 0:
        out["rollouts_per_s"] = s["sims"] * (mc.rollouts_per_leaf if mc.rollout_device == "gpu"
                                             else 1) / dt
    for k in ("t_select", "t_submit", "t_eval", "t_rollout_wait", "t_backup"):
        out[k + "_frac"] = round(s.get(k, 0.0) / dt, 3)
    return out


# The N-GPU search's geometry (leaves per GPU wave, waves per GPU awaiting values, rank 0's share
# of a wave), chosen by effective throughput = one GPU's serving rate x N (capped by rank 0's
# host ceiling) x budget efficiency (benchmarks/search_efficiency.py --effective,
# profiles/search_efficiency_r6.json). The leaves in flight grow with N x wave, so the wave
# shrinks as N grows: 512 / N leaves per GPU, at least 128 (argmax at N = 4 and 8, within 2 % of
# it at N = 2 where 256 keeps efficiency 0.98 against 0.85 at 512).
DIST_GEOMETRY = {"batch": 512, "min_batch": 128, "depth": 2, "master_share": 1.0}


def distributed_wave(world, mode="master"):
    """Leaves per GPU wave of the N-GPU search (mode "shared": every rank runs the one-GPU
    search, 512)."""
    if mode != "master" or world <= 1:
        return 512
    return max(DIST_GEOMETRY["min_batch"], DIST_GEOMETRY["batch"] // world)


def measure_distributed(dp, device, playouts=8192, warmup=512, moves=1, filters=192,
                        layers=12, batch=512, rollouts_per_leaf=1, lmbda=0.5, nthreads=16,
                        seed=1, mode="master", depth=None, master_share=None,
                        rollout_group=None):
    """Search over all ranks (search/distributed.py). mode "master" (default): one tree on rank 0
    with leaf waves served by every rank through the shared-memory channel (DistributedMCTS);
    "shared": every rank runs the pipelined single-GPU search with shared root statistics
    (SharedRootMCTS; its duplicated expansions are measured and reported).
    Collective: every rank calls it; rank 0's dict has the job's sims/s, the others None."""
    if mode == "shared":
        return _measure_shared(dp, device, playouts, warmup, moves, filters, layers, batch,
                               rollouts_per_leaf, lmbda, nthreads, seed)
    import torch
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.models.value import CNNValue
    from rocalphago_amd.search.distributed import DistributedMCTS
    depth = DIST_GEOMETRY["depth"] if depth is None else depth
    share = DIST_GEOMETRY["master_share"] if master_share is None else master_share
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=filters, layers=layers,
                    device=device, seed=seed)
    val = CNNValue(DEFAULT_FEATURES + ["color"], board=19, filters_per_layer=filters,
                   layers=layers, device=device, seed=seed + 1)
    kw = {} if rollout_group is None else {"rollout_group": int(rollout_group)}
    mc = DistributedMCTS(pol, val, dp=dp, lmbda=lmbda, batch=batch, nthreads=nthreads,
                         rollouts_per_leaf=rollouts_per_leaf, seed=seed, depth=depth,
                         master_share=share, force_master=True, **kw)
    st = GameState()
    mc.n_playout = warmup
    mv = mc.get_move(st)  # compiles / allocates; the tree is discarded below
    mc._search = None
    mc.n_playout = playouts
    mc.stats = {"waves": 0, "sims": 0}
    mc.leaves_per_rank[:] = 0
    torch.cuda.synchronize()
    dp.barrier()
    t0 = time.perf_counter()
    for _ in range(moves):
        mv = mc.get_move(st)
        st.do_move(mv)
        mc.update_with_move(mv)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dp.rank != 0:
        return None
    s = mc.stats
    m = mc.master_stats
    out = {"sims_per_s": s["sims"] / dt, "sims": s["sims"], "seconds": dt, "waves": s["waves"],
           "batch": batch, "depth": depth, "master_share": share, "nslots": mc.nslots,
           "rollouts_per_leaf": rollouts_per_leaf, "rollout_device": "gpu", "gpus": dp.world,
           "leaves_per_rank": [int(c) for c in mc.leaf_counts()], "mode": "master",
           "duplication": 1.0, "max_leaves_in_flight": int(m.get("max_inflight", 0))}
    if lmbda > 0:
        out["rollouts_per_s"] = s["sims"] * rollouts_per_leaf / dt
    # rank 0's master-loop split (csrc/mcts/master.hpp run_master)
    for k in ("t_select", "t_ship", "t_value", "t_rollout", "t_idle"):
        out[k + "_frac"] = round(s.get(k, 0.0) / dt, 3)
    return out


def _measure_shared(dp, device, playouts, warmup, moves, filters, layers, batch,
                    rollouts_per_leaf, lmbda, nthreads, seed):
    import torch
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.models.value import CNNValue
    from rocalphago_amd.search.distributed import SharedRootMCTS
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=filters, layers=layers,
                    device=device, seed=seed)
    val = CNNValue(DEFAULT_FEATURES + ["color"], board=19, filters_per_layer=filters,
                   layers=layers, device=device, seed=seed + 1)
    gpu = device.type == "cuda"
    mc = SharedRootMCTS(pol, val, dp=dp, lmbda=lmbda, batch=batch, nthreads=nthreads,
                        rollout_device="gpu" if gpu else "cpu",
                        rollouts_per_leaf=rollouts_per_leaf, seed=seed, pipeline=3)
    st = GameState()
    mc.search(st, warmup * dp.world)  # compiles / allocates; the tree is discarded below
    mc._search = None
    mc.stats = {"waves": 0, "sims": 0}
    if gpu:
        torch.cuda.synchronize()
    dp.barrier()
    t0 = time.perf_counter()
    for _ in range(moves):
        mc.n_playout = playouts
        mv = mc.get_move(st)
        st.do_move(mv)
        mc.update_with_move(mv)
    if gpu:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    s = mc.stats
    # duplication of the ranks' trees (same move-path = same node): all expanded nodes over the
    # distinct ones, on the trees of the last move's search
    keys = mc._search.expanded_keys() if mc._search is not None else []
    dup = 1.0
    if dp.world > 1:
        import torch.distributed as dist
        allk = [None] * dp.world
        dist.all_gather_object(allk, [int(k) for k in keys])
        flat = [k for ks in allk for k in ks]
        dup = len(flat) / max(1, len(set(flat)))
    t = torch.tensor([float(s["sims"]), dt, float(mc.exchanges)], dtype=torch.float64,
                     device=device if dp.backend != "gloo" else "cpu")
    if dp.world > 1:
        import torch.distributed as dist
        per = [torch.zeros_like(t) for _ in range(dp.world)]
        dist.all_gather(per, t)
        per = [p.cpu().numpy() for p in per]
    else:
        per = [t.cpu().numpy()]
    if dp.rank != 0:
        return None
    tot = sum(p[0] for p in per)
    dtm = max(p[1] for p in per)
    out = {"sims_per_s": tot / dtm, "sims": int(tot), "seconds": dtm, "batch": batch,
           "rollouts_per_leaf": rollouts_per_leaf, "rollout_device": mc.rollout_device,
           "gpus": dp.world, "mode": "shared", "duplication": round(dup, 3),
           "leaves_per_rank": [int(p[0]) for p in per],
           "root_exchanges_per_rank": [int(p[2]) for p in per]}
    if lmbda > 0:
        out["rollouts_per_s"] = tot * rollouts_per_leaf / dtm
    for k in ("t_select", "t_submit", "t_eval", "t_backup"):
        out[k + "_frac"] = round(s.get(k, 0.0) / dt, 3)
    return out


def measure_sims_per_s(device, **kw):
    return measure(device, **kw)["sims_per_s"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--playouts", type=int, default=8192)
    ap.add_argument("--batch", type=int, default=None,
                    help="leaves per wave (default: 512 on one GPU -- with pipeline 3 measured "
                         "best, profiles/mcts_sweep_r2.txt -- and distributed_wave(N) per GPU "
                         "with --distributed)")
    ap.add_argument("--rollout-device", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--rollouts-per-leaf", type=int, default=1,
                    help="playouts per leaf (1 = AlphaGo's APV-MCTS: one rollout per simulation)")
    ap.add_argument("--lmbda", type=float, default=0.5)
    ap.add_argument("--filters", type=int, default=192)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--pipeline", type=int, default=3, help="waves in flight (1 = serial)")
    ap.add_argument("--max-inflight", type=int, default=8, help="rollout waves in flight")
    ap.add_argument("--rollout-group", type=int, default=8, help="waves per rollout launch")
    ap.add_argument("--dist-rollout-group", type=int, default=None,
                    help="--distributed: waves per rollout launch on each serving GPU "
                         "(default DistributedMCTS's)")
    ap.add_argument("--moves", type=int, default=1)
    ap.add_argument("--eval-priority", type=int, default=None,
                    help="stream priority of the wave passes (e.g. -1: above the rollouts)")
    ap.add_argument("--rollout-priority", type=int, default=None,
                    help="stream priority of the GPU rollouts")
    ap.add_argument("--rollout-slice", type=int, default=None,
                    help="moves per GPU rollout launch (0: one launch per playout; default "
                         "search/gpu_rollout.DEFAULT_SLICE)")
    ap.add_argument("--depth", type=int, default=None,
                    help="--distributed: waves per GPU awaiting values (default DIST_GEOMETRY)")
    ap.add_argument("--master-share", type=float, default=None,
                    help="--distributed: rank 0's wave relative to the others'")
    ap.add_argument("--distributed", action="store_true",
                    help="one search over all torchrun ranks (search/distributed.py)")
    ap.add_argument("--mode", default="master", choices=["shared", "master"],
                    help="--distributed: one tree on rank 0 (default) or shared root statistics")
    args = ap.parse_args()
    import torch
    from rocalphago_amd.search import apv, gpu_rollout
    if args.rollout_slice is not None:
        gpu_rollout.DEFAULT_SLICE = args.rollout_slice
    if args.eval_priority is not None:
        apv.ParallelMCTS.eval_priority = args.eval_priority
    if args.rollout_priority is not None:
        gpu_rollout.DEFAULT_PRIORITY = args.rollout_priority
    if args.distributed:
        from rocalphago_amd.parallel.dp import DPContext
        dp = DPContext()
        r = measure_distributed(dp, dp.device, playouts=args.playouts,
                                batch=distributed_wave(dp.world, args.mode)
                                if args.batch is None else args.batch,
                                moves=args.moves, rollouts_per_leaf=args.rollouts_per_leaf,
                                lmbda=args.lmbda, filters=args.filters, nthreads=args.threads,
                                mode=args.mode, depth=args.depth,
                                master_share=args.master_share,
                                rollout_group=args.dist_rollout_group)
        if r is not None:
            r.update({"metric": "MCTS simulations/s (19x19 APV-MCTS, one search over %d GPUs)"
                      % dp.world, "lmbda": args.lmbda})
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v)
                              for k, v in r.items()}))
        dp.shutdown()
        return
    dev = torch.device("cuda")
    r = measure(dev, playouts=args.playouts, batch=args.batch or 512, moves=args.moves,
                rollout_device=args.rollout_device, rollouts_per_leaf=args.rollouts_per_leaf,
                lmbda=args.lmbda, filters=args.filters, nthreads=args.threads,
                pipeline=args.pipeline, max_inflight=args.max_inflight,
                rollout_group=args.rollout_group)
    r["pipeline"] = args.pipeline
    r.update({"metric": "MCTS simulations/s (19x19 APV-MCTS, policy+value on GPU)",
              "model": "policy 48x192x13 + value 49x192x13+FC256", "lmbda": args.lmbda})
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
