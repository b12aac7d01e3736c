"""Flagship benchmark: SL policy-network training throughput on MI355X.

Metric (BASELINE.json): positions/sec of SL-policy training on 19x19 — the north-star policy net
(48 feature planes, 5x5 + 11 x 3x3 convs at 192 filters + 1x1 head + per-position bias + softmax,
3,882,794 params), bf16 compute on the hand-written gfx950 kernels, synthetic device-resident
positions with random dihedral augmentation, random-init weights, full SGD step (forward, fused
softmax cross-entropy, backward, RCCL gradient all-reduce for N>1, fused SGD update) in the timed
region. Weak scaling: fixed per-GPU batch.

  python bench.py --gpus N --steps K --warmup W        (N>1: launched under torchrun)

Rank 0 prints ONE JSON line; value = whole-job positions/s (max step time over ranks).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PAPER_SL_POSITIONS_PER_S = 3000.0  # paper-derived SL throughput (50 GPUs)
PAPER_VALUE_POSITIONS_PER_S = 2600.0  # paper-derived value-net throughput


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def allreduce_probe(dp, dev, nbytes=15531176, reps=10):
    """One timed all-reduce of the north-star gradient size (3,882,794 fp32 = 15.5 MB) over the
    job's process group before the SL phase: the RCCL bandwidth the bucketed gradient all-reduce
    can get (busbw = 2 (N-1)/N x bytes / time, the ring's per-rank traffic rate)."""
    import torch
    import torch.distributed as dist
    buf = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
    for _ in range(2):
        dist.all_reduce(buf)
    torch.cuda.synchronize()
    dp.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_reduce(buf)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ok = bool(torch.all(buf == float(dp.world) ** (reps + 2)).item())
    n = dp.world
    return {"comm_ranks": n, "comm_backend": dp.backend,
            "allreduce_bytes": nbytes, "allreduce_us": round(dt * 1e6, 1),
            "allreduce_algbw_GBps": round(nbytes / dt / 1e9, 2),
            "allreduce_busbw_GBps": round(2.0 * (n - 1) / n * nbytes / dt / 1e9, 2),
            "allreduce_ok": ok}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="positions per GPU per step")
    ap.add_argument("--filters", type=int, default=None,
                    help="default 192 (policy/value), 128 (resnet, ResnetPolicy's default)")
    ap.add_argument("--layers", type=int, default=None,
                    help="default 12 (policy/value), 20 (resnet)")
    ap.add_argument("--dataset", type=int, default=65536, help="synthetic positions per GPU")
    ap.add_argument("--model", default="policy", choices=["policy", "value", "resnet"],
                    help="policy: SL policy net (headline); value: value net (BASELINE config 4); "
                         "resnet: ResnetPolicy SL training (batch-statistics BN)")
    ap.add_argument("--no-mcts", action="store_true",
                    help="skip the APV-MCTS sims/s measurement (run after the timed SL steps)")
    ap.add_argument("--mcts-playouts", type=int, default=8192)
    ap.add_argument("--mcts-mode", default="master", choices=["master", "shared"],
                    help="N>1 search: one tree on rank 0 whose leaf waves every GPU serves "
                         "(master), or N trees with shared root statistics (shared; measured "
                         "1/N budget efficiency, kept for comparison)")
    ap.add_argument("--mcts-guard-s", type=int, default=180,
                    help="N>1: wall-clock limit of the multi-GPU search measurement")
    ap.add_argument("--trace", default=None,
                    help="also write a Chrome trace (torch.profiler) of 5 untimed steps here")
    ap.add_argument("--stall-timeout", type=float, default=120.0,
                    help="N>1: a rank without progress for this long prints which rank(s) "
                         "stalled and exits non-zero (parallel/watchdog.py); collectives time "
                         "out shortly after")
    args = ap.parse_args()
    if args.filters is None:
        args.filters = 128 if args.model == "resnet" else 192
    if args.layers is None:
        args.layers = 20 if args.model == "resnet" else 12

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launched by hand: spawn one rank per GPU (child process, no exec)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    if "WORLD_SIZE" in os.environ:
        # a failed / timed-out RCCL collective tears the rank down instead of hanging it
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    import torch

    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.training.data import TRANSFORM_NAMES, DeviceDataset
    from rocalphago_amd.training.supervised import SupervisedTrainer

    from rocalphago_amd.parallel.watchdog import RankWatchdog, inject_stall
    dp = DPContext(timeout_s=int(args.stall_timeout) + 60)
    dev = dp.device
    wd = RankWatchdog(dp.rank, dp.world, args.stall_timeout, phase="setup") \
        if dp.enabled else None
    if dev.type != "cuda":
        raise SystemExit("bench.py needs a GPU")
    comm = allreduce_probe(dp, dev) if dp.enabled else None
    torch.manual_seed(1234)
    gen = torch.Generator(device=dev)
    gen.manual_seed(99 + dp.rank)
    if args.model in ("policy", "resnet"):
        if args.model == "resnet":
            from rocalphago_amd.models.policy import ResnetPolicy
            policy = ResnetPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=args.filters,
                                  layers=args.layers, device=dev, seed=1234)
        else:
            policy = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=args.filters,
                               layers=args.layers, device=dev, seed=1234)
        model = policy.model
        dp.broadcast_model(model)
        model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.003, decay=0.0001),
                      metrics=["accuracy"])
        ds = DeviceDataset.synthetic(args.dataset, 48, 19, dev, seed=17 + dp.rank)
        trainer = SupervisedTrainer(model, ds, args.batch, TRANSFORM_NAMES, dp, seed=5)
        N = ds.N
    else:
        from rocalphago_amd.features.preprocessing import VALUE_FEATURES
        from rocalphago_amd.models.value import CNNValue
        from rocalphago_amd.training.value_trainer import ValueTrainer
        value = CNNValue(VALUE_FEATURES, board=19, filters_per_layer=args.filters,
                         layers=args.layers, device=dev, seed=1234)
        model = value.model
        dp.broadcast_model(model)
        model.compile(loss="mse", optimizer=K.SGD(lr=0.003, decay=8.664339379294006e-08))
        g = torch.Generator(device=dev)
        g.manual_seed(17 + dp.rank)
        N = args.dataset
        states = (torch.rand((N, 49, 19, 19), generator=g, device=dev) < 0.3).to(torch.uint8)
        values = (torch.randint(0, 2, (N, 1), generator=g, device=dev) * 2 - 1).float()
        trainer = ValueTrainer(model, states, values, args.batch, TRANSFORM_NAMES, dp, seed=5)
    nparams = sum(int(w.numel()) for w in model.net._views)
    if trainer.plan is None:
        raise SystemExit("HIP fused plan not active for the %s network" % args.model)

    counter = [0]
    # epoch-shuffled sampling, as the trainers' samplers: one device permutation per pass over the
    # synthetic set, each step a contiguous slice of it (no per-step RNG launch)
    order = {"perm": None, "pos": N}

    def step():
        # heartbeat 2k: step k started; 2k+1: its gradients reached the all-reduce
        k = counter[0]
        counter[0] += 1
        inject_stall(dp.rank, k)  # RAG_STALL=rank:step rehearsal of a hung rank
        if wd is not None:
            wd.beat(2 * k)
        if order["pos"] + args.batch > N:
            order["perm"] = torch.randperm(N, generator=gen, device=dev)
            order["pos"] = 0
        idx = order["perm"][order["pos"]:order["pos"] + args.batch]
        order["pos"] += args.batch
        trainer.step(idx)
        if wd is not None:
            wd.beat(2 * k + 1)

    if wd is not None:
        wd.set_phase("sl-warmup")
    for _ in range(args.warmup):
        step()
    dp.barrier()
    torch.cuda.synchronize()
    if wd is not None:
        wd.set_phase("sl-timed")
        counter[0] = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dp.barrier()
    dt = time.perf_counter() - t0
    # per-rank step time and the number of ranks that reached this point (self-check)
    rank_t = torch.zeros(dp.world, dtype=torch.float64, device=dev)
    rank_t[dp.rank] = dt
    dp.allreduce_sum_(rank_t)
    per_rank_ms = [round(float(x) / args.steps * 1e3, 3) for x in rank_t.cpu()]
    ranks_seen = int((rank_t > 0).sum())
    dt = float(rank_t.max())
    if args.trace:
        # host + device timeline of a few extra (untimed) steps, Chrome-trace JSON
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(5):
                step()
            torch.cuda.synchronize()
        path = args.trace if dp.world == 1 else "%s.rank%d.json" % (args.trace, dp.rank)
        prof.export_chrome_trace(path)
    if args.model in ("policy", "resnet"):
        loss, acc = trainer.pop_metrics()
    else:
        loss = trainer.pop_loss()
    ms = dt / args.steps * 1e3
    value = dp.world * args.batch * args.steps / dt
    result = {
        # BASELINE.json's headline metric; value = the SL-policy training positions/s half
        # (MCTS sims/s is reported alongside, measured after the timed SL region)
        "metric": "positions/sec SL-policy train + MCTS sims/sec (19x19) at 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "positions/s",
        "n_gpus": dp.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / PAPER_SL_POSITIONS_PER_S, 2),
        "dtype": "bf16",
        "data": "synthetic (random 48-plane 19x19 uint8 positions, device-resident, random "
                "dihedral augmentation); random-init weights",
        "config": {"model": "19x19 SL policy net (13 layers, %d filters, 48 planes): 5x5 + "
                            "%dx 3x3 conv + 1x1 head + position bias + softmax, %d params"
                            % (args.filters, args.layers - 1, nparams),
                   "global_batch": args.batch * dp.world, "per_gpu_batch": args.batch,
                   "seq_len": 361, "parallelism": "dp%d" % dp.world},
        "train_loss": round(loss, 4),
        "ranks_seen": ranks_seen,
        "per_rank_ms_per_step": per_rank_ms,
        "baseline_note": "vs_baseline = value / 3000 positions/s (paper-derived SL throughput, "
                         "BASELINE.md; the reference publishes no numbers)",
    }
    if args.model == "value":
        result["metric"] = "positions/sec value-net train (19x19) at 1/2/4/8 MI355X"
        result["vs_baseline"] = round(value / PAPER_VALUE_POSITIONS_PER_S, 2)
        result["data"] = "synthetic (random 49-plane 19x19 uint8 positions, +-1 outcomes, " \
                         "device-resident, random dihedral augmentation); random-init weights"
        result["config"]["model"] = "19x19 value net (49 planes, %d filters, 13 conv layers, " \
                                    "FC256 + tanh, MSE), %d params" % (args.filters, nparams)
        result["baseline_note"] = "vs_baseline = value / 2600 positions/s (paper-derived value " \
                                  "training throughput, BASELINE.md)"
    if args.model == "resnet":
        result["metric"] = "positions/sec ResnetPolicy SL train (19x19) at 1/2/4/8 MI355X"
        result["vs_baseline"] = None
        result["config"]["model"] = "19x19 ResnetPolicy (48 planes, %d filters, %d layers, " \
                                    "column BN + ReLU + residual units), %d params" % (
                                        args.filters, args.layers, nparams)
        result["baseline_note"] = "no published baseline for the residual policy"
    if comm is not None:
        result.update(comm)
    if wd is not None:
        wd.set_phase("mcts", limit_s=max(args.stall_timeout, args.mcts_guard_s + 30))
    if not args.no_mcts and args.model == "policy":
        # N = 1: the pipelined single-GPU search. N > 1: ONE search whose leaf waves are dealt
        # to all N GPUs (search/distributed.py) — the whole job's sims/s is that search's.
        # Every rank reaches the all-reduce whether or not its measurement worked (no hang).
        r, err = None, None
        guard = None
        if dp.world > 1:
            # The SL number is final here. A multi-GPU search that stalls (it was rehearsed on
            # gloo only) must not turn the scaling run into a hang: after MCTS_GUARD_S every rank
            # leaves with status 0 and rank 0 prints the line with an mcts_error instead.
            import threading

            def _expire():
                if dp.is_root:
                    result["mcts_error"] = "multi-GPU search exceeded %ds" % args.mcts_guard_s
                    print(json.dumps(result), flush=True)
                sys.stdout.flush()
                os._exit(0)
            guard = threading.Timer(args.mcts_guard_s, _expire)
            guard.daemon = True
            guard.start()
        try:
            if dp.world > 1:
                # ONE tree (rank 0, native master loop) whose leaf waves every GPU serves through
                # a shared-memory channel (search/distributed.py); its budget efficiency against
                # one tree of the same budget is measured separately by search/efficiency.py
                # (profiles/search_efficiency_r6.json) and not folded into this rate
                from benchmarks.mcts_bench import distributed_wave, measure_distributed
                r = measure_distributed(dp, dev, playouts=args.mcts_playouts * dp.world,
                                        mode=args.mcts_mode,
                                        batch=distributed_wave(dp.world, args.mcts_mode))
                r = r or {"sims_per_s": 0.0, "rollouts_per_s": 0.0}
            else:
                from benchmarks.mcts_bench import measure
                # untimed warmup: 8 waves (allocations, a full 6-wave rollout group); 12 moves timed
                # (~1 s: 4 moves (0.3 s) varied by +-4 % run to run)
                r = measure(dev, playouts=args.mcts_playouts, warmup=4096, moves=12)
        except Exception as e:  # the SL metric stands on its own
            import traceback
            traceback.print_exc()  # on stderr, per rank: the cause of a failed measurement
            err = "rank %d: %s" % (dp.rank, str(e)[:200])
        # explicit dtype: rank 0's numbers are numpy float64 and the others' Python floats, and
        # torch.tensor would infer float64 on one rank and float32 on the rest (a collective
        # mismatch: gloo aborts, RCCL would hang until the guard fired)
        tot = torch.tensor([float(r["sims_per_s"]) if r else 0.0,
                            float(r.get("rollouts_per_s", 0.0)) if r else 0.0,
                            1.0 if r else 0.0], dtype=torch.float64, device=dev)
        dp.allreduce_sum_(tot)
        if guard is not None:
            guard.cancel()
        if int(tot[2]) == dp.world:
            result["mcts_sims_per_s"] = round(float(tot[0]), 1)
            result["mcts_rollouts_per_s"] = round(float(tot[1]), 1)
            result["mcts_config"] = "APV-MCTS 19x19, policy 48x192x13 + value 49x192x13+FC256 " \
                                    "on GPU, lambda 0.5, %d GPU rollouts/leaf, wave %d, %d " \
                                    "playouts/move, %s" % (
                                        r["rollouts_per_leaf"] if "rollouts_per_leaf" in r
                                        else 1, r.get("batch", 512),
                                        args.mcts_playouts * dp.world,
                                        "one tree over %d GPUs" % dp.world if dp.world > 1
                                        else "1 GPU")
            if dp.is_root and "leaves_per_rank" in r:
                result["mcts_leaves_per_rank"] = r["leaves_per_rank"]
            if dp.is_root and dp.world > 1:
                # rank 0's host split of the N-GPU search (fractions of its wall time): the
                # diagnosis of a scale run, not just its rate
                for k, v in r.items():
                    if k.startswith("t_") and k.endswith("_frac"):
                        result["mcts_" + k] = v
                for k in ("waves", "max_leaves_in_flight", "master_share"):
                    if k in r:
                        result["mcts_" + k] = r[k]
            if dp.is_root and dp.world > 1:
                # over-crediting guard: simulations of one tree are all distinct; with N
                # independent trees (mode shared) the duplicated expansions are measured live
                dup = float(r.get("duplication", 1.0))
                result["mcts_mode"] = r.get("mode", args.mcts_mode)
                result["mcts_tree_duplication"] = round(dup, 3)
                result["mcts_unique_sims_per_s"] = round(float(tot[0]) / max(dup, 1.0), 1)
        else:
            result["mcts_error"] = err or "MCTS measurement failed on %d rank(s)" % (
                dp.world - int(tot[2]))
    if dp.is_root:
        print(json.dumps(result), flush=True)
    if wd is not None:
        wd.stop()
    dp.shutdown()


if __name__ == "__main__":
    main()
