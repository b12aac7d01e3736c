"""Host ceiling of the APV-MCTS tree: the search driven by a *null evaluator* —
constant priors over the sensible moves and constant values returned instantly — so that the
measured simulations/s is what the host-side tree work alone (selection with virtual loss, leaf
board construction, leaf packing, expansion and backup) can sustain. No GPU is used.

  python benchmarks/mcts_null_bench.py [--playouts 65536] [--batch 512] [--threads 16]
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      benchmarks/mcts_null_bench.py --distributed --threads 4
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
      benchmarks/mcts_null_bench.py --distributed --mode master --batch 512 --threads 2
  python benchmarks/mcts_null_bench.py --distributed --mode master    (one process: N = 1)

Single process: one JSON line with sims/s and the per-phase split (select, pack, eval = the
null evaluator itself, backup). ``--distributed`` (gloo, CPU): the shared-root multi-rank search
of search/distributed.py with the null evaluator on every rank and no rollouts — the aggregate
rate the ranks' host work plus the per-wave root all-reduce sustain, i.e. the host ceiling of
the N-GPU search.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class NullEvaluator(object):
    """Evaluator with the NetworkEvaluator call shape: (priors [n, P], values [n], sensible
    [n, P]) for native boards. The sensible mask is exact (legal, not an own eye: the children
    the real search creates), priors are a fixed random vector, values 0."""

    def __init__(self, size=19, nthreads=8, seed=0):
        from rocalphago_amd._native import engine
        self.rg = engine()
        self.P = size * size
        self.nthreads = nthreads
        r = np.random.RandomState(seed).rand(self.P).astype(np.float32) + 0.05
        self.prior_row = r / r.sum()
        self.policy = self  # "has a policy" for the search's bookkeeping
        self.value = None
        self.shared = False
        self._sens_off = 0
        self.t_eval = 0.0

    def _plans(self):
        return None

    delay = 0.0  # seconds per call: a stand-in for the GPU pass of a wave (--eval-ms)

    def sensible(self, boards):
        sfid = [self.rg.FEATURE_IDS["sensibleness"]] if hasattr(self.rg, "FEATURE_IDS") else [9]
        return self.rg.batch_features(boards, sfid, self.nthreads).reshape(len(boards), -1)

    def __call__(self, boards):
        t = time.perf_counter()
        n = len(boards)
        pri = np.broadcast_to(self.prior_row, (n, self.P))
        sens = self.sensible(boards)
        if self.delay > 0:
            rest = self.delay - (time.perf_counter() - t)
            if rest > 0:
                time.sleep(rest)
        self.t_eval += time.perf_counter() - t
        return np.ascontiguousarray(pri), np.zeros(n, np.float32), sens


def run_single(args):
    from rocalphago_amd._native import engine
    from rocalphago_amd.engine.gamestate import GameState
    rg = engine()
    st = GameState()
    ev = NullEvaluator(nthreads=args.threads)
    s = rg.Search(st.native, args.threads)
    s.lmbda = args.lmbda
    s.c_puct = 5.0
    s.n_vl = 3
    target = args.playouts
    t_sel = t_pack = t_eval = t_back = 0.0
    P = 361
    t0 = time.perf_counter()
    waves = 0
    while s.root_visits < target:
        a = time.perf_counter()
        wid, n = s.select(min(args.batch, target - s.root_visits))
        b = time.perf_counter()
        if n == 0:
            break
        boards = s.leaf_boards(wid)
        if args.pack:
            rg.gpu_feature_inputs(boards, False, args.threads)
            if args.lmbda > 0:
                s.rollout_inputs(wid)
        c = time.perf_counter()
        pri, val, sens = ev(boards)
        d = time.perf_counter()
        s.backup_value(wid, pri, val, sens)
        if args.lmbda > 0:
            s.backup_rollout(wid, np.zeros(n, np.float32))
        e = time.perf_counter()
        t_sel += b - a
        t_pack += c - b
        t_eval += d - c
        t_back += e - d
        waves += 1
    dt = time.perf_counter() - t0
    sims = s.sims
    host = dt - t_eval
    out = {"metric": "MCTS host ceiling (null evaluator), 19x19", "sims": sims,
           "sims_per_s_incl_eval": round(sims / dt, 1),
           "sims_per_s_host": round(sims / host, 1), "waves": waves, "batch": args.batch,
           "threads": args.threads, "nodes": s.num_nodes, "collisions_last": s.collisions,
           "us_per_sim": {"select": round(t_sel / sims * 1e6, 3),
                          "pack": round(t_pack / sims * 1e6, 3),
                          "null_eval": round(t_eval / sims * 1e6, 3),
                          "backup": round(t_back / sims * 1e6, 3)}}
    print(json.dumps(out))
    _ = P


def run_distributed(args):
    """Shared-root search (search/distributed.SharedRootMCTS) on every torchrun rank with the
    null evaluator and no rollouts (lambda 0): what N ranks' host tree work plus the per-wave root
    all-reduce can sustain together, i.e. the host ceiling of the N-GPU search. gloo on CPU."""
    import torch
    import torch.distributed as dist
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.search.distributed import SharedRootMCTS
    dp = DPContext(device="cpu", backend="gloo")
    ev = NullEvaluator(nthreads=args.threads, seed=dp.rank)
    mc = SharedRootMCTS(None, value=True, evaluator=ev, dp=dp, lmbda=0.0, batch=args.batch,
                        nthreads=args.threads, pipeline=1, n_playout=args.playouts)
    st = GameState()
    mc.search(st, 4 * args.batch * dp.world)  # warm-up; a fresh tree below
    mc._search = None
    dp.barrier()
    t0 = time.perf_counter()
    s = mc.search(st, args.playouts)
    dt = time.perf_counter() - t0
    t = torch.tensor([float(s.sims), dt, float(mc.exchanges)], dtype=torch.float64)
    per = [torch.zeros_like(t) for _ in range(dp.world)]
    if dp.enabled:
        dist.all_gather(per, t)
    else:
        per = [t]
    if dp.rank == 0:
        sims = sum(int(p[0]) for p in per)
        wall = max(float(p[1]) for p in per)
        print(json.dumps({
            "metric": "MCTS host ceiling, shared-root N-rank search (null evaluator, gloo), 19x19",
            "ranks": dp.world, "threads_per_rank": args.threads, "batch": args.batch,
            "sims": sims, "seconds": round(wall, 3), "sims_per_s": round(sims / wall, 1),
            "sims_per_s_per_rank": round(sims / wall / dp.world, 1),
            "exchanges_rank0": int(per[0][2]), "playouts_per_move": args.playouts}), flush=True)
    if dp.enabled:
        dp.shutdown()


def run_master(args):
    """DistributedMCTS (search/distributed.py, the multi-GPU bench's search) with the null
    evaluator and null rollouts on every rank: ONE tree on rank 0 whose native master loop
    (csrc/mcts/master.hpp) ships waves of ``--batch`` leaves per rank as move paths through the
    shared-memory channel; every rank (rank 0 on a second thread, ``--master-share``) replays
    them, "evaluates" them and answers. Rank 0's sims/s is the host ceiling of the N-GPU search,
    its split (select / ship / value backup / rollout backup / idle, fractions of its wall time)
    says what bounds it. ``--eval-ms``: a fixed evaluation time per wave on every rank (the GPU
    pass it stands for). gloo only for the set-up (torchrun, 127.0.0.1)."""
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.search.distributed import DistributedMCTS
    dp = DPContext(device="cpu", backend="gloo")
    # rank 0 owns the tree: on a real node every rank has its own cores, so the master may get
    # more host threads than the evaluating ranks (--threads-master)
    nt = args.threads_master if dp.rank == 0 and args.threads_master else args.threads
    ev = NullEvaluator(nthreads=args.threads, seed=dp.rank)
    ev.delay = args.eval_ms * 1e-3
    mc = DistributedMCTS(None, value=True, evaluator=ev, dp=dp, lmbda=args.lmbda,
                         batch=args.batch, nthreads=nt, depth=args.depth,
                         rollout_slots=args.rollout_slots, master_share=args.master_share,
                         board=19, force_master=True, worker_threads=args.threads)
    mc.worker_rollouts = "null"
    st = GameState()
    mc.n_playout = 4 * args.batch * dp.world
    mc.get_move(st)  # warm-up (arenas, pools); a fresh tree below
    mc._search = None
    mc.stats = {"waves": 0, "sims": 0}
    mc.leaves_per_rank[:] = 0
    mc.n_playout = args.playouts
    dp.barrier()
    t0 = time.perf_counter()
    if dp.rank == 0:
        s = mc.search(st)
        dt = time.perf_counter() - t0
        mc.stop()
        m = mc.master_stats
        keys = ("t_select", "t_ship", "t_value", "t_rollout", "t_idle")
        busy = sum(m[k] for k in keys[:4])
        out = {"metric": "DistributedMCTS host ceiling (native master loop + shared-memory "
                         "channel; null evaluator + null rollouts), 19x19",
               "ranks": dp.world, "threads_master": nt, "threads_per_rank": args.threads,
               "batch_per_rank": args.batch, "master_share": args.master_share,
               "depth": args.depth, "nslots": mc.nslots, "lmbda": args.lmbda,
               "eval_ms_per_wave": args.eval_ms, "sims": int(m["sims"]),
               "seconds": round(dt, 3), "sims_per_s": round(m["sims"] / dt, 1),
               "waves": int(m["waves"]), "max_leaves_in_flight": int(m["max_inflight"]),
               "us_per_sim": {k[2:]: round(m[k] / max(1, m["sims"]) * 1e6, 3) for k in keys},
               # rank 0's own tree work per simulation (everything but waiting for the ranks)
               # and the rate it alone would sustain
               "master_busy_us_per_sim": round(busy / max(1, m["sims"]) * 1e6, 3),
               "master_ceiling_sims_per_s": round(m["sims"] / max(busy, 1e-9), 1),
               "frac": {k[2:]: round(m[k] / dt, 3) for k in keys},
               "tree_timers_s": [round(x, 4) for x in s.timers],
               "leaves_per_rank": [int(c) for c in m["leaves"]]}
        print(json.dumps(out), flush=True)
    else:
        mc.serve()
    if dp.enabled:
        dp.shutdown()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--playouts", type=int, default=65536)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--lmbda", type=float, default=0.5)
    ap.add_argument("--pack", type=int, default=1, help="also build the GPU input arrays")
    ap.add_argument("--distributed", action="store_true")
    ap.add_argument("--mode", default="shared", choices=("shared", "master"),
                    help="--distributed: shared-root trees or the one-tree master search")
    ap.add_argument("--eval-ms", type=float, default=0.0,
                    help="master: fixed evaluation time per wave and rank")
    ap.add_argument("--depth", type=int, default=2, help="master: waves per rank awaiting values")
    ap.add_argument("--rollout-slots", type=int, default=6,
                    help="master: further waves per rank holding virtual loss until rollouts")
    ap.add_argument("--master-share", type=float, default=1.0,
                    help="master: rank 0's wave relative to the other ranks' (0: none)")
    ap.add_argument("--threads-master", type=int, default=0,
                    help="master: rank 0's tree threads (default --threads)")
    args = ap.parse_args()
    if args.distributed and args.mode == "master":
        run_master(args)
        return
    if args.distributed:
        run_distributed(args)
        return
    run_single(args)


if __name__ == "__main__":
    main()
