"""Host ceiling of the APV-MCTS tree: the search driven by a *null evaluator* —
constant priors over the sensible moves and constant values returned instantly — so that the
measured simulations/s is what the host-side tree work alone (selection with virtual loss, leaf
board construction, leaf packing, expansion and backup) can sustain. No GPU is used.

  python benchmarks/mcts_null_bench.py [--playouts 65536] [--batch 512] [--threads 16]
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      benchmarks/mcts_null_bench.py --distributed --threads 4

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

    def sensible(self, boards):
        sfid = [self.rg.FEATURE_IDS["sensibleness"]] if hasattr(self.rg, "FEATURE_IDS") else [9]
        return self.rg.batch_features(boards, sfid, self.nthreads).reshape(len(boards), -1)

    def __call__(self, boards):
        t = time.perf_counter()
        n = len(boards)
        pri = np.broadcast_to(self.prior_row, (n, self.P))
        sens = self.sensible(boards)
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--playouts", type=int, default=65536)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--lmbda", type=float, default=0.5)
    ap.add_argument("--pack", type=int, default=1, help="also build the GPU input arrays")
    ap.add_argument("--distributed", action="store_true")
    args = ap.parse_args()
    if args.distributed:
        run_distributed(args)
        return
    run_single(args)


if __name__ == "__main__":
    main()
