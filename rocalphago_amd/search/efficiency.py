"""Is the multi-GPU search one search? (VERDICT r3 missing #1)

The reference accumulates every playout into one root of one tree
(/root/reference/AlphaGo/mcts.py:191-206) and leaves ``ParallelMCTS`` a stub (:219-220). An
N-rank search with a total budget of T playouts is only worth N GPUs if it finds what one tree
with T playouts finds. This module measures that, on the CPU with a deterministic evaluator
(fixed random-init policy and value networks, value-only leaves or — lmbda > 0 — rollouts
seeded by the leaf position, so every design plays the same rollout from a given leaf), so that
the only difference between two searches is how the work is split:

* ``truth``: one tree with ``truth_mult`` x the largest budget;
* the single-tree ladder: one tree with t, 2t, 4t, ... playouts (t = one rank's share);
* the N-rank search under test with T = N t playouts in total (``SharedRootMCTS`` or any other
  ``search_cls``), one gloo process per rank.

Per configuration over many positions: best-move agreement with the truth, KL(truth || root
visits) with +0.5 smoothing, and for the N-rank searches the duplication — the expanded nodes of
all ranks' trees over the distinct ones (1.0 = the ranks never expanded the same node; the keys
are move-path hashes, ``Search.expanded_keys``). The *budget efficiency* is T_eq / T, where T_eq
is the single-tree budget with the same mean KL (log-linear interpolation on the ladder): 1.0
means the N-rank search is as good as one tree with all N ranks' playouts, 1/N that it is no
better than one rank alone.
"""
import os
import socket

import numpy as np

FEATS = ["board", "ones", "turns_since", "liberties", "capture_size", "sensibleness"]
NET_ARCH = {"filters": 16, "layers": 3, "features": FEATS}
# bump when a change to the search / rollouts changes the single trees (cached truth + ladder)
CACHE_VERSION = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def positions(n, size=9, seed=0, min_moves=4, max_moves=30):
    """``n`` positions reached by random legal non-eye-filling moves from the empty board."""
    from ..engine.gamestate import GameState
    rng = np.random.RandomState(seed)
    out = []
    while len(out) < n:
        st = GameState(size=size)
        k = rng.randint(min_moves, max_moves + 1)
        for _ in range(k):
            moves = st.get_legal_moves(include_eyes=False)
            if not moves:
                break
            st.do_move(moves[rng.randint(len(moves))])
        if not st.is_end_of_game and st.get_legal_moves(include_eyes=False):
            out.append(st)
    return out


def nets(size, seed=3, filters=NET_ARCH["filters"], layers=NET_ARCH["layers"]):
    import torch
    from ..models.policy import CNNPolicy
    from ..models.value import CNNValue
    torch.set_num_threads(1)
    pol = CNNPolicy(FEATS, board=size, filters_per_layer=filters, layers=layers, device="cpu",
                    seed=seed)
    val = CNNValue(FEATS + ["color"], board=size, filters_per_layer=filters, layers=layers,
                   device="cpu", seed=seed + 1)
    return pol, val


def _search_kw(batch, lmbda=0.0):
    """Search settings of every tree in the study; lmbda > 0 adds native CPU rollouts (one per
    leaf, AlphaGo's mixing V = (1 - lmbda) v + lmbda z, as the bench's search)."""
    return dict(lmbda=lmbda, batch=batch, nthreads=1, pipeline=1, c_puct=5.0, virtual_loss=3,
                rollout_limit=200)


def shipped_waves(per_rank, world, bench_budget=8192, bench_wave=512, bench_min=128, cap=False):
    """(single-tree wave, per-rank wave at N = world) of the bench's geometry scaled to a study
    budget: the bench searches 8192 playouts per GPU per move with 512-leaf waves on one GPU and
    max(128, 512 / N) leaves per GPU wave on N GPUs (benchmarks/mcts_bench.py distributed_wave,
    round 6; max(64, 512 / N) in round 5); the study keeps the same leaves-in-flight to budget
    ratios."""
    w1 = max(1, int(round(per_rank * bench_wave / bench_budget)))
    wmin = max(1, int(round(per_rank * bench_min / bench_budget)))
    if cap:  # the round's leaves capped at the one-GPU wave (no per-GPU minimum)
        return w1, max(1, w1 // world)
    return w1, max(wmin, w1 // world)


def root_visits(s, P):
    """Visits of every root child as a dense [P + 1] vector (index P = pass)."""
    mv, vis, _, _ = s.root_stats()
    v = np.zeros(P + 1, np.float64)
    for m, n in zip(mv, vis):
        v[P if m < 0 else m] += n
    return v


def single_tree(pol, val, states, budget, batch, lmbda=0.0, seed=1):
    """Root visit vectors and expanded-node counts of one tree per state."""
    from .apv import ParallelMCTS
    out, nodes = [], []
    for st in states:
        mc = ParallelMCTS(pol, val, n_playout=budget, seed=seed, **_search_kw(batch, lmbda))
        mc.keyed_rollouts = True
        s = mc.search(st, budget)
        out.append(root_visits(s, st.size * st.size))
        nodes.append(len(s.expanded_keys()))
    return np.array(out), np.array(nodes)


def _rank_worker(rank, world, port, outdir, cfg):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from ..parallel.dp import DPContext
    from . import distributed
    dp = DPContext(device="cpu")
    cls = getattr(distributed, cfg["search_cls"])
    pol, val = nets(cfg["size"], cfg["net_seed"])
    states = positions(cfg["n_positions"], cfg["size"], cfg["pos_seed"])
    vis, keys, offs = [], [], [0]
    master = cfg["search_cls"] == "DistributedMCTS"
    for st in states:
        kw = _search_kw(cfg["batch"], cfg.get("lmbda", 0.0))
        if master:
            kw["rollout_delay"] = cfg.get("rollout_delay", 0)
            kw["depth"] = cfg.get("depth", 1)
            kw["force_master"] = True
        mc = cls(pol, val, dp=dp, n_playout=cfg["total"], **kw)
        mc.keyed_rollouts = True
        if master:
            # the GPU pipeline's leaves in flight, deterministically (DistributedMCTS doc)
            mc.emulate_latency = True
            mc.idle_us = 20000
        P = st.size * st.size
        if master and rank > 0:
            mc.serve()  # evaluates rank 0's waves until it stops
            vis.append(np.zeros(P + 1))
            k = np.zeros(0, np.uint64)
        else:
            s = mc.search(st, cfg["total"])
            if master:
                mc.stop()
            vis.append(root_visits(s, P))
            k = s.expanded_keys()
        keys.append(k)
        offs.append(offs[-1] + len(k))
    np.savez(os.path.join(outdir, "rank%d.npz" % rank), visits=np.array(vis),
             keys=np.concatenate(keys) if keys else np.zeros(0, np.uint64), offs=np.array(offs))
    dp.shutdown()


def multi_rank(world, total, cfg, outdir):
    """Run the N-rank search on every position (gloo, one process per rank); returns the summed
    root visits [n, P+1] and the duplication (all expanded nodes / distinct nodes) per position."""
    import torch.multiprocessing as mp
    cfg = dict(cfg, total=int(total))
    mp.spawn(_rank_worker, args=(world, _port(), outdir, cfg), nprocs=world, join=True)
    per = [np.load(os.path.join(outdir, "rank%d.npz" % r)) for r in range(world)]
    vis = sum(p["visits"] for p in per)
    dup = []
    for i in range(vis.shape[0]):
        ks = [p["keys"][p["offs"][i]:p["offs"][i + 1]] for p in per]
        allk = np.concatenate(ks)
        dup.append(len(allk) / max(1, len(np.unique(allk))))
    return vis, np.array(dup)


def kl(truth, x):
    """Mean over positions of KL(truth || x) between root-visit distributions (+0.5 smoothing
    on the truth's legal children)."""
    out = []
    for t, v in zip(truth, x):
        legal = t > 0
        legal |= v > 0
        p = (t[legal] + 0.5) / (t[legal] + 0.5).sum()
        q = (v[legal] + 0.5) / (v[legal] + 0.5).sum()
        out.append(float((p * np.log(p / q)).sum()))
    return float(np.mean(out))


def js(truth, x):
    """Mean over positions of the Jensen-Shannon divergence between root-visit distributions
    (+0.5 smoothing on either's children). Symmetric: unlike KL(truth || x) it does not reward a
    search for spreading visits thinly (virtual loss flattens the visits of wide searches)."""
    out = []
    for t, v in zip(truth, x):
        legal = (t > 0) | (v > 0)
        p = (t[legal] + 0.5) / (t[legal] + 0.5).sum()
        q = (v[legal] + 0.5) / (v[legal] + 0.5).sum()
        m = 0.5 * (p + q)
        out.append(float(0.5 * (p * np.log(p / m)).sum() + 0.5 * (q * np.log(q / m)).sum()))
    return float(np.mean(out))


def agreement(truth, x):
    return float(np.mean([np.argmax(t) == np.argmax(v) for t, v in zip(truth, x)]))


def equivalent_budget(ladder, k):
    """Single-tree budget with mean KL ``k`` by log-linear interpolation over ``ladder``
    [(budget, kl)] (budgets ascending); clamped to the ladder's ends."""
    b = np.log2([x[0] for x in ladder])
    y = np.array([x[1] for x in ladder])
    if k >= y[0]:
        return float(2 ** b[0])
    if k <= y[-1]:
        return float(2 ** b[-1])
    for i in range(len(y) - 1):
        if y[i] >= k >= y[i + 1]:
            f = (y[i] - k) / max(y[i] - y[i + 1], 1e-12)
            return float(2 ** (b[i] + f * (b[i + 1] - b[i])))
    # non-monotone ladder: nearest point
    return float(2 ** b[int(np.argmin(np.abs(y - k)))])


def study(worlds=(2, 4, 8), per_rank=128, batch=16, n_positions=50, size=9, truth_mult=4,
          search_cls="SharedRootMCTS", outdir="/tmp/rag_eff", pos_seed=0, net_seed=3,
          ladder_top=None, split_wave=False, lmbda=0.0, rollout_delay=0, shipped=False,
          capped=False, depth=1, wave=None, metric="kl", ladder=None):
    """The whole comparison; returns a JSON-able dict. ``split_wave``: the N-rank search's
    per-rank wave is batch / N (the job keeps the one-GPU search's leaves in flight per round
    instead of N times as many). ``shipped``: the bench's geometry instead (shipped_waves: the
    single trees' wave and the per-rank waves scaled from the 19x19 bench; ``batch`` ignored),
    normally with ``lmbda`` 0.5 and ``rollout_delay`` 6 as the bench runs it.
    ``metric``: "kl" (KL(truth || visits)) or "js" (Jensen-Shannon, symmetric) for the
    equivalent-budget interpolation (both are reported). ``ladder``: None (single trees, one
    wave in flight) or {"depth": d, "rollout_delay": r}: the ladder is the one-tree search on ONE
    rank at the single-GPU geometry (wave, d waves awaiting values, rollouts returned r waves
    later), so the efficiency compares N GPUs with one GPU searching N times as long."""
    dist_fn = js if metric == "js" else kl
    os.makedirs(outdir, exist_ok=True)
    pol, val = nets(size, net_seed)
    states = positions(n_positions, size, pos_seed)
    if shipped:
        batch = shipped_waves(per_rank, 1)[0]
    top = ladder_top or per_rank * max(worlds)
    truth_budget = per_rank * max(worlds) * truth_mult  # (not scaled by a longer ladder)
    # the single trees (truth and ladder) depend only on these: cached across studies that vary
    # the N-rank search alone (e.g. its rollout delay)
    # (keyed by every setting of those trees — search parameters, networks, positions — and a
    # version tag bumped whenever the search or rollout code changes what a tree finds)
    import hashlib
    import json
    key = json.dumps({"v": CACHE_VERSION, "search": _search_kw(batch, lmbda), "nets": NET_ARCH,
                      "n": n_positions, "size": size, "pos_seed": pos_seed,
                      "net_seed": net_seed, "truth": truth_budget, "per_rank": per_rank},
                     sort_keys=True)
    ck = os.path.join(outdir, "single_%s.npz" % hashlib.sha1(key.encode()).hexdigest()[:16])
    cache = dict(np.load(ck)) if os.path.exists(ck) else {}

    def single(budget, seed=1):
        key = "b%d" % budget
        if key not in cache:
            v, nodes = single_tree(pol, val, states, budget, batch, lmbda, seed=seed)
            cache[key], cache[key + "_n"] = v, nodes
            np.savez(ck, **cache)
        return cache[key], cache[key + "_n"]

    truth, truth_nodes = single(truth_budget, seed=99)
    cfg = {"size": size, "net_seed": net_seed, "pos_seed": pos_seed,
           "n_positions": n_positions, "batch": batch, "search_cls": search_cls,
           "lmbda": lmbda, "rollout_delay": rollout_delay, "depth": depth}

    def one_gpu(budget):  # the ladder on one rank at the single-GPU geometry (cached)
        key = "g%d_d%d_r%d" % (budget, ladder["depth"], ladder["rollout_delay"])
        if key not in cache:
            d = os.path.join(outdir, "ladder_%s" % key)
            os.makedirs(d, exist_ok=True)
            lcfg = dict(cfg, search_cls="DistributedMCTS", depth=ladder["depth"],
                        rollout_delay=ladder["rollout_delay"])
            v, _ = multi_rank(1, budget, lcfg, d)
            cache[key], cache[key + "_n"] = v, np.full(len(v), float(budget))
            np.savez(ck, **cache)
        return cache[key], cache[key + "_n"]

    ladder_pts, rows = [], {}
    b = per_rank
    while b <= top:
        v, nodes = single(b) if ladder is None else one_gpu(b)
        k = dist_fn(truth, v)
        ladder_pts.append((b, k))
        rows["single_%d" % b] = {"budget": b, "kl": round(kl(truth, v), 4),
                                 "js": round(js(truth, v), 5),
                                 "agree": round(agreement(truth, v), 3),
                                 "nodes": float(nodes.mean())}
        b *= 2
    for w in worlds:
        d = os.path.join(outdir, "%s_w%d" % (search_cls, w))
        os.makedirs(d, exist_ok=True)
        if wave is not None:  # an explicit per-rank wave (the effective-throughput sweep)
            wcfg = dict(cfg, batch=int(wave))
        elif shipped:
            wcfg = dict(cfg, batch=shipped_waves(per_rank, w, cap=capped)[1])
        else:
            wcfg = dict(cfg, batch=max(1, batch // w)) if split_wave else cfg
        vis, dup = multi_rank(w, per_rank * w, wcfg, d)
        teq = equivalent_budget(ladder_pts, dist_fn(truth, vis))
        rows["%s_%d" % (search_cls, w)] = {
            "ranks": w, "budget": per_rank * w, "kl": round(kl(truth, vis), 4),
            "js": round(js(truth, vis), 5),
            "wave_per_rank": wcfg["batch"], "depth": depth, "rollout_delay": rollout_delay,
            "agree": round(agreement(truth, vis), 3), "duplication": round(float(dup.mean()), 3),
            "equivalent_single_tree_budget": round(teq, 1),
            "efficiency": round(teq / (per_rank * w), 3)}
    return {"positions": n_positions, "board": size, "per_rank_playouts": per_rank,
            "wave": batch, "truth_budget": truth_budget, "search": search_cls,
            "lmbda": lmbda, "rollout_delay": rollout_delay, "shipped_geometry": bool(shipped),
            "capped": bool(capped), "metric": metric, "ladder": ladder or "single trees",
            "truth_nodes": float(truth_nodes.mean()), "rows": rows}
