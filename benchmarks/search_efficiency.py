"""Budget efficiency of the multi-rank searches (rocalphago_amd/search/efficiency.py): N ranks
(gloo, CPU, deterministic evaluator) with N x t playouts against one tree with t .. N t
playouts, over many positions. One JSON line per search design.

  python benchmarks/search_efficiency.py [--ranks 2 4 8] [--positions 50] [--per-rank 128]
  python benchmarks/search_efficiency.py --designs DistributedMCTS/shipped --per-rank 512 \
      --lmbda 0.5 --rollout-delay 6 --truth-mult 16     (the bench's geometry)
  python benchmarks/search_efficiency.py --effective --per-rank 512 --lmbda 0.5 \
      --rollout-delay 6 --truth-mult 16 --gpu-waves 64 128 256 512 --depths 1 2 \
      --ranks 1 2 4 8 --gpu-rates profiles/mcts_wave_rates_r6.json \
      --master-ceiling 900000 > profiles/search_efficiency_r6.json
      (every per-GPU wave / depth of the one-tree search at N = 1, 2, 4, 8;
       efficiency x the modelled rate min(N x one GPU's rate at that wave, the master's
       ceiling) = effective simulations/s; the argmax per N is the shipped geometry)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--positions", type=int, default=50)
    ap.add_argument("--per-rank", type=int, default=128)
    ap.add_argument("--wave", type=int, default=16)
    ap.add_argument("--board", type=int, default=9)
    ap.add_argument("--designs", nargs="+",
                    default=["SharedRootMCTS", "DistributedMCTS", "DistributedMCTS/split"])
    ap.add_argument("--out", default="/tmp/rag_search_eff")
    ap.add_argument("--lmbda", type=float, default=0.0,
                    help="0.5: rollouts mixed in as the bench's search does")
    ap.add_argument("--rollout-delay", type=int, default=0)
    ap.add_argument("--truth-mult", type=int, default=4)
    ap.add_argument("--effective", action="store_true",
                    help="sweep the one-tree search's per-GPU wave and depth (module doc)")
    ap.add_argument("--gpu-waves", type=int, nargs="+", default=[64, 128, 256, 512],
                    help="--effective: per-GPU waves of the 19x19 bench (8192 playouts per GPU "
                         "per move), scaled to the study's budget")
    ap.add_argument("--depths", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--metric", default="js", choices=["js", "kl"],
                    help="--effective: distance to the truth behind the equivalent budget")
    ap.add_argument("--ladder-top", type=int, default=None,
                    help="--effective: the ladder's largest budget (default the largest N-rank "
                         "budget; larger lets efficiencies above 1 show instead of clamping)")
    ap.add_argument("--ladder-depth", type=int, default=3,
                    help="--effective: the one-GPU yardstick's waves awaiting values (the "
                         "single-GPU bench's pipeline)")
    ap.add_argument("--gpu-rates", default=None,
                    help="--effective: JSON {wave: one GPU's sims/s} measured on MI355X")
    ap.add_argument("--master-ceiling", type=float, default=None,
                    help="--effective: rank 0's host ceiling, sims/s (mcts_null_bench)")
    ap.add_argument("--master-ceilings", default=None,
                    help="--effective: per-wave ceilings 'WAVE:SIMS_PER_S,...' (override "
                         "--master-ceiling for those waves)")
    ap.add_argument("--from-rows", default=None,
                    help="--effective: take the efficiency rows from this earlier output and "
                         "only recompute the modelled / effective rates")
    args = ap.parse_args()
    if args.effective:
        effective(args)
        return
    from rocalphago_amd.search.efficiency import study
    for d in args.designs:
        # design suffixes: /split (per-rank wave = wave / N), /shipped (the bench's geometry:
        # efficiency.shipped_waves), /capped (the same with the round capped at one GPU's wave)
        cls, _, opt = d.partition("/")
        r = study(worlds=tuple(args.ranks), per_rank=args.per_rank, batch=args.wave,
                  n_positions=args.positions, size=args.board, search_cls=cls,
                  outdir=os.path.join(args.out, d.replace("/", "_")), split_wave=opt == "split",
                  shipped=opt in ("shipped", "capped"), capped=opt == "capped",
                  lmbda=args.lmbda, rollout_delay=args.rollout_delay,
                  truth_mult=args.truth_mult)
        r["design"] = d
        print(json.dumps(r), flush=True)


def effective(args):
    """Efficiency of every (per-GPU wave, depth) at every N, then effective simulations/s =
    efficiency x min(N x one GPU's rate at that wave, the master's ceiling)."""
    from rocalphago_amd.search.efficiency import study
    rates = serving = None
    if args.gpu_rates:
        with open(args.gpu_rates) as f:
            js = json.load(f)
        rates = {int(k): float(v) for k, v in js["sims_per_s_by_wave"].items()}
        # one GPU serving the multi-GPU search at (wave, depth), where measured
        serving = {(int(w), int(d)): float(v) for w, dv in js.get("serving_sims_per_s",
                                                                  {}).items()
                   for d, v in dv.items()}
    ceilings = {}
    for item in (args.master_ceilings or "").split(","):
        if item:
            w, v = item.split(":")
            ceilings[int(w)] = float(v)

    def model(row):
        w, d, n = row["gpu_wave"], row["depth"], row["ranks"]
        per_gpu = (serving or {}).get((w, d), (rates or {}).get(w))
        if per_gpu is None:
            return row
        row["per_gpu_sims_per_s"] = per_gpu
        rate = n * per_gpu
        cap = ceilings.get(w, args.master_ceiling)
        if cap:
            row["master_ceiling"] = cap
            rate = min(rate, cap)
        row["modelled_sims_per_s"] = round(rate, 1)
        row["effective_sims_per_s"] = round(rate * row["efficiency"], 1)
        return row

    rows = []
    if args.from_rows:
        with open(args.from_rows) as f:
            txt = f.read()
        prev = json.loads(txt[txt.index("{\n"):] if "{\n" in txt else txt)
        rows = [model(dict(r)) for r in prev["rows"]]
    for w in ([] if args.from_rows else args.gpu_waves):
        sw = max(1, int(round(w * args.per_rank / 8192.0)))  # the study's wave
        for d in args.depths:
            r = study(worlds=tuple(args.ranks), per_rank=args.per_rank,
                      n_positions=args.positions, size=args.board, search_cls="DistributedMCTS",
                      outdir=os.path.join(args.out, "eff"), lmbda=args.lmbda,
                      rollout_delay=args.rollout_delay, truth_mult=args.truth_mult,
                      shipped=True, depth=d, wave=sw, metric=args.metric,
                      ladder={"depth": args.ladder_depth,
                              "rollout_delay": args.rollout_delay},
                      ladder_top=args.ladder_top)
            for n in args.ranks:
                row = dict(r["rows"]["DistributedMCTS_%d" % n])
                row.update(gpu_wave=w, study_wave=sw)
                rows.append(model(row))
                print(json.dumps(row), file=sys.stderr, flush=True)
    best = {}
    for row in rows:
        k = row["ranks"]
        if "effective_sims_per_s" in row and (k not in best or row["effective_sims_per_s"] >
                                               best[k]["effective_sims_per_s"]):
            best[k] = row
    print(json.dumps({"what": "one-tree multi-GPU search (DistributedMCTS): budget efficiency "
                              "per (per-GPU wave, waves per GPU awaiting values) at N ranks "
                              "against ONE GPU at the single-GPU bench geometry searching N "
                              "times as long (the ladder), and effective sims/s = efficiency x "
                              "modelled sims/s",
                      "metric": args.metric, "ladder_depth": args.ladder_depth,
                      "per_rank_playouts": args.per_rank, "board": args.board,
                      "positions": args.positions, "lmbda": args.lmbda,
                      "rollout_delay": args.rollout_delay, "truth_mult": args.truth_mult,
                      "gpu_rates": rates,
                      "serving_rates": {"%d/%d" % k: v for k, v in (serving or {}).items()},
                      "one_gpu_effective_sims_per_s": (rates or {}).get(512),
                      "master_ceiling": args.master_ceiling,
                      "master_ceilings_by_wave": ceilings,
                      "rows": rows, "best_by_ranks": best}, indent=1), flush=True)


if __name__ == "__main__":
    main()
