"""Budget efficiency of the multi-rank searches (rocalphago_amd/search/efficiency.py): N ranks
(gloo, CPU, deterministic evaluator) with N x t playouts against one tree with t .. N t
playouts, over many positions. One JSON line per search design.

  python benchmarks/search_efficiency.py [--ranks 2 4 8] [--positions 50] [--per-rank 128]
  python benchmarks/search_efficiency.py --designs DistributedMCTS/shipped --per-rank 512 \
      --lmbda 0.5 --rollout-delay 6 --truth-mult 16     (the bench's geometry)
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
    args = ap.parse_args()
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


if __name__ == "__main__":
    main()
