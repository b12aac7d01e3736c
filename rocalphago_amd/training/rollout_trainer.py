"""Training the fast rollout policy from game records.

The rollout policy (csrc/mcts/rollout.hpp, run natively and by the GPU rollout kernel) is a
linear softmax over the legal candidate moves of a position: 7 binary local features (response
to the last move, save-atari, capture, self-atari, distance-2 of the last move, near one's own
previous move, first line) plus one weight per 3x3 pattern of the 8 surrounding points (65536).
AlphaGo trains such a policy by maximum likelihood on expert moves; this module does the same:

  * positions come from SGF files (main line); for every move the native policy enumerates the
    candidates with their feature bits and pattern index, illegal candidates (suicide / ko) are
    dropped exactly as the sampler drops them, and the played move is the target;
  * the log-likelihood (with L2 on the pattern table) is maximised with Adam in PyTorch; the
    pattern table is a sparse gather, so an epoch over thousands of positions takes seconds.

  python -m rocalphago_amd.training.rollout_trainer GAMES_DIR out.npz [--epochs 30]

``load_rollout_policy(path)`` returns a ``_rocgo.RolloutPolicy`` with the trained weights, usable
by ``ParallelMCTS(rollout=...)`` on the CPU and the GPU alike.
"""
import argparse
import glob
import json
import os

import numpy as np
import torch

from .._native import engine as _engine
from ..utils.go_util import sgf_iter_states

_rg = _engine()
NF = _rg.ROLLOUT_FEATURES
NPAT = _rg.ROLLOUT_PATTERNS


def _positions_from_sgf(text, policy, max_candidates=384):
    """Yield (feature bits [n] uint8, pattern idx [n] int32, target index) per move."""
    for gs, move, player in sgf_iter_states(text, include_end=False):
        if move is None:
            continue
        b = gs.native
        if b.current_player != player:
            gs.current_player = player
            b = gs.native
        mv, fb, pat = policy.candidates(b)
        legal = np.array([b.is_legal(int(a)) for a in mv], dtype=bool)
        mv, fb, pat = mv[legal], fb[legal], pat[legal]
        flat = move[0] * gs.size + move[1]
        hit = np.nonzero(mv == flat)[0]
        if len(hit) == 0 or len(mv) > max_candidates:
            continue  # e.g. the played move fills an own eye: not a rollout candidate
        yield fb, pat, int(hit[0])


def build_dataset(sgf_paths, policy=None):
    """Padded arrays: bits [N, C, NF] float32, pattern [N, C] int64, mask [N, C] bool,
    target [N] int64."""
    policy = policy or _rg.RolloutPolicy()
    rows = []
    for path in sgf_paths:
        with open(path) as f:
            text = f.read()
        try:
            rows.extend(_positions_from_sgf(text, policy))
        except Exception:  # malformed record: skip the file, like the converter does
            continue
    if not rows:
        raise ValueError("no usable positions")
    C = max(len(r[0]) for r in rows)
    N = len(rows)
    bits = np.zeros((N, C, NF), np.float32)
    pat = np.zeros((N, C), np.int64)
    mask = np.zeros((N, C), bool)
    tgt = np.zeros(N, np.int64)
    for i, (fb, pt, t) in enumerate(rows):
        n = len(fb)
        bits[i, :n] = (fb[:, None] >> np.arange(NF)[None, :]) & 1
        pat[i, :n] = pt
        mask[i, :n] = True
        tgt[i] = t
    return {"bits": bits, "pattern": pat, "mask": mask, "target": tgt}


class RolloutModel(torch.nn.Module):
    def __init__(self, init=None):
        super(RolloutModel, self).__init__()
        init = init or _rg.RolloutPolicy()
        self.w = torch.nn.Parameter(torch.tensor(np.asarray(init.weights, np.float32)))
        self.pat = torch.nn.Parameter(torch.tensor(np.asarray(init.pattern, np.float32)))

    def forward(self, bits, pattern, mask):
        logits = bits @ self.w + self.pat[pattern]
        return logits.masked_fill(~mask, float("-inf"))


def evaluate(model, ds, device="cpu"):
    with torch.no_grad():
        bits = torch.from_numpy(ds["bits"]).to(device)
        lg = model(bits, torch.from_numpy(ds["pattern"]).to(device),
                   torch.from_numpy(ds["mask"]).to(device))
        tgt = torch.from_numpy(ds["target"]).to(device)
        loss = torch.nn.functional.cross_entropy(lg, tgt).item()
        acc = (lg.argmax(1) == tgt).float().mean().item()
    return loss, acc


def train(ds, epochs=30, lr=0.05, l2=1e-4, batch=512, seed=0, device="cpu", init=None,
          verbose=False):
    torch.manual_seed(seed)
    model = RolloutModel(init).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    N = len(ds["target"])
    t = {k: torch.from_numpy(v).to(device) for k, v in ds.items()}
    g = torch.Generator().manual_seed(seed)
    history = []
    for ep in range(epochs):
        perm = torch.randperm(N, generator=g).to(device)
        tot = 0.0
        for s in range(0, N, batch):
            idx = perm[s:s + batch]
            lg = model(t["bits"][idx], t["pattern"][idx], t["mask"][idx])
            loss = torch.nn.functional.cross_entropy(lg, t["target"][idx])
            reg = l2 * (model.pat ** 2).sum()
            opt.zero_grad()
            (loss + reg).backward()
            opt.step()
            tot += loss.item() * len(idx)
        history.append(tot / N)
        if verbose:
            print("epoch %d loss %.4f" % (ep, tot / N))
    return model, history


def to_policy(model):
    p = _rg.RolloutPolicy()
    p.weights = model.w.detach().cpu().numpy()
    p.pattern = model.pat.detach().cpu().numpy()
    return p


def save_rollout_policy(policy, path):
    np.savez(path, weights=np.asarray(policy.weights, np.float32),
             pattern=np.asarray(policy.pattern, np.float32))


def load_rollout_policy(path):
    d = np.load(path, allow_pickle=False)
    p = _rg.RolloutPolicy()
    p.weights = d["weights"]
    p.pattern = d["pattern"]
    return p


def run_training(cmd_line_args=None):
    ap = argparse.ArgumentParser(description="Train the fast rollout policy on SGF games.")
    ap.add_argument("games", help="directory of .sgf files (searched recursively)")
    ap.add_argument("out", help="output .npz (weights + pattern table)")
    ap.add_argument("--epochs", type=int, default=30)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--l2", type=float, default=1e-4)
    ap.add_argument("--holdout", type=float, default=0.1, help="fraction of games held out")
    ap.add_argument("--verbose", "-v", action="store_true")
    args = ap.parse_args(cmd_line_args)
    paths = sorted(glob.glob(os.path.join(args.games, "**", "*.sgf"), recursive=True))
    if not paths:
        raise SystemExit("no .sgf files under %s" % args.games)
    n_hold = int(len(paths) * args.holdout) if len(paths) > 1 else 0
    train_paths, hold_paths = paths[n_hold:], paths[:n_hold]
    ds = build_dataset(train_paths)
    base_loss, base_acc = evaluate(RolloutModel(), ds)
    model, hist = train(ds, args.epochs, args.lr, args.l2, verbose=args.verbose)
    loss, acc = evaluate(model, ds)
    meta = {"positions": int(len(ds["target"])), "train_games": len(train_paths),
            "default_policy": {"loss": base_loss, "acc": base_acc},
            "trained": {"loss": loss, "acc": acc}}
    if hold_paths:
        hd = build_dataset(hold_paths)
        meta["holdout"] = dict(zip(("loss", "acc"), evaluate(model, hd)))
    save_rollout_policy(to_policy(model), args.out)
    with open(os.path.splitext(args.out)[0] + ".json", "w") as f:
        json.dump(meta, f, indent=2)
    if args.verbose:
        print(json.dumps(meta))
    return meta


if __name__ == "__main__":
    run_training()
