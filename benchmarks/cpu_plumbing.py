"""BASELINE config #1: 9x9 SL policy (3-layer CNN, 8 input planes) on the CPU, world_size 1 —
a plumbing check of the whole SL pipeline without a GPU: native feature extraction of real game
positions, the Keras-compatible model on the PyTorch CPU path, SGD, and the JSON line.

  python benchmarks/cpu_plumbing.py [--steps 20] [--batch 64]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

FEATS = ["board", "ones", "legal", "sensibleness", "zeros", "color"]  # 3+1+1+1+1+1 = 8 planes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--positions", type=int, default=2048)
    args = ap.parse_args()
    from rocalphago_amd._native import engine
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.features.preprocessing import Preprocess
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.training.data import DeviceDataset
    from rocalphago_amd.training.supervised import SupervisedTrainer

    rg = engine()
    rp = rg.RolloutPolicy()
    pre = Preprocess(FEATS)
    # real positions: rollout-policy games on 9x9, the next move as the label
    boards, labels = [], []
    rs = np.random.RandomState(0)
    t0 = time.perf_counter()
    while len(boards) < args.positions:
        st = GameState(size=9)
        for k in range(120):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            if mv >= 0:
                boards.append(st.native.copy())
                labels.append(mv)
            st.do_move(None if mv < 0 else divmod(mv, 9))
            if st.is_end_of_game or len(boards) >= args.positions:
                break
    X = rg.batch_features(boards, pre.feature_ids, 8)
    t_feat = time.perf_counter() - t0
    dev = torch.device("cpu")
    ds = DeviceDataset(X, np.asarray(labels, np.int64), dev)
    policy = CNNPolicy(FEATS, board=9, filters_per_layer=32, layers=3, device=dev, seed=1)
    policy.model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.05),
                         metrics=["accuracy"])
    tr = SupervisedTrainer(policy.model, ds, args.batch, ["noop", "rot90", "fliplr"], None)
    g = torch.Generator().manual_seed(3)
    for _ in range(args.warmup):
        tr.step(torch.randint(0, ds.N, (args.batch,), generator=g))
    tr.pop_metrics()
    t = time.perf_counter()
    for _ in range(args.steps):
        tr.step(torch.randint(0, ds.N, (args.batch,), generator=g))
    dt = time.perf_counter() - t
    loss, acc = tr.pop_metrics()
    print(json.dumps({
        "metric": "positions/sec SL-policy train, 9x9 3-layer CNN, 8 planes, CPU (plumbing)",
        "value": round(args.batch * args.steps / dt, 1), "unit": "positions/s", "n_gpus": 0,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2),
        "dtype": "fp32", "data": "rollout-policy 9x9 games, native feature extraction",
        "feature_extraction_positions_per_s": round(len(boards) / t_feat, 1),
        "train_loss": round(loss, 4), "train_acc": round(acc, 4), "status": "pass"}))


if __name__ == "__main__":
    main()
