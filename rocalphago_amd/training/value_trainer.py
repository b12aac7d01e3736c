"""Value-network training — the reference's reinforcement_value_trainer.py is empty and
value.py only has TODO stubs; this module provides both halves:

* ``generate_value_dataset``: self-play with a policy (batched, lock-step games), ONE position
  sampled uniformly per game (decorrelated, as in the AlphaGo paper), label z = +1 if the player
  to move at that position eventually won, -1 if lost, 0 for a tie. Written as HDF5
  (``states`` uint8 [N, F, S, S] with the value features incl. ``color``, ``values`` float32
  [N, 1], ``features``).
* ``ValueTrainer`` / ``run_training``: MSE regression of a CNNValue on such a dataset with the
  same device-resident pipeline as supervised training (random symmetries — the value is
  invariant), RCCL data parallelism and the same output directory contract (metadata.json,
  weights.{epoch:05d}.hdf5).
"""
import json
import os
import time

import numpy as np
import torch

from ..engine import gamestate as go
from ..features.preprocessing import VALUE_FEATURES, Preprocess
from ..io import h5lite
from ..models import kerasish as K
from ..models.value import CNNValue
from ..parallel.dp import BucketedAllReduce, DPContext
from .data import transform_ids
from ..utils.metrics import RankMetrics
from .supervised import (Heartbeat, MetadataWriterCallback, _fault_step, _opt_sidecar,
                         resume_epoch_base, save_checkpoint)


def _python_value_games(player, n, board, move_limit, target):
    """Lock-step Python self-play of ``n`` games; returns (snapshot states, final states)."""
    states = [go.GameState(size=board) for _ in range(n)]
    snap = [None] * n
    unfinished = list(range(n))
    while unfinished:
        sts = [states[i] for i in unfinished]
        for i, st in zip(unfinished, sts):
            if snap[i] is None and len(st.history) >= target[i]:
                snap[i] = st.copy()
        moves = player.get_moves(sts)
        nxt = []
        for i, st, mv in zip(unfinished, sts, moves):
            st.do_move(mv)
            if not st.is_end_of_game and len(st.history) < move_limit:
                nxt.append(i)
        unfinished = nxt
    snaps = [snap[i] if snap[i] is not None else states[i] for i in range(n)]
    return snaps, [s.get_winner() for s in states]


def _use_native(player, native):
    if native is False:
        return False
    from .selfplay import NativeSelfPlay
    ok = NativeSelfPlay.supported(player, player)
    if native and not ok:
        raise RuntimeError("native self-play needs a fused-HIP policy player on a GPU")
    return ok


def generate_value_dataset(player, n_games, out_file=None, board=19, features=VALUE_FEATURES,
                           move_limit=500, rng=None, batch_games=64, rank=0, world=1,
                           native=None):
    """Self-play ``n_games`` with ``player`` (needs get_moves); return (states, values).

    Data-parallel generation: with ``world`` > 1 every rank plays its slice of the games
    (``rank::world``, its own random stream) and returns its rows; with ``out_file`` each rank
    writes ``<out_file>.part<rank>`` and the caller merges them (``merge_value_shards``; the
    ``generate`` CLI does this on rank 0 after a barrier). ``native`` (default: when the
    player runs on the fused HIP path) advances all games of a ply in one native call and one
    GPU pass (training/selfplay.py) instead of the per-game Python loop."""
    rng = rng or np.random.RandomState(0)
    if world > 1:
        shared = getattr(player, "rng", None) is rng
        rng = np.random.RandomState(rng.randint(0, 2 ** 31 - 1) + 7919 * rank)
        if shared:
            # the player draws its moves (and the native self-play seeds) from its own rng: a
            # player built on the caller's stream would play the same games on every rank
            player.rng = np.random.RandomState(rng.randint(0, 2 ** 31 - 1))
    mine = len(range(rank, n_games, world))
    pp = Preprocess(features)
    use_native = _use_native(player, native)
    sp = None
    if use_native:
        from .selfplay import NativeSelfPlay
        sp = NativeSelfPlay(player, player)
        zw, zb, _ = go._zobrist(board)
        lookup = {go.WHITE: zw, go.BLACK: zb}
    all_states, all_values = [], []
    done = 0
    while done < mine:
        n = min(batch_games, mine - done)
        target = [int(rng.randint(0, move_limit // 2)) for _ in range(n)]
        if use_native:
            boards, winners = sp.sample_positions(n, board, target, move_limit)
            snaps = [go.GameState._wrap(b, board, lookup) for b in boards]
            winners = [int(w) for w in winners]
        else:
            snaps, winners = _python_value_games(player, n, board, move_limit, target)
        for s, w in zip(snaps, winners):
            all_states.append(s)
            all_values.append(0.0 if w == 0 else (1.0 if w == s.current_player else -1.0))
        done += n
    F = pp.output_dim
    X = pp.states_to_tensor_u8(all_states) if all_states else \
        np.zeros((0, F, board, board), np.uint8)
    y = np.asarray(all_values, np.float32).reshape(-1, 1)
    if out_file:
        path = out_file if world == 1 else "%s.part%03d" % (out_file, rank)
        _write_value_file(path, X, y, features)
    return X, y


def _write_value_file(path, X, y, features):
    with h5lite.File(path, "w") as f:
        f.create_dataset("states", data=X, chunks=(64,) + X.shape[1:], compression="lzf",
                         maxshape=(None,) + X.shape[1:])
        f["values"] = y
        f["features"] = np.bytes_(",".join(features))


def merge_value_shards(out_file, world, remove=True):
    """Concatenate the per-rank ``<out_file>.partNNN`` files into ``out_file`` (streamed one
    shard at a time; rank order)."""
    parts = ["%s.part%03d" % (out_file, r) for r in range(world)]
    values, feats, ds = [], None, None
    with h5lite.File(out_file, "w") as f:
        for p in parts:
            src = h5lite.File(p)
            X = src["states"][()]
            values.append(np.asarray(src["values"][()], np.float32).reshape(-1, 1))
            feats = src["features"][()]
            if ds is None:
                ds = f.create_dataset("states", shape=(0,) + X.shape[1:], dtype=np.uint8,
                                      chunks=(64,) + X.shape[1:], compression="lzf",
                                      maxshape=(None,) + X.shape[1:])
            if len(X):
                ds.append(X)
            src.close()
        f["values"] = np.concatenate(values) if values else np.zeros((0, 1), np.float32)
        f["features"] = feats if feats is not None else np.bytes_("")
    if remove:
        for p in parts:
            os.remove(p)
    return out_file


def run_generate(cmd_line_args=None):
    """``generate`` CLI: self-play a value dataset with a policy, sharded over the ranks of a
    ``torchrun`` job (one GPU each), merged by rank 0."""
    import argparse
    from ..models.policy import CNNPolicy
    from ..players.ai import ProbabilisticPolicyPlayer
    parser = argparse.ArgumentParser(description="Generate a value-network dataset by self-play.")
    parser.add_argument("model", help="CNNPolicy JSON model file")
    parser.add_argument("weights", help="policy weights (HDF5)")
    parser.add_argument("out_file", help="output HDF5 (states, values, features)")
    parser.add_argument("--games", "-n", type=int, default=1000)
    parser.add_argument("--move-limit", type=int, default=500)
    parser.add_argument("--temperature", type=float, default=0.67)
    parser.add_argument("--batch-games", type=int, default=256)
    parser.add_argument("--seed", type=int, default=0)
    parser.add_argument("--python-loop", action="store_true",
                        help="per-game Python self-play instead of the native batch")
    args = parser.parse_args(cmd_line_args)
    dp = DPContext()
    pol = CNNPolicy.load_model(args.model, device=dp.device)
    pol.model.load_weights(args.weights)
    # one random stream per rank for the player's moves (the same seed everywhere would give
    # every rank the same game trajectories); the snapshot targets draw from ``rng``
    rng = np.random.RandomState(args.seed)
    player = ProbabilisticPolicyPlayer(pol, temperature=args.temperature,
                                       move_limit=args.move_limit,
                                       rng=np.random.RandomState(args.seed + 7919 * dp.rank))
    board = pol.model.input_shape[-1]
    features = list(pol.preprocessor.feature_list) + ["color"]
    t0 = time.time()
    X, _ = generate_value_dataset(player, args.games, out_file=args.out_file, board=board,
                                  features=features, move_limit=args.move_limit, rng=rng,
                                  batch_games=args.batch_games, rank=dp.rank, world=dp.world,
                                  native=False if args.python_loop else None)
    dp.barrier()
    if dp.world > 1 and dp.is_root:
        merge_value_shards(args.out_file, dp.world)
    dp.barrier()
    dt = time.time() - t0
    if dp.is_root:
        print(json.dumps({"games": args.games, "seconds": round(dt, 3),
                          "games_per_s": round(args.games / max(dt, 1e-9), 3),
                          "world": dp.world, "out_file": args.out_file}))
    return args.out_file


class ValueTrainer(object):
    """Device-resident value-net loop (MSE), shared by run_training and bench.py."""

    def __init__(self, value_model, states, values, batch_size, symmetries=None, dp=None,
                 seed=0, metrics=None):
        self.model = value_model
        self.dev = value_model.device
        self.states = states if isinstance(states, torch.Tensor) else \
            torch.from_numpy(np.ascontiguousarray(states, np.uint8)).to(self.dev)
        self.values = values if isinstance(values, torch.Tensor) else \
            torch.from_numpy(np.asarray(values, np.float32).reshape(-1, 1)).to(self.dev)
        self.B = batch_size
        self.dp = dp
        self.metrics = metrics
        self.planes = value_model.input_shape[-3]  # (None,) F, S, S
        self.sym = torch.tensor(transform_ids(symmetries or ["noop"]), dtype=torch.int32,
                                device=self.dev)
        self.gen = torch.Generator(device=self.dev)
        self.seed = seed + (dp.rank if dp else 0)
        self.gen.manual_seed(self.seed)
        self.plan = value_model._plan_for() if self.dev.type == "cuda" else None
        self.bucketer = None
        if self.plan is not None and dp is not None and dp.enabled:
            # layer-triggered buckets: the all-reduce of the top layers (+ the dense head) runs
            # while the lower layers' wgrad/dgrad kernels are still queued
            self.bucketer = BucketedAllReduce(dp, value_model.net.flat_grad,
                                              self.plan.layer_offsets(),
                                              timer=metrics.comm if metrics else None)
        self.loss_sum = torch.zeros((), device=self.dev)
        self.count = 0
        self.steps = 0  # steps taken by this trainer (never reset)

    def step(self, index):
        n = index.numel()
        model = self.model
        if self.plan is not None:
            # one launch for the transforms and the targets (batch.hip), as the SL step does
            from ..ops import hipops as ops
            tf, y = ops.value_batch(index.long().contiguous(), self.values.reshape(-1),
                                    self.sym, self.seed, self.draw_counter())
            B = self.plan.prepare(self.states, index=index, transforms=tf)
            hook = self.bucketer.layer_done if self.bucketer else None
            loss = self.plan.fwd_bwd(B, y, None, on_layer_grads=hook)
            if self.bucketer:
                self.bucketer.finish()
            model.optimizer.apply(model.net)
            self.loss_sum.add_(loss, alpha=n)
        else:
            tf = self.sym[torch.randint(0, self.sym.numel(), (n,), generator=self.gen,
                                        device=self.dev)]
            y = self.values[index]
            X = self._host_states(index, tf)
            saved = model.grad_allreduce
            if self.dp is not None and self.dp.enabled:
                model.grad_allreduce = self.dp.allreduce_mean_
            loss = model.train_on_batch(X, y.cpu().numpy())
            model.grad_allreduce = saved
            self.loss_sum += float(loss) * n
        self.count += n
        self.steps += 1
        if self.metrics is not None:
            self.metrics.step_done()

    def draw_counter(self):
        """Counter of the hashed per-sample transform draw (batch.hip value_batch): the
        optimizer's global iteration, which the checkpoint saves, so a resumed run draws the same
        transforms and no two steps share a draw. (``self.count`` was a per-window sample count
        that ``pop_loss`` resets: every logging window repeated the previous window's draws.)
        Models without an iteration counter fall back to this trainer's own step count."""
        it = getattr(self.model.optimizer, "iterations", None)
        return int(it) if it is not None else self.steps

    def _host_states(self, index, tf=None):
        from .data import apply_transform_np
        st = self.states[index]
        if st.dtype == torch.int64:  # bit-packed (training/replay.py)
            from .replay import unpack_bits
            st = unpack_bits(st, self.planes)
        st = st.cpu().numpy()
        if tf is None:
            return st.astype(np.float32)
        return np.stack([apply_transform_np(s, int(t))
                         for s, t in zip(st, tf.cpu().numpy())]).astype(np.float32)

    @classmethod
    def from_replay(cls, value_model, buffer, batch_size, symmetries=None, dp=None, seed=0):
        """Train directly on a ReplayBuffer (bit-packed positions, float outcomes); sample
        indices with ``buffer.sample``."""
        return cls(value_model, buffer.states[:len(buffer)],
                   buffer.targets[:len(buffer)].reshape(-1, 1), batch_size, symmetries, dp, seed)

    def pop_loss(self):
        t = torch.stack([self.loss_sum, torch.tensor(float(self.count), device=self.dev)])
        if self.dp is not None and self.dp.enabled:
            self.dp.allreduce_sum_(t)
        t = t.cpu().numpy()
        self.loss_sum.zero_()
        self.count = 0
        return float(t[0] / max(t[1], 1))

    def evaluate(self, indices, batch=None):
        """Mean squared error over dataset rows ``indices`` (no augmentation), in minibatch
        chunks straight from the device-resident uint8 states. Under DP every rank evaluates a
        strided shard and the (sum, count) pair is all-reduced."""
        batch = batch or max(self.B, 256)
        if not isinstance(indices, torch.Tensor):
            indices = torch.as_tensor(np.asarray(indices, np.int64), device=self.dev)
        if self.dp is not None and self.dp.enabled:
            indices = indices[self.dp.rank::self.dp.world]
        tot = torch.zeros(2, dtype=torch.float64, device=self.dev)
        with torch.no_grad():
            for s in range(0, indices.numel(), batch):
                idx = indices[s:s + batch]
                y = self.values[idx].reshape(-1).double()
                if self.plan is not None:
                    pred = self.plan.forward(self.states, index=idx).reshape(-1).double()
                else:
                    pred = torch.as_tensor(self.model.predict(self._host_states(idx)),
                                           device=self.dev).reshape(-1).double()
                tot[0] += ((pred - y) ** 2).sum()
                tot[1] += idx.numel()
        if self.dp is not None and self.dp.enabled:
            self.dp.allreduce_sum_(tot)
        t = tot.cpu().numpy()
        return float(t[0] / max(t[1], 1))


def run_training(cmd_line_args=None):
    import argparse
    parser = argparse.ArgumentParser(description='Train a value network on self-play positions.')
    parser.add_argument("model", help="Path to a CNNValue JSON model file")
    parser.add_argument("train_data", help="HDF5 with 'states' and 'values' (see generate_value_dataset)")  # noqa: E501
    parser.add_argument("out_directory", help="directory where metadata and weights will be saved")
    parser.add_argument("--minibatch", "-B", "--per-gpu-batch", type=int, default=32,
                        help="positions per rank per step (global batch = this x WORLD_SIZE)")
    parser.add_argument("--epochs", "-E", type=int, default=10)
    parser.add_argument("--epoch-length", "-l", type=int, default=None,
                        help="training positions per epoch (default: the training split)")
    parser.add_argument("--learning-rate", "-r", type=float, default=0.003)
    parser.add_argument("--decay", "-d", type=float, default=8.664339379294006e-08)
    parser.add_argument("--train-val-test", nargs=3, type=float, default=[0.93, .05, .02])
    parser.add_argument("--symmetries", default='noop,rot90,rot180,rot270,fliplr,flipud,diag1,diag2')  # noqa: E501
    parser.add_argument("--weights", default=None, help="resume from weights in out_directory")
    parser.add_argument("--seed", type=int, default=0)
    parser.add_argument("--dtype", help="GPU compute precision: bf16 (fused HIP kernels) or fp32 (reference precision, generic executor). Default: bf16", choices=["bf16", "fp32"], default="bf16")  # noqa: E501
    parser.add_argument("--verbose", "-v", default=False, action="store_true")
    args = parser.parse_args(cmd_line_args)

    dp = DPContext()
    resume = args.weights is not None
    net = CNNValue.load_model(args.model, device=dp.device).set_dtype(args.dtype)
    model = net.model
    if resume:
        model.load_weights(os.path.join(args.out_directory, args.weights))
    dp.broadcast_model(model)
    data = h5lite.File(args.train_data)
    states, values = data["states"][()], data["values"][()]
    if states.shape[1] != net.preprocessor.output_dim:
        raise ValueError("dataset has %d planes, model expects %d" %
                         (states.shape[1], net.preprocessor.output_dim))
    n = len(states)
    n_train = int(args.train_val_test[0] * n)
    n_train -= n_train % args.minibatch
    if dp.is_root and not os.path.exists(args.out_directory):
        os.makedirs(args.out_directory)
    dp.barrier()
    meta_file = os.path.join(args.out_directory, "metadata.json")
    meta = MetadataWriterCallback(meta_file)
    if resume and os.path.exists(meta_file):
        with open(meta_file) as f:
            meta.metadata = json.load(f)
    meta.metadata["training_data"] = args.train_data
    meta.metadata["model_file"] = args.model
    meta.metadata["cmd_line_args"] = meta.metadata.get("cmd_line_args", []) + [vars(args)]
    ckpt = K.ModelCheckpoint(os.path.join(args.out_directory, "weights.{epoch:05d}.hdf5"))
    ckpt.set_model(model)
    sgd = K.SGD(lr=args.learning_rate, decay=args.decay)
    model.compile(loss="mean_squared_error", optimizer=sgd)
    cursor = 0
    opt_state = _opt_sidecar(os.path.join(args.out_directory, args.weights)) if resume else None
    if opt_state:
        sgd.iterations = int(opt_state["iterations"])
        cursor = int(opt_state.get("cursor", 0))
    epoch_base = resume_epoch_base(meta.metadata, opt_state)
    heartbeat = Heartbeat(args.out_directory, dp.is_root)
    perm = np.random.RandomState(args.seed).permutation(n)
    rank_metrics = RankMetrics(args.out_directory, dp.rank, dp.world, dp.device)
    trainer = ValueTrainer(model, states, values, args.minibatch, args.symmetries.split(","), dp,
                           seed=args.seed, metrics=rank_metrics)
    tr = torch.from_numpy(perm[:n_train].astype(np.int64)).to(dp.device)
    va = torch.from_numpy(perm[n_train:].astype(np.int64)).to(dp.device)
    # every rank runs the SAME number of steps per epoch (ceil over the global batch), taking
    # its slice of each global batch modulo n_train — so the gradient all-reduces pair up
    # whatever n_train / (minibatch * world) is
    gb = args.minibatch * dp.world
    per_epoch = args.epoch_length or n_train
    steps = -(-per_epoch // gb) if n_train else 0
    fault = _fault_step(dp.rank)
    arange = torch.arange(args.minibatch, device=dp.device)
    for epoch in range(args.epochs):
        t0 = time.time()
        for _ in range(steps):
            if fault is not None and sgd.iterations >= fault:
                raise RuntimeError("injected fault at step %d (RAG_FAULT_AT_STEP)" % fault)
            trainer.step(tr[(cursor + dp.rank * args.minibatch + arange) % n_train])
            cursor = (cursor + gb) % n_train
            heartbeat(sgd.iterations)
        logs = {"loss": trainer.pop_loss()}
        if va.numel():
            logs["val_loss"] = trainer.evaluate(va)
        dt = time.time() - t0
        gepoch = epoch_base + epoch
        rank_metrics.log(epoch=gepoch, step=int(sgd.iterations))
        save_checkpoint(ckpt, gepoch, logs,
                        {"iterations": int(sgd.iterations), "cursor": int(cursor),
                         "lr": args.learning_rate, "decay": args.decay})
        meta.record(gepoch, logs)
        if dp.is_root:
            with open(os.path.join(args.out_directory, "metrics.jsonl"), "a") as f:
                f.write(json.dumps(dict(logs, epoch=gepoch, seconds=round(dt, 3),
                                        positions_per_s=round(steps * gb / max(dt, 1e-9), 1),
                                        world=dp.world, step=int(sgd.iterations))) + "\n")
        if args.verbose and dp.is_root:
            print("epoch %d: %s (%.1fs)" % (gepoch, json.dumps(logs), dt))
    dp.barrier()
    return meta.metadata


if __name__ == '__main__':
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "generate":
        run_generate(sys.argv[2:])
    else:
        run_training()
