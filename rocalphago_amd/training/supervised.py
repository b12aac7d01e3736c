"""Supervised policy training — reference AlphaGo/training/supervised_policy_trainer.py.

Same CLI (``run_training(cmd_line_args)``: model json, HDF5 dataset, output dir, --minibatch,
--epochs, --epoch-length, --learning-rate, --decay, --weights (resume), --train-val-test,
--symmetries, --verbose) and the same output directory contract: ``metadata.json`` (epochs /
best_epoch / training_data / model_file / cmd_line_args), ``shuffle.npz`` and
``weights.{epoch:05d}.hdf5`` with 0-based epochs (SURVEY §2.5 d).

Engine: the dataset is loaded into device memory once (training/data.py); each step packs,
gathers and augments the batch on the GPU, runs the fused HIP forward/backward
(models/fused.py) and one fused SGD kernel; with WORLD_SIZE > 1 (torchrun) gradients are
all-reduced over RCCL in layer buckets overlapped with backward (parallel/dp.py). The generator
API of the reference (``shuffled_hdf5_batch_generator``) is kept for compatibility and used by
the CPU path.
"""
import json
import os
import time

import numpy as np
import torch

from ..features.preprocessing import Preprocess
from ..io import h5lite
from ..models import kerasish as K
from ..models.policy import CNNPolicy
from ..ops import hipops as ops
from ..parallel.dp import BucketedAllReduce, DPContext
from ..utils.metrics import RankMetrics
from .data import BOARD_TRANSFORMATIONS, DeviceDataset, transform_ids


def one_hot_action(action, size=19):
    categorical = np.zeros((size, size))
    categorical[action] = 1
    return categorical


def shuffled_hdf5_batch_generator(state_dataset, action_dataset, indices, batch_size,
                                  transforms=[]):
    """Reference generator (supervised_policy_trainer.py:19-45): random symmetry per sample."""
    state_batch_shape = (batch_size,) + tuple(state_dataset.shape[1:])
    game_size = state_batch_shape[-1]
    Xbatch = np.zeros(state_batch_shape)
    Ybatch = np.zeros((batch_size, game_size * game_size))
    batch_idx = 0
    while True:
        for data_idx in indices:
            transform = np.random.choice(transforms)
            state = np.array([transform(plane) for plane in state_dataset[data_idx]])
            action_xy = tuple(action_dataset[data_idx])
            action = transform(one_hot_action(action_xy, game_size))
            Xbatch[batch_idx] = state
            Ybatch[batch_idx] = action.flatten()
            batch_idx += 1
            if batch_idx == batch_size:
                batch_idx = 0
                yield (Xbatch, Ybatch)


class MetadataWriterCallback(K.Callback):
    def __init__(self, path):
        super(MetadataWriterCallback, self).__init__()
        self.file = path
        self.metadata = {"epochs": [], "best_epoch": 0}

    def on_epoch_end(self, epoch, logs={}):
        # Keras numbers the epochs of every fit call from 0: append (the reference's behaviour)
        self.record(len(self.metadata["epochs"]), logs)

    def record(self, epoch, logs):
        """Log ``logs`` as global epoch ``epoch`` (0-based, the weights file's number): the list
        is cut or padded so that entry i always describes ``weights.<i>.hdf5``, and
        ``best_epoch`` is recomputed from the entries kept."""
        eps = self.metadata["epochs"]
        del eps[epoch:]
        while len(eps) < epoch:
            eps.append({})  # an epoch whose log was lost (never written before a kill)
        eps.append(logs)
        self.metadata["best_epoch"] = best_epoch(eps)
        if K._is_rank0():
            _atomic_json(self.file, self.metadata, indent=2)


def best_epoch(epochs):
    """Index of the lowest val_loss (loss without a validation split) among the logged epochs;
    the earliest on ties, 0 when nothing is logged."""
    best, key = 0, None
    for i, logs in enumerate(epochs):
        k = "val_loss" if "val_loss" in logs else "loss"
        if k not in logs:
            continue
        if key is None or logs[k] < epochs[best].get(key, float("inf")):
            best, key = i, k
    return best


class SupervisedTrainer(object):
    """Device-resident SL loop shared by run_training and bench.py.

    ``step(index)`` trains on dataset rows ``index`` (device int64) with random symmetries and
    returns device scalars (loss_sum, hit_sum) without synchronising the host."""

    def __init__(self, policy_model, dataset, batch_size, symmetries=None, dp=None,
                 loss="categorical_crossentropy", seed=0, metrics=None):
        self.model = policy_model
        self.metrics = metrics  # utils.metrics.RankMetrics (optional)
        self.ds = dataset
        self.B = batch_size
        self.dp = dp
        self.loss = loss
        self.sym = torch.tensor(transform_ids(symmetries or ["noop"]), dtype=torch.int32,
                                device=dataset.device)
        self.gen = torch.Generator(device=dataset.device)
        self.gen.manual_seed(seed + (dp.rank if dp else 0))
        self.seed = (seed * 1000003 + (dp.rank if dp else 0)) & 0xFFFFFFFF
        self.plan = policy_model._plan_for() if dataset.device.type == "cuda" else None
        self.bucketer = None
        if self.plan is not None and dp is not None and dp.enabled:
            self.bucketer = BucketedAllReduce(dp, policy_model.net.flat_grad,
                                              self.plan.layer_offsets(),
                                              timer=metrics.comm if metrics else None)
        # BatchNorm running statistics (ResnetPolicy) are averaged over ranks after each step
        self.sync_bn = dp is not None and dp.enabled and bool(policy_model.net.buffer_views())
        self.loss_sum = torch.zeros((), device=dataset.device)
        self.hit_sum = torch.zeros((), device=dataset.device)
        self.metric_acc = torch.zeros(2, device=dataset.device)  # fused-plan (loss, hits)
        self.count = 0

    def _transforms(self, n):
        sel = torch.randint(0, self.sym.numel(), (n,), generator=self.gen,
                            device=self.ds.device)
        return self.sym[sel]

    def step(self, index):
        n = index.numel()
        model = self.model
        if self.plan is not None:
            # one launch for the transforms and transformed labels, seeded by (trainer seed,
            # optimizer iteration) so a resumed run draws the same transforms
            tf, labels = ops.sl_batch(index.long().contiguous(), self.ds.labels,
                                      self.ds.tf_table, self.sym, self.seed,
                                      getattr(model.optimizer, "iterations", self.count))
            B = self.plan.prepare(self.ds.states, index=index, transforms=tf)
            mode = self.plan.loss_mode(self.loss)
            hook = self.bucketer.layer_done if self.bucketer else None
            # loss / hit sums accumulate in the head kernel (no per-step reduction launches)
            self.plan.fwd_bwd(B, labels, None, mode, 1.0 / B, on_layer_grads=hook,
                              metrics=self.metric_acc)
            if self.bucketer:
                self.bucketer.finish()
            model.optimizer.apply(model.net)
        else:
            X, Y = self.ds.host_batch(index, self._transforms(n))
            saved = model.grad_allreduce
            if self.dp is not None and self.dp.enabled:
                model.grad_allreduce = self.dp.allreduce_mean_
            r = model.train_on_batch(X, Y)
            model.grad_allreduce = saved
            loss, acc = (r if isinstance(r, list) else (r, 0.0))
            self.loss_sum += loss * n
            self.hit_sum += (acc or 0.0) * n
        if self.sync_bn:
            self.dp.sync_buffers_(model.net)
        self.count += n
        if self.metrics is not None:
            self.metrics.step_done()

    def pop_metrics(self):
        """(mean loss, accuracy) since the last call, averaged over all ranks."""
        t = torch.stack([self.loss_sum + self.metric_acc[0], self.hit_sum + self.metric_acc[1],
                         torch.tensor(float(self.count), device=self.loss_sum.device)])
        if self.dp is not None and self.dp.enabled:
            self.dp.allreduce_sum_(t)
        t = t.cpu().numpy()
        self.loss_sum.zero_()
        self.hit_sum.zero_()
        self.metric_acc.zero_()
        self.count = 0
        return float(t[0] / max(t[2], 1)), float(t[1] / max(t[2], 1))

    def evaluate(self, indices, batch=None):
        """Validation loss/accuracy over dataset rows (no augmentation). Under DP each rank
        evaluates its own strided shard and the sums are all-reduced, so the work is split N
        ways and every row is counted once."""
        batch = batch or self.B
        model = self.model
        tot = torch.zeros(3, device=self.ds.device)
        noop = torch.zeros(0, dtype=torch.int32, device=self.ds.device)
        if self.dp is not None and self.dp.enabled:
            indices = indices[self.dp.rank::self.dp.world]
        for s in range(0, len(indices), batch):
            idx = indices[s:s + batch]
            if self.plan is not None:
                B = self.plan.prepare(self.ds.states, index=idx)
                self.plan.trunk.forward(B)
                w, b0 = self.plan.head_params()
                pb = model.net.params_of(self.plan.bias_name)[0]
                lab = self.ds.labels[idx]
                self.plan.head.forward(B, w, b0, pb, labels=lab, mode=1, gscale=0.0)
                tot[0] += self.plan.head.loss[:B].sum()
                tot[1] += self.plan.head.hit[:B].sum()
                tot[2] += B
            else:
                X, Y = self.ds.host_batch(idx, noop.new_zeros(idx.numel()))
                r = model.test_on_batch(X, Y)
                loss, acc = (r if isinstance(r, list) else (r, 0.0))
                tot += torch.tensor([loss * len(X), acc * len(X), len(X)], device=tot.device)
        if self.dp is not None and self.dp.enabled:
            self.dp.allreduce_sum_(tot)
        t = tot.cpu().numpy()
        return float(t[0] / max(t[2], 1)), float(t[1] / max(t[2], 1))


def run_training(cmd_line_args=None):
    """Run SL training; command-line args may be passed in as a list."""
    import argparse
    parser = argparse.ArgumentParser(description='Perform supervised training on a policy network.')
    parser.add_argument("model", help="Path to a JSON model file (i.e. from CNNPolicy.save_model())")  # noqa: E501
    parser.add_argument("train_data", help="A .h5 file of training data")
    parser.add_argument("out_directory", help="directory where metadata and weights will be saved")
    parser.add_argument("--minibatch", "-B", "--per-gpu-batch", help="Size of training data minibatches (per rank / per GPU; the global batch is this x WORLD_SIZE). Default: 16", type=int, default=16)  # noqa: E501
    parser.add_argument("--epochs", "-E", help="Total number of iterations on the data. Default: 10", type=int, default=10)  # noqa: E501
    parser.add_argument("--epoch-length", "-l", help="Number of training examples considered 'one epoch'. Default: # training data", type=int, default=None)  # noqa: E501
    parser.add_argument("--learning-rate", "-r", help="Learning rate - how quickly the model learns at first. Default: .03", type=float, default=.03)  # noqa: E501
    parser.add_argument("--decay", "-d", help="The rate at which learning decreases. Default: .0001", type=float, default=.0001)  # noqa: E501
    parser.add_argument("--verbose", "-v", help="Turn on verbose mode", default=False, action="store_true")  # noqa: E501
    parser.add_argument("--weights", help="Name of a .h5 weights file (in the output directory) to load to resume training", default=None)  # noqa: E501
    parser.add_argument("--packed", help="Keep the dataset bit-packed on the device (2.9 KB instead of 17 KB per 19x19 position)", default=False, action="store_true")  # noqa: E501
    parser.add_argument("--train-val-test", help="Fraction of data to use for training/val/test. Must sum to 1. Invalid if restarting training", nargs=3, type=float, default=[0.93, .05, .02])  # noqa: E501
    parser.add_argument("--symmetries", help="Comma-separated list of transforms, subset of noop,rot90,rot180,rot270,fliplr,flipud,diag1,diag2", default='noop,rot90,rot180,rot270,fliplr,flipud,diag1,diag2')  # noqa: E501
    parser.add_argument("--seed", help="RNG seed for shuffling / symmetries", type=int, default=None)  # noqa: E501
    parser.add_argument("--dtype", help="GPU compute precision: bf16 (fused HIP kernels) or fp32 (reference precision, generic executor). Default: bf16", choices=["bf16", "fp32"], default="bf16")  # noqa: E501
    if cmd_line_args is None:
        args = parser.parse_args()
    else:
        args = parser.parse_args(cmd_line_args)

    dp = DPContext()
    resume = args.weights is not None
    if args.verbose and dp.is_root:
        if resume:
            print("trying to resume from %s with weights %s" %
                  (args.out_directory, os.path.join(args.out_directory, args.weights)))
        elif os.path.exists(args.out_directory):
            print("directory %s exists. any previous data will be overwritten" %
                  args.out_directory)
        else:
            print("starting fresh output directory %s" % args.out_directory)

    policy = CNNPolicy.load_model(args.model, device=dp.device).set_dtype(args.dtype)
    model_features = policy.preprocessor.feature_list
    model = policy.model
    if resume:
        model.load_weights(os.path.join(args.out_directory, args.weights))
    dp.broadcast_model(model)

    dataset = h5lite.File(args.train_data)
    if 'features' in dataset:
        dataset_features = dataset['features'][()]
        if isinstance(dataset_features, bytes):
            dataset_features = dataset_features.decode("utf-8")
        dataset_features = dataset_features.split(",")
        if len(dataset_features) != len(model_features) or \
                any(df != mf for (df, mf) in zip(dataset_features, model_features)):
            raise ValueError("Model JSON file expects features \n\t%s\n"
                             "But dataset contains \n\t%s" % ("\n\t".join(model_features),
                                                              "\n\t".join(dataset_features)))
        elif args.verbose and dp.is_root:
            print("Verified that dataset features and model features exactly match.")
    else:
        n_dataset_planes = dataset["states"].shape[1]
        n_model_planes = Preprocess(model_features).output_dim
        if n_dataset_planes != n_model_planes:
            raise ValueError("Model JSON file expects a total of %d planes from features \n\t%s\n"
                             "But dataset contains %d planes" % (n_model_planes,
                                                                 "\n\t".join(model_features),
                                                                 n_dataset_planes))
        elif args.verbose and dp.is_root:
            print("Verified agreement of number of model and dataset feature planes, but cannot "
                  "verify exact match using old dataset format.")

    n_total_data = len(dataset["states"])
    n_train_data = int(args.train_val_test[0] * n_total_data)
    n_train_data = n_train_data - (n_train_data % args.minibatch)
    n_val_data = n_total_data - n_train_data  # quirk Q10: validation = everything after train

    if args.verbose and dp.is_root:
        print("datset loaded\n\t%d total samples\n\t%d training samples\n\t%d validaion samples"
              % (n_total_data, n_train_data, n_val_data))

    if dp.is_root and not os.path.exists(args.out_directory):
        os.makedirs(args.out_directory)
    dp.barrier()

    meta_file = os.path.join(args.out_directory, "metadata.json")
    meta_writer = MetadataWriterCallback(meta_file)
    if os.path.exists(meta_file) and resume:
        with open(meta_file, "r") as f:
            meta_writer.metadata = json.load(f)
        if args.verbose and dp.is_root:
            print("previous metadata loaded: %d epochs. new epochs will be appended." %
                  len(meta_writer.metadata["epochs"]))
    meta_writer.metadata["training_data"] = args.train_data
    meta_writer.metadata["model_file"] = args.model
    meta_writer.metadata["cmd_line_args"] = meta_writer.metadata.get("cmd_line_args", [])
    meta_writer.metadata["cmd_line_args"].append(vars(args))
    meta_writer.set_model(model)

    checkpointer = K.ModelCheckpoint(os.path.join(args.out_directory, "weights.{epoch:05d}.hdf5"))
    checkpointer.set_model(model)

    rng = np.random.RandomState(args.seed) if args.seed is not None else np.random
    shuffle_file = os.path.join(args.out_directory, "shuffle.npz")
    if os.path.exists(shuffle_file) and resume:
        with open(shuffle_file, "rb") as f:
            shuffle_indices = np.load(f)
    else:
        shuffle_indices = rng.permutation(n_total_data)
        if dp.enabled:
            t = torch.from_numpy(shuffle_indices).to(dp.device)
            dp.broadcast_(t)
            shuffle_indices = t.cpu().numpy()
        if dp.is_root:
            with open(shuffle_file, "wb") as f:
                np.save(f, shuffle_indices)
    train_indices = shuffle_indices[0:n_train_data]
    val_indices = shuffle_indices[n_train_data:n_train_data + n_val_data]

    symmetries = args.symmetries.strip().split(",")
    for s in symmetries:
        if s not in BOARD_TRANSFORMATIONS:
            raise ValueError("unknown symmetry %s" % s)

    sgd = K.SGD(lr=args.learning_rate, decay=args.decay)
    model.compile(loss='categorical_crossentropy', optimizer=sgd, metrics=["accuracy"])
    # exact resume: the optimizer step count (Keras decay schedule) and the data cursor live in
    # a sidecar next to each weights file (the reference does not save them)
    cursor = 0
    opt_state = _opt_sidecar(os.path.join(args.out_directory, args.weights)) if resume else None
    if opt_state:
        sgd.iterations = int(opt_state["iterations"])
        cursor = int(opt_state.get("cursor", 0))
    epoch_base = resume_epoch_base(meta_writer.metadata, opt_state)
    heartbeat = Heartbeat(args.out_directory, dp.is_root)

    if args.packed:
        from .replay import PackedDataset
        ds = PackedDataset.from_hdf5(dataset, dp.device)
    else:
        ds = DeviceDataset.from_hdf5(dataset, dp.device)
    rank_metrics = RankMetrics(args.out_directory, dp.rank, dp.world, dp.device)
    trainer = SupervisedTrainer(model, ds, args.minibatch, symmetries, dp,
                                seed=args.seed or 0, metrics=rank_metrics)
    samples_per_epoch = args.epoch_length or n_train_data
    dev_train = torch.from_numpy(np.asarray(train_indices, dtype=np.int64)).to(dp.device)
    dev_val = torch.from_numpy(np.asarray(val_indices, dtype=np.int64)).to(dp.device)

    if args.verbose and dp.is_root:
        print("STARTING TRAINING")
    # each rank consumes its own contiguous slice of every global batch, cycling through the
    # fixed shuffled order (the reference generator never reshuffles between epochs)
    gb = args.minibatch * dp.world
    n_train = dev_train.numel()
    fault = _fault_step(dp.rank)
    metrics_file = os.path.join(args.out_directory, "metrics.jsonl")
    for epoch in range(args.epochs):
        t0 = time.time()
        seen = 0
        while seen < samples_per_epoch and n_train > 0:
            if fault is not None and sgd.iterations >= fault:
                raise RuntimeError("injected fault at step %d (RAG_FAULT_AT_STEP)" % fault)
            pos = (cursor + dp.rank * args.minibatch + torch.arange(args.minibatch,
                                                                  device=dp.device)) % n_train
            trainer.step(dev_train[pos])
            cursor = (cursor + gb) % n_train
            seen += args.minibatch
            heartbeat(sgd.iterations)
        loss, acc = trainer.pop_metrics()
        dt = time.time() - t0
        rank_metrics.log(epoch=epoch_base + epoch, step=int(sgd.iterations))
        logs = {"loss": loss, "acc": acc}
        if n_val_data > 0:
            vl, va = trainer.evaluate(dev_val)
            logs["val_loss"], logs["val_acc"] = vl, va
        gepoch = epoch_base + epoch
        # checkpoint (sidecar, then weights) before the metadata that records the epoch
        save_checkpoint(checkpointer, gepoch, logs,
                        {"iterations": int(sgd.iterations), "cursor": int(cursor),
                         "lr": args.learning_rate, "decay": args.decay})
        meta_writer.record(gepoch, logs)
        if dp.is_root:
            with open(metrics_file, "a") as f:
                f.write(json.dumps(dict(logs, epoch=gepoch, seconds=round(dt, 3),
                                        positions_per_s=round(seen * dp.world / max(dt, 1e-9), 1),
                                        world=dp.world, step=int(sgd.iterations))) + "\n")
        if args.verbose and dp.is_root:
            print("epoch %d: %s (%.1fs)" % (gepoch, json.dumps(logs), dt))
    dp.barrier()
    return meta_writer.metadata


def _opt_sidecar(weights_path):
    p = os.path.splitext(weights_path)[0] + ".opt.json"
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def _atomic_json(path, obj, **kw):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f, **kw)
    os.replace(tmp, path)


def save_checkpoint(checkpointer, epoch, logs, opt_state):
    """Epoch checkpoint that a killed job can always resume from (the supervisor's
    watchdog may SIGKILL at any instant): the optimizer/data-cursor sidecar
    ``weights.NNNNN.opt.json`` is written first, then the weights file — both through a
    temporary file and an atomic rename — so a ``weights.*.hdf5`` that exists is complete and has
    its sidecar (parallel/supervisor.latest_checkpoint only resumes from such pairs)."""
    if not K._is_rank0():
        checkpointer.on_epoch_end(epoch, logs)  # no-op off rank 0
        return
    path = checkpointer.filepath.format(epoch=epoch, **logs)
    # the epoch's logs ride in the sidecar: a kill between the checkpoint and metadata.json
    # leaves the metadata one entry short, and resume restores that entry from here
    _atomic_json(os.path.splitext(path)[0] + ".opt.json", dict(opt_state, epoch=epoch,
                                                               logs=logs))
    checkpointer.on_epoch_end(epoch, logs)


class Heartbeat(object):
    """Touches OUT_DIR/heartbeat at most every ``every_s`` seconds from the training loop (rank
    0), so the supervisor's no-progress watchdog sees a live job within long epochs."""

    def __init__(self, out_dir, enabled=True, every_s=10.0):
        self.path = os.path.join(out_dir, "heartbeat")
        self.enabled = enabled
        self.every = every_s
        self.last = 0.0

    def __call__(self, step):
        if not self.enabled:
            return
        now = time.time()
        if now - self.last < self.every:
            return
        self.last = now
        with open(self.path, "w") as f:
            f.write("%d %.3f\n" % (step, now))


def resume_epoch_base(metadata, opt_state):
    """First epoch number of a resumed run: one past the checkpoint's own epoch (from its
    sidecar), with the metadata's epoch log cut back to it (an epoch logged after the last
    complete checkpoint is re-run, not skipped)."""
    epochs = metadata.setdefault("epochs", [])
    if opt_state is None or "epoch" not in opt_state:
        return len(epochs)
    base = int(opt_state["epoch"]) + 1
    del epochs[base:]
    if len(epochs) < base:
        # killed after the checkpoint, before metadata.json recorded its epoch
        while len(epochs) < base - 1:
            epochs.append({})
        epochs.append(dict(opt_state.get("logs") or {}))
    metadata["best_epoch"] = best_epoch(epochs)
    return base


def _fault_step(rank):
    """RAG_FAULT_AT_STEP=n (or "r:n" for rank r only): raise at optimizer step n — fault
    injection for the checkpoint/resume tests."""
    spec = os.environ.get("RAG_FAULT_AT_STEP")
    if not spec:
        return None
    if ":" in spec:
        r, n = spec.split(":", 1)
        return int(n) if int(r) == rank else None
    return int(spec)


if __name__ == '__main__':
    run_training()
