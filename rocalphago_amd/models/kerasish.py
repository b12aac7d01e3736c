"""A minimal, single-backend Keras-1 model surface (SURVEY §2.3 "Keras Model surface").

The reference models are Keras 1.2 objects (policy.py, value.py, nn_util.py) and its trainers call
into that API (``compile``, ``train_on_batch``, ``fit_generator``, ``save_weights`` ...).
This module re-creates exactly that surface over our own execution engine:

  * the Keras-1 JSON model spec is interpreted (Sequential and functional ``Model``; layers
    Convolution2D, Dense, Flatten, Activation, Bias, BatchNormalization, Merge, InputLayer,
    Dropout, and the optional PassLogit) and re-emitted by ``to_json`` (nn_util.py:79,100);
  * weights live in ONE flat fp32 buffer (parameters are views), in Keras order/shapes (conv OIHW,
    Dense (in, out), Bias (S*S,)) so ``get_weights``/``set_weights`` and the HDF5 layout
    (nn_util.py:81,104; random_minimodel_weights.hdf5) match the reference;
  * on a GPU, recognised architectures run on the HIP engine (models/engine.py): the
    sequential conv policy (CNNPolicy) and conv value net (CNNValue) — forward, fused
    loss, backward and the SGD update are all hand-written gfx950 kernels; other graphs (ResNet)
    run the generic graph executor with HIP convolutions (HipConv2dFn);
  * Keras-1 semantics that matter for training dynamics are reproduced: 'uniform' init
    U(-0.05, 0.05), SGD lr/(1 + decay*iterations), objectives averaged over the last axis then the
    batch (so REINFORCE log_loss carries a 1/(S*S) factor), clip epsilon 1e-7.

This is an API shim over one backend, not a Keras re-implementation or a multi-backend dispatch.
"""
import json
import math
import os

import numpy as np
import torch
import torch.nn.functional as F

from .. import _native
from ..io import h5lite

EPSILON = 1e-7

# --------------------------------------------------------------------------- device policy


def default_device():
    env = os.environ.get("RAG_DEVICE")
    if env:
        return torch.device(env)
    if torch.cuda.is_available():
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        return torch.device("cuda", lr % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


PRECISIONS = ("bf16", "fp32")


def default_precision():
    """GPU compute precision of new models: ``RAG_DTYPE`` (bf16 | fp32), default bf16."""
    p = os.environ.get("RAG_DTYPE", "bf16").lower()
    if p not in PRECISIONS:
        raise ValueError("RAG_DTYPE must be one of %s, got %r" % (PRECISIONS, p))
    return p


# --------------------------------------------------------------------------- layers

_COUNTERS = {}


def _auto_name(prefix):
    _COUNTERS[prefix] = _COUNTERS.get(prefix, 0) + 1
    return "%s_%d" % (prefix, _COUNTERS[prefix])


class Layer(object):
    """Keras-1 layer description: class name + config (+ functional inbound names)."""

    def __init__(self, class_name, config, inbound=None):
        self.class_name = class_name
        self.config = dict(config)
        if not self.config.get("name"):
            self.config["name"] = _auto_name(class_name.lower())
        self.inbound = inbound or []

    @property
    def name(self):
        return self.config["name"]

    # shapes are Keras 'th': (None, C, H, W) / (None, N)
    def output_shape(self, in_shapes):
        c, cfg = self.class_name, self.config
        s = in_shapes[0] if in_shapes else tuple(cfg.get("batch_input_shape", (None,)))
        if c == "InputLayer":
            return tuple(cfg["batch_input_shape"])
        if c == "Convolution2D":
            if cfg.get("border_mode", "valid") != "same":
                raise NotImplementedError("only border_mode='same' convolutions are supported")
            return (None, cfg["nb_filter"], s[2], s[3])
        if c == "Flatten":
            return (None, int(np.prod(s[1:])))
        if c == "Dense":
            return (None, cfg["output_dim"])
        if c == "PassLogit":
            return (None, s[1] + 1)
        return s

    def weight_specs(self, in_shape):
        c, cfg, n = self.class_name, self.config, self.name
        if c == "Convolution2D":
            specs = [(n + "_W", (cfg["nb_filter"], in_shape[1], cfg["nb_row"], cfg["nb_col"]),
                      cfg.get("init", "glorot_uniform"))]
            if cfg.get("bias", True):
                specs.append((n + "_b", (cfg["nb_filter"],), "zero"))
            return specs
        if c == "Dense":
            specs = [(n + "_W", (in_shape[1], cfg["output_dim"]), cfg.get("init",
                                                                        "glorot_uniform"))]
            if cfg.get("bias", True):
                specs.append((n + "_b", (cfg["output_dim"],), "zero"))
            return specs
        if c == "Bias":
            return [("param_0", tuple(in_shape[1:]), "zero")]
        if c == "PassLogit":
            return [(n + "_W", (in_shape[1],), "zero"), (n + "_b", (1,), "zero")]
        if c == "BatchNormalization":
            axis = cfg.get("axis", -1)
            dim = in_shape[axis]
            return [(n + "_gamma", (dim,), "one"), (n + "_beta", (dim,), "zero"),
                    (n + "_running_mean", (dim,), "zero"), (n + "_running_std", (dim,), "one")]
        return []

    def to_config(self):
        out = {"class_name": self.class_name, "config": self.config}
        return out


def Convolution2D(nb_filter, nb_row, nb_col, init="glorot_uniform", activation="linear",
                  border_mode="valid", subsample=(1, 1), bias=True, input_shape=None, name=None,
                  **kw):
    cfg = {"name": name, "nb_filter": nb_filter, "nb_row": nb_row, "nb_col": nb_col,
           "init": init, "activation": activation, "border_mode": border_mode,
           "subsample": list(subsample), "dim_ordering": "th", "bias": bias, "trainable": True,
           "W_regularizer": None, "b_regularizer": None, "activity_regularizer": None,
           "W_constraint": None, "b_constraint": None}
    if input_shape:
        cfg["batch_input_shape"] = [None] + list(input_shape)
        cfg["input_dtype"] = "float32"
    return Layer("Convolution2D", cfg)


def Dense(output_dim, init="glorot_uniform", activation="linear", bias=True, input_dim=None,
          name=None, **kw):
    cfg = {"name": name, "output_dim": output_dim, "init": init, "activation": activation,
           "bias": bias, "trainable": True, "W_regularizer": None, "b_regularizer": None,
           "activity_regularizer": None, "W_constraint": None, "b_constraint": None,
           "input_dim": input_dim}
    return Layer("Dense", cfg)


def Flatten(name=None):
    return Layer("Flatten", {"name": name, "trainable": True})


def Activation(activation, name=None):
    return Layer("Activation", {"name": name, "activation": activation, "trainable": True})


def BiasLayer(name=None):
    return Layer("Bias", {"name": name, "trainable": True})


def PassLogit(name=None):
    """Optional pass move for the policy head (off by default): appends one logit
    ``W . z + b`` computed from the S*S position logits z, so the softmax runs over S*S + 1
    classes with pass last. Parameters W (S*S,) and b (1,) start at zero."""
    return Layer("PassLogit", {"name": name, "trainable": True})


def BatchNormalization(epsilon=1e-3, mode=0, axis=-1, momentum=0.99, name=None):
    return Layer("BatchNormalization", {"name": name, "epsilon": epsilon, "mode": mode,
                                        "axis": axis, "momentum": momentum, "trainable": True,
                                        "gamma_regularizer": None, "beta_regularizer": None})


# --------------------------------------------------------------------------- init

def _init(shape, kind, gen):
    if kind in ("zero", "zeros"):
        return np.zeros(shape, np.float32)
    if kind in ("one", "ones"):
        return np.ones(shape, np.float32)
    if len(shape) == 4:
        rf = shape[2] * shape[3]
        fan_in, fan_out = shape[1] * rf, shape[0] * rf
    elif len(shape) == 2:
        fan_in, fan_out = shape[0], shape[1]
    else:
        fan_in = fan_out = int(np.sqrt(np.prod(shape)))
    if kind == "uniform":
        return gen.uniform(-0.05, 0.05, shape).astype(np.float32)
    if kind == "normal":
        return (gen.standard_normal(shape) * 0.05).astype(np.float32)
    if kind == "glorot_uniform":
        s = math.sqrt(6.0 / (fan_in + fan_out))
        return gen.uniform(-s, s, shape).astype(np.float32)
    if kind == "glorot_normal":
        return (gen.standard_normal(shape) * math.sqrt(2.0 / (fan_in + fan_out))).astype(
            np.float32)
    if kind == "he_normal":
        return (gen.standard_normal(shape) * math.sqrt(2.0 / fan_in)).astype(np.float32)
    if kind == "he_uniform":
        s = math.sqrt(6.0 / fan_in)
        return gen.uniform(-s, s, shape).astype(np.float32)
    if kind == "lecun_uniform":
        s = math.sqrt(3.0 / fan_in)
        return gen.uniform(-s, s, shape).astype(np.float32)
    raise ValueError("unknown init %s" % kind)


def _act(x, name):
    if name in (None, "linear"):
        return x
    if name == "relu":
        return F.relu(x)
    if name == "tanh":
        return torch.tanh(x)
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name == "softmax":
        return F.softmax(x, dim=-1)
    if name == "softplus":
        return F.softplus(x)
    raise ValueError("unknown activation %s" % name)


# --------------------------------------------------------------------------- HIP conv (generic)

class HipConv2dFn(torch.autograd.Function):
    """'same' conv on HIP for the generic graph executor (NCHW fp32 in/out)."""

    @staticmethod
    def forward(ctx, x, w, b):
        from ..ops import hipops as ops
        B, C, S, _ = x.shape
        cout, cin, ks, _ = w.shape
        cinp, coutp = ops.pad_channels(cin), ops.pad_channels(cout)
        hi = max(1, ks // 2)
        xp = ops.pack_nchw(x, hi, cinp)
        wf, wb = ops.pack_weights(w, coutp, cinp, wb=torch.empty(
            (ks * ks, cinp, coutp), dtype=torch.bfloat16, device=x.device))
        bias = torch.zeros(coutp, device=x.device)
        if b is not None:
            bias[:cout] = b
        y = ops.alloc_padded(B, S, max(1, ks // 2), coutp, x.device)
        ops.conv_igemm(xp, wf, bias, y, B, S, hi, max(1, ks // 2), cinp, coutp, ks, False)
        ctx.save_for_backward(xp, wb)
        ctx.meta = (B, S, cin, cout, ks, cinp, coutp, hi, b is not None)
        return ops.unpack(y, cout, max(1, ks // 2))

    @staticmethod
    def backward(ctx, gy):
        from ..ops import hipops as ops
        xp, wb = ctx.saved_tensors
        B, S, cin, cout, ks, cinp, coutp, hi, has_b = ctx.meta
        hg = max(1, ks // 2)
        g = ops.pack_nchw(gy, hg, coutp)
        dx = ops.alloc_padded(B, S, hi, cinp, gy.device)
        ops.conv_igemm(g, wb, None, dx, B, S, hg, hi, coutp, cinp, ks, False)
        dw = torch.empty((cout, cin, ks, ks), device=gy.device)
        db = torch.empty((cout,), device=gy.device)
        ops.conv_wgrad(g, xp, dw, db, B, S, hi, cout, coutp, cin, cinp, ks, hg=hg)
        return ops.unpack(dx, cin, hi), dw, (db if has_b else None)


# --------------------------------------------------------------------------- the network

class KerasNet(torch.nn.Module):
    """Parameters (one flat fp32 buffer) + a generic executor for a Keras-1 layer graph."""

    def __init__(self, layers, functional=False, inputs=None, outputs=None, device=None,
                 seed=None):
        super(KerasNet, self).__init__()
        self.layer_defs = layers
        self.functional = functional
        self.input_names = inputs or []
        self.output_names = outputs or []
        self.device = torch.device(device) if device is not None else default_device()
        # shapes
        shapes = {}
        if functional:
            for ld in layers:
                ins = [shapes[n] for n in ld.inbound]
                shapes[ld.name] = ld.output_shape(ins)
            self.input_shape = shapes[self.input_names[0]]
        else:
            prev = None
            for ld in layers:
                shapes[ld.name] = ld.output_shape([prev] if prev is not None else [])
                prev = shapes[ld.name]
            first = layers[0].config.get("batch_input_shape")
            self.input_shape = tuple(first) if first else None
        self.shapes = shapes
        # weights
        gen = np.random.RandomState(seed) if seed is not None else np.random
        self.weight_names = []
        self.layer_weights = {}
        inits = []
        prev = self.input_shape
        for ld in layers:
            ins = [shapes[n] for n in ld.inbound] if functional else [prev]
            specs = ld.weight_specs(ins[0]) if ins and ins[0] is not None else []
            self.layer_weights[ld.name] = []
            for wname, shape, init in specs:
                self.layer_weights[ld.name].append((wname, shape))
                self.weight_names.append((ld.name, wname, shape))
                inits.append(_init(shape, init, gen))
            prev = shapes[ld.name]
        sizes = [int(np.prod(s)) for (_, _, s) in self.weight_names]
        # 4-element alignment per tensor keeps vector loads aligned in the kernels
        offs, total = [], 0
        for n in sizes:
            offs.append(total)
            total += (n + 3) // 4 * 4
        self.flat = torch.zeros(max(total, 4), dtype=torch.float32, device=self.device)
        self.flat_grad = torch.zeros_like(self.flat)
        self._views, self._gviews = [], []
        for (lname, wname, shape), off, n, val in zip(self.weight_names, offs, sizes, inits):
            v = self.flat[off:off + n].view(shape)
            v.copy_(torch.from_numpy(val))
            self._views.append(v)
            self._gviews.append(self.flat_grad[off:off + n].view(shape))
        self.version = 0
        self._engine = None
        self.training_mode = False
        # compute precision on the GPU: "bf16" = the fused HIP plans / HipConv2dFn (bf16
        # operands, fp32 accumulation); "fp32" = reference precision through the generic
        # executor with fp32 torch convolutions (parity checks against fp32 checkpoints)
        self.precision = default_precision()

    # ---- weights
    def params_of(self, lname):
        return [v for (ln, _, _), v in zip(self.weight_names, self._views) if ln == lname]

    def grads_of(self, lname):
        return [v for (ln, _, _), v in zip(self.weight_names, self._gviews) if ln == lname]

    def buffer_views(self):
        """Non-trainable state (BatchNorm running averages), as views into ``flat``."""
        return [v for (_, wname, _), v in zip(self.weight_names, self._views)
                if "_running_" in wname]

    def get_weights(self):
        return [v.detach().cpu().numpy().copy() for v in self._views]

    def set_weights(self, weights):
        if len(weights) != len(self._views):
            raise ValueError("expected %d weight arrays, got %d" % (len(self._views),
                                                                     len(weights)))
        for v, w in zip(self._views, weights):
            w = np.asarray(w, dtype=np.float32)
            if tuple(w.shape) != tuple(v.shape):
                raise ValueError("weight shape mismatch %s vs %s" % (w.shape, tuple(v.shape)))
            v.copy_(torch.from_numpy(w))
        self.bump()

    def bump(self):
        self.version += 1

    def weights_version(self):
        return (self.version, self.flat._version)

    def to_device(self, device):
        device = torch.device(device)
        if device == self.flat.device:
            return
        flat = self.flat.to(device)
        self.flat = flat
        self.flat_grad = torch.zeros_like(flat)
        views, gviews, off = [], [], 0
        for (ln, wn, shape) in self.weight_names:
            n = int(np.prod(shape))
            views.append(self.flat[off:off + n].view(shape))
            gviews.append(self.flat_grad[off:off + n].view(shape))
            off += (n + 3) // 4 * 4
        self._views, self._gviews = views, gviews
        self.device = device
        self._engine = None
        self.bump()

    @property
    def uses_learning_phase(self):
        return any(ld.class_name in ("BatchNormalization", "Dropout") for ld in self.layer_defs)

    # ---- generic executor (autograd-capable, used on CPU and for non-fused graphs)
    def _run_layer(self, ld, xs, params, training):
        c, cfg = ld.class_name, ld.config
        x = xs[0] if xs else None
        if c == "InputLayer":
            return x
        if c == "Convolution2D":
            W = params[0]
            b = params[1] if len(params) > 1 else None
            if x.is_cuda and self.precision == "bf16" and not _native.torch_fallback_allowed():
                y = HipConv2dFn.apply(x, W, b)
            else:
                y = F.conv2d(x, W, b, padding=cfg["nb_row"] // 2)
            return _act(y, cfg.get("activation"))
        if c == "Flatten":
            return x.reshape(x.shape[0], -1)
        if c == "Bias":
            return x + params[0]
        if c == "PassLogit":
            return torch.cat([x, (x @ params[0] + params[1]).unsqueeze(-1)], dim=-1)
        if c == "Activation":
            return _act(x, cfg["activation"])
        if c == "Dense":
            y = x @ params[0]
            if len(params) > 1:
                y = y + params[1]
            return _act(y, cfg.get("activation"))
        if c == "Dropout":
            return F.dropout(x, cfg.get("p", 0.5), training)
        if c == "BatchNormalization":
            gamma, beta, rmean, rvar = params
            axis = cfg.get("axis", -1) % x.dim()
            eps = cfg.get("epsilon", 1e-3)
            perm = [i for i in range(x.dim()) if i != axis] + [axis]
            xt = x.permute(perm)
            if training:
                red = list(range(xt.dim() - 1))
                mean = xt.mean(red)
                var = xt.var(red, unbiased=False)
                m = cfg.get("momentum", 0.99)
                with torch.no_grad():
                    rmean.mul_(m).add_((1 - m) * mean.detach())
                    rvar.mul_(m).add_((1 - m) * var.detach())
            else:
                mean, var = rmean, rvar
            y = (xt - mean) / torch.sqrt(var + eps) * gamma + beta
            inv = [0] * len(perm)
            for i, p in enumerate(perm):
                inv[p] = i
            return y.permute(inv)
        if c == "Merge":
            mode = cfg.get("mode", "sum")
            if mode == "sum":
                out = xs[0]
                for t in xs[1:]:
                    out = out + t
                return out
            if mode == "mul":
                out = xs[0]
                for t in xs[1:]:
                    out = out * t
                return out
            if mode == "concat":
                return torch.cat(xs, dim=cfg.get("concat_axis", -1))
            raise NotImplementedError("Merge mode %s" % mode)
        raise NotImplementedError("layer %s" % c)

    def forward(self, x, training=False, params=None):
        params = self._views if params is None else params
        by_layer = {}
        i = 0
        for ld in self.layer_defs:
            k = len(self.layer_weights[ld.name])
            by_layer[ld.name] = params[i:i + k]
            i += k
        if not self.functional:
            for ld in self.layer_defs:
                x = self._run_layer(ld, [x], by_layer[ld.name], training)
            return x
        vals = {}
        for ld in self.layer_defs:
            if ld.class_name == "InputLayer":
                vals[ld.name] = x
                continue
            vals[ld.name] = self._run_layer(ld, [vals[n] for n in ld.inbound], by_layer[ld.name],
                                            training)
        return vals[self.output_names[0]]


# --------------------------------------------------------------------------- optimizers

class SGD(object):
    """Keras-1 SGD: lr_t = lr / (1 + decay * iterations); momentum / nesterov optional.
    ``lr`` is a plain float attribute and may be reassigned (the RL trainer flips its sign).
    FOLD: on the GPU without momentum, step the fused trunk's weights inside their repack
    (fused.sgd_fold) instead of in a separate pass (False: the A/B, scripts/dbg/fold_ab.py)."""
    FOLD = True

    def __init__(self, lr=0.01, momentum=0.0, decay=0.0, nesterov=False, **kw):
        self.lr = lr
        self.momentum = momentum
        self.decay = decay
        self.initial_decay = decay
        self.nesterov = nesterov
        self.iterations = 0
        self._velocity = None

    def get_config(self):
        return {"lr": float(self.lr), "momentum": self.momentum, "decay": self.decay,
                "nesterov": self.nesterov}

    def current_lr(self):
        lr = float(self.lr)
        if self.initial_decay > 0:
            lr = lr * (1.0 / (1.0 + self.decay * self.iterations))
        return lr

    def apply(self, net):
        """p -= lr_t * g over the whole flat buffer (one fused kernel on GPU)."""
        lr = self.current_lr()
        if self.momentum and self._velocity is None:
            self._velocity = torch.zeros_like(net.flat)
        fold = getattr(net, "_sgd_fold", None)
        if net.flat.is_cuda and not self.momentum and self.FOLD and fold is not None and \
                fold(lr):
            pass  # the trunk's step rode in its weight repack (fused.sgd_fold)
        elif net.flat.is_cuda:
            from ..ops import hipops as ops
            ops.sgd_(net.flat, net.flat_grad, lr, self.momentum, self._velocity, 0.0,
                     self.nesterov)
        else:
            with torch.no_grad():
                if self.momentum:
                    self._velocity.mul_(self.momentum).add_(net.flat_grad, alpha=-lr)
                    if self.nesterov:
                        net.flat.add_(self._velocity * self.momentum - lr * net.flat_grad)
                    else:
                        net.flat.add_(self._velocity)
                else:
                    net.flat.add_(net.flat_grad, alpha=-lr)
        self.iterations += 1
        net.bump()


# --------------------------------------------------------------------------- callbacks

class Callback(object):
    def __init__(self):
        self.model = None
        self.params = {}

    def set_model(self, model):
        self.model = model

    def set_params(self, params):
        self.params = params

    def on_train_begin(self, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass

    def on_epoch_begin(self, epoch, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass

    def on_batch_begin(self, batch, logs=None):
        pass

    def on_batch_end(self, batch, logs=None):
        pass


class ModelCheckpoint(Callback):
    """Save weights to ``filepath.format(epoch=..., **logs)`` at each epoch end (0-based)."""

    def __init__(self, filepath, monitor="val_loss", verbose=0, save_best_only=False,
                 save_weights_only=True, mode="auto"):
        super(ModelCheckpoint, self).__init__()
        self.filepath = filepath
        self.monitor = monitor
        self.save_best_only = save_best_only
        self.best = np.inf
        self.verbose = verbose

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        path = self.filepath.format(epoch=epoch, **logs)
        if self.save_best_only:
            cur = logs.get(self.monitor)
            if cur is None or cur >= self.best:
                return
            self.best = cur
        if _is_rank0():
            self.model.save_weights(path, overwrite=True)


class History(Callback):
    def on_train_begin(self, logs=None):
        self.epoch = []
        self.history = {}

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


def _is_rank0():
    import torch.distributed as dist
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


# --------------------------------------------------------------------------- objectives

def categorical_crossentropy(y_true, y_pred):
    p = y_pred / y_pred.sum(-1, keepdim=True)
    p = p.clamp(EPSILON, 1.0 - EPSILON)
    return -(y_true * torch.log(p)).sum(-1)


def mean_squared_error(y_true, y_pred):
    return ((y_pred - y_true) ** 2).mean(-1)


def binary_crossentropy(y_true, y_pred):
    p = y_pred.clamp(EPSILON, 1.0 - EPSILON)
    return -(y_true * torch.log(p) + (1 - y_true) * torch.log(1 - p)).mean(-1)


OBJECTIVES = {"categorical_crossentropy": categorical_crossentropy, "mse": mean_squared_error,
              "mean_squared_error": mean_squared_error,
              "binary_crossentropy": binary_crossentropy}


def _objective(fn, y_true, y_pred, sample_weight=None):
    """Keras-1 weighted objective: mean over all non-batch axes, weights, then batch mean."""
    score = fn(y_true, y_pred)
    if score.dim() > 1:
        score = score.mean(dim=list(range(1, score.dim())))
    if sample_weight is not None:
        score = score * sample_weight
        score = score / (sample_weight != 0).float().mean().clamp_min(1e-12)
    return score.mean()


# --------------------------------------------------------------------------- the Model

class Model(object):
    """Keras-1-like model object (Sequential or functional)."""

    def __init__(self, layers, functional=False, inputs=None, outputs=None, name=None,
                 device=None, seed=None):
        self.layers = layers
        self.functional = functional
        self.name = name or ("sequential_1" if not functional else "model_1")
        self.net = KerasNet(layers, functional, inputs, outputs, device=device, seed=seed)
        self.loss = None
        self.optimizer = None
        self.metrics = []
        self.stop_training = False
        self._plan = None
        self._plan_checked = False
        self.grad_allreduce = None  # set by parallel.dp for data-parallel training

    # ---- shape / misc
    @property
    def input_shape(self):
        return self.net.input_shape

    @property
    def output_shape(self):
        last = self.net.output_names[0] if self.functional else self.layers[-1].name
        return self.net.shapes[last]

    @property
    def uses_learning_phase(self):
        return self.net.uses_learning_phase

    @property
    def device(self):
        return self.net.device

    def to(self, device):
        self.net.to_device(device)
        self._plan, self._plan_checked = None, False
        return self

    @property
    def precision(self):
        return self.net.precision

    def set_precision(self, precision):
        """``"bf16"`` (default: fused HIP kernels) or ``"fp32"`` (reference precision, generic
        executor with fp32 convolutions; no fused plan)."""
        if precision not in PRECISIONS:
            raise ValueError("precision must be one of %s, got %r" % (PRECISIONS, precision))
        self.net.precision = precision
        self._plan, self._plan_checked = None, False
        return self

    # ---- serialisation
    def get_config(self):
        if not self.functional:
            return [ld.to_config() for ld in self.layers]
        layers = []
        for ld in self.layers:
            d = {"class_name": ld.class_name, "name": ld.name, "config": ld.config,
                 "inbound_nodes": [[[n, 0, 0] for n in ld.inbound]] if ld.inbound else []}
            layers.append(d)
        return {"name": self.name, "layers": layers,
                "input_layers": [[n, 0, 0] for n in self.net.input_names],
                "output_layers": [[n, 0, 0] for n in self.net.output_names]}

    def to_json(self, **kw):
        return json.dumps({"class_name": "Model" if self.functional else "Sequential",
                           "keras_version": "1.2.0", "config": self.get_config()}, **kw)

    def get_weights(self):
        return self.net.get_weights()

    def set_weights(self, weights):
        self.net.set_weights(weights)

    def save_weights(self, filepath, overwrite=True):
        if os.path.exists(filepath) and not overwrite:
            raise IOError("%s exists" % filepath)
        tmp = filepath + ".tmp"
        with h5lite.File(tmp, "w") as f:
            f.attrs["layer_names"] = [ld.name.encode("utf-8") for ld in self.layers]
            vals = dict(zip([w for (_, w, _) in self.net.weight_names], self.net.get_weights()))
            for ld in self.layers:
                g = f.create_group(ld.name)
                names = [w for (w, _) in self.net.layer_weights[ld.name]]
                g.attrs["weight_names"] = np.array([n.encode("utf-8") for n in names],
                                                   dtype="S%d" % max([1] + [len(n) for n in
                                                                            names]))
                for n in names:
                    g[n] = vals[n]
        os.replace(tmp, filepath)

    def load_weights(self, filepath, kernel_flip=False):
        """Load a Keras-1 weight file (layer order = the file's layer_names, as Keras does).
        ``kernel_flip`` converts Theano (true convolution) kernels to cross-correlation."""
        f = h5lite.File(filepath)
        names = [n.decode("utf-8") if isinstance(n, bytes) else n for n in
                 f.attrs["layer_names"]]
        file_layers = [n for n in names if len(f[n].attrs.get("weight_names", [])) > 0]
        my_layers = [ld.name for ld in self.layers if self.net.layer_weights[ld.name]]
        if len(file_layers) != len(my_layers):
            raise ValueError("weight file has %d layers with weights, model has %d" %
                             (len(file_layers), len(my_layers)))
        weights = []
        for fl, ml in zip(file_layers, my_layers):
            g = f[fl]
            wn = [w.decode("utf-8") if isinstance(w, bytes) else w for w in
                  g.attrs["weight_names"]]
            arrs = [np.asarray(g[w][()], dtype=np.float32) for w in wn]
            if kernel_flip:
                arrs = [a[:, :, ::-1, ::-1].copy() if a.ndim == 4 else a for a in arrs]
            weights.extend(arrs)
        self.set_weights(weights)

    # ---- compile / train / predict
    def compile(self, loss, optimizer, metrics=None, **kw):
        self.loss = loss
        self.optimizer = optimizer if not isinstance(optimizer, str) else SGD()
        self.metrics = list(metrics or [])

    def _loss_fn(self):
        if callable(self.loss):
            return self.loss
        return OBJECTIVES[self.loss]

    def _plan_for(self):
        if not self._plan_checked:
            from .fused import detect_plan
            self._plan = detect_plan(self) if (self.net.device.type == "cuda" and
                                               self.net.precision == "bf16") else None
            self._plan_checked = True
        return self._plan

    def _to_tensor(self, X):
        if isinstance(X, torch.Tensor):
            t = X
        else:
            X = np.asarray(X)
            t = torch.from_numpy(X if X.dtype in (np.uint8, np.float32) else
                                 X.astype(np.float32))
        return t.to(self.net.device, non_blocking=True)

    def predict(self, X, batch_size=None, verbose=0):
        """Forward pass in chunks of ``batch_size`` rows (default 1024): the fused plan sizes
        its activation buffers for one chunk, not for the whole input."""
        plan = self._plan_for()
        n = len(X)
        bs = int(batch_size or 1024)
        outs = []
        with torch.no_grad():
            for s in range(0, max(n, 1), bs):
                x = self._to_tensor(X[s:s + bs])
                if plan is not None:
                    out = plan.forward(x)
                else:
                    out = self.net.forward(x.float(), training=False)
                outs.append(out.detach().cpu())
        return torch.cat(outs).numpy() if len(outs) > 1 else outs[0].numpy()

    def predict_on_batch(self, X):
        return self.predict(X)

    def train_on_batch(self, X, Y, sample_weight=None):
        if self.optimizer is None:
            raise RuntimeError("compile() the model before training")
        plan = self._plan_for()
        x = self._to_tensor(X)
        y = self._to_tensor(Y).float()
        sw = None if sample_weight is None else self._to_tensor(sample_weight).float()
        result = None
        if plan is not None:
            result = plan.train_step(x, y, self.loss, sw, want_acc="accuracy" in self.metrics)
        if result is None:
            result = self._generic_train_step(x, y, sw)
        loss, acc = result
        if self.grad_allreduce is not None:
            self.grad_allreduce(self.net.flat_grad)
        self.optimizer.apply(self.net)
        if self.metrics:
            return [loss, acc]
        return loss

    def _generic_train_step(self, x, y, sw):
        net = self.net
        # clones: BN running averages are updated in place during the forward, which must not
        # bump the version counter of tensors autograd saved (they would share the flat storage)
        params = [v.detach().clone().requires_grad_() for v in net._views]
        out = net.forward(x.float(), training=True, params=params)
        loss = _objective(self._loss_fn(), y, out, sw)
        grads = torch.autograd.grad(loss, params, allow_unused=True)
        with torch.no_grad():
            for (_, wname, _), v, p in zip(net.weight_names, net._views, params):
                if "_running_" in wname:
                    v.copy_(p)
            for gv, g in zip(net._gviews, grads):
                if g is None:
                    gv.zero_()
                else:
                    gv.copy_(g)
        acc = None
        if "accuracy" in self.metrics:
            acc = _accuracy(y, out.detach())
        return float(loss.detach()), acc

    def test_on_batch(self, X, Y):
        out = torch.from_numpy(np.asarray(self.predict(X)))
        y = torch.as_tensor(np.asarray(Y), dtype=torch.float32)
        loss = float(_objective(self._loss_fn(), y, out))
        if self.metrics:
            return [loss, _accuracy(y, out)]
        return loss

    def evaluate(self, X, Y, batch_size=32, verbose=0):
        return self.test_on_batch(X, Y)

    def fit_generator(self, generator, samples_per_epoch, nb_epoch, verbose=1, callbacks=None,
                      validation_data=None, nb_val_samples=None, **kw):
        callbacks = list(callbacks or [])
        hist = History()
        callbacks = [hist] + callbacks
        for cb in callbacks:
            cb.set_model(self)
            cb.on_train_begin()
        for epoch in range(nb_epoch):
            for cb in callbacks:
                cb.on_epoch_begin(epoch)
            seen, tot_loss, tot_acc, nb = 0, 0.0, 0.0, 0
            while seen < samples_per_epoch:
                X, Y = next(generator)
                r = self.train_on_batch(X, Y)
                loss, acc = (r if isinstance(r, list) else (r, None))
                n = len(X)
                tot_loss += loss * n
                tot_acc += (acc or 0.0) * n
                seen += n
                nb += 1
                for cb in callbacks:
                    cb.on_batch_end(nb, {"loss": loss, "size": n})
            logs = {"loss": tot_loss / max(1, seen)}
            if "accuracy" in self.metrics:
                logs["acc"] = tot_acc / max(1, seen)
            if validation_data is not None and nb_val_samples:
                vseen, vl, va = 0, 0.0, 0.0
                while vseen < nb_val_samples:
                    X, Y = next(validation_data)
                    r = self.test_on_batch(X, Y)
                    l, a = (r if isinstance(r, list) else (r, None))
                    vl += l * len(X)
                    va += (a or 0.0) * len(X)
                    vseen += len(X)
                logs["val_loss"] = vl / vseen
                if "accuracy" in self.metrics:
                    logs["val_acc"] = va / vseen
            for cb in callbacks:
                cb.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        for cb in callbacks:
            cb.on_train_end()
        return hist


def _accuracy(y, out):
    if out.shape[-1] == 1:
        return float(((out > 0.5).float() == y).float().mean())
    return float((y.argmax(-1) == out.argmax(-1)).float().mean())


def Sequential(layers=None, **kw):
    return Model(list(layers or []), functional=False, **kw)


# --------------------------------------------------------------------------- JSON loading

def model_from_json(json_string, custom_objects=None, device=None):
    spec = json.loads(json_string)
    cls = spec.get("class_name", "Sequential")
    cfg = spec["config"]
    if cls == "Sequential":
        layers = [Layer(l["class_name"], l["config"]) for l in cfg]
        return Model(layers, functional=False, device=device)
    if cls == "Model":
        layers = []
        for l in cfg["layers"]:
            inbound = []
            for node in l.get("inbound_nodes", []):
                for ref in node:
                    inbound.append(ref[0])
            c = dict(l["config"])
            c["name"] = l["name"]
            layers.append(Layer(l["class_name"], c, inbound))
        return Model(layers, functional=True,
                     inputs=[r[0] for r in cfg["input_layers"]],
                     outputs=[r[0] for r in cfg["output_layers"]],
                     name=cfg.get("name"), device=device)
    raise ValueError("unsupported Keras model class %s" % cls)
