"""Fused HIP execution plans for the two flagship architectures.

``detect_plan`` pattern-matches a kerasish Sequential model:

  PolicyPlan:  [Conv2D 'same' (+ReLU)]* -> Conv2D 1x1 (1 filter, linear) -> Flatten -> Bias ->
               [PassLogit] -> Activation(softmax)       (CNNPolicy, reference policy.py:96-136)
  ValuePlan:   [Conv2D 'same' (+ReLU)]* -> Conv2D 1x1 (1 filter) -> Flatten -> Dense(H) ->
               Dense(1, tanh)                          (CNNValue / reference value.py:14-28)
  ResnetPlan:  (functional) Conv2D linear -> [n_skip x (BN -> ReLU -> Conv2D linear) + sum-merge]*
               -> ReLU -> Conv2D 1x1 -> Flatten -> Bias -> softmax
                                                       (ResnetPolicy, reference policy.py:196-244)

and executes them on the HIP engine (models/engine.py): one packed-input kernel (uint8 or fp32
planes, optional gather + dihedral transform), one MFMA conv launch per layer, the fused head
(softmax + loss + dL/dz in one kernel), per-layer wgrad/dgrad, with gradients written straight
into the model's flat fp32 gradient buffer (ready for one all-reduce and the fused SGD kernel).
"""
import torch

from ..ops import hipops as ops
from .engine import BNSpec, ConvSpec, HipTrunk, PolicyHeadEngine, ResTrunk, ValueHeadEngine


def _conv_ok(ld):
    c = ld.config
    return (ld.class_name == "Convolution2D" and c.get("border_mode") == "same" and
            c["nb_row"] == c["nb_col"] and c["nb_row"] % 2 == 1 and
            tuple(c.get("subsample", (1, 1))) == (1, 1) and
            c.get("activation", "linear") in ("relu", "linear"))


def detect_plan(model):
    if model.functional:
        return _detect_resnet(model)
    L = model.layers
    n = 0
    while n < len(L) and L[n].class_name == "Convolution2D":
        n += 1
    if n < 2 or not all(_conv_ok(ld) for ld in L[:n]):
        return None
    head = L[n - 1]
    if head.config["nb_filter"] != 1 or head.config["nb_row"] != 1 or \
            head.config.get("activation", "linear") != "linear":
        return None
    if L[n - 2].config["nb_row"] > 3:
        return None
    rest = [ld.class_name for ld in L[n:]]
    S = model.input_shape[-1]
    if S > 25 or model.input_shape[-2] != S:
        return None
    if rest == ["Flatten", "Bias", "Activation"] and L[-1].config["activation"] == "softmax":
        return PolicyPlan(model, L[:n - 1], head, L[n + 1])
    if rest == ["Flatten", "Bias", "PassLogit", "Activation"] and \
            L[-1].config["activation"] == "softmax":
        return PolicyPlan(model, L[:n - 1], head, L[n + 1], L[n + 2])
    if rest == ["Flatten", "Dense", "Dense"] and L[-1].config["output_dim"] == 1 and \
            L[-1].config.get("activation") == "tanh" and \
            L[n + 1].config.get("activation", "linear") in ("relu", "linear", "tanh"):
        return ValuePlan(model, L[:n - 1], head, L[n + 1], L[n + 2])
    return None


class _TrunkPlan(object):
    def __init__(self, model, convs, head_conv):
        net = model.net
        self.model = model
        self.net = net
        specs = []
        for ld in convs:
            W = net.params_of(ld.name)[0]
            specs.append(ConvSpec(ld.config["nb_row"], W.shape[1], W.shape[0],
                                  ld.config.get("activation", "linear") == "relu"))
        self.S = model.input_shape[-1]
        self.trunk = HipTrunk(specs, self.S, net.device)
        self.conv_names = [ld.name for ld in convs]
        self.head_name = head_conv.name
        self.K = specs[-1].cout
        net._sgd_fold = self.sgd_fold  # the optimizer's step folded into the weight repack

    # the fold pays only while the rest of the flat buffer is one or two plain SGD launches: the
    # ResNet's BN parameters sit between its conv layers, and stepping them range by range took
    # 20 launches (90 us per step) against one 11 us pass over the whole buffer
    # (profiles/sgd_fold_r6.txt)
    SGD_FOLD_MAX_GAPS = 2

    def sgd_fold(self, lr):
        """SGD step of the whole flat buffer with the trunk's part folded into its repack
        (engine._PackedConvs.sgd_pack) and the rest by the plain kernel. False: not possible
        (e.g. the packing tables are not built yet, or the rest is too fragmented), nothing
        done."""
        from .engine import complement
        Ws, bs = self._params()
        net = self.net
        ver = (net.version + 1, net.flat._version)  # after the optimizer's bump()
        ranges = self.trunk.sgd_pack(Ws, bs, net.flat, net.flat_grad, lr, ver,
                                     max_gaps=self.SGD_FOLD_MAX_GAPS, step_rest=True)
        if ranges is None:
            return False
        for a, b in complement(ranges, net.flat.numel()):
            ops.sgd_(net.flat[a:b], net.flat_grad[a:b], lr)
        self.folded_steps = getattr(self, "folded_steps", 0) + 1
        return True

    def sync_weights(self):
        """Repack the bf16 trunk weights if the fp32 masters changed (a replayed graph reads the
        packed copies at fixed addresses)."""
        Ws, bs = self._params()
        self.trunk.sync_weights(Ws, bs, self.net.weights_version())

    def _params(self):
        Ws, bs = [], []
        for name in self.conv_names:
            p = self.net.params_of(name)
            Ws.append(p[0])
            bs.append(p[1] if len(p) > 1 else None)
        return Ws, bs

    def _grads(self):
        dWs, dbs = [], []
        for name in self.conv_names:
            g = self.net.grads_of(name)
            dWs.append(g[0])
            dbs.append(g[1] if len(g) > 1 else None)
        return dWs, dbs

    def prepare(self, x, index=None, transforms=None):
        """Pack input planes [N, F, S, S] (uint8 or fp32, on device), or bit-packed positions
        [N, S, S] int64 (training/replay.py), into the trunk input."""
        B = x.shape[0] if index is None else index.shape[0]
        self.trunk.ensure_batch(B)
        Ws, bs = self._params()
        self.trunk.sync_weights(Ws, bs, self.net.weights_version())
        if x.dtype not in (torch.uint8, torch.float32, torch.int64):
            x = x.float()
        # planes beyond the first conv's inputs (e.g. the value net's colour plane in the search's
        # shared input) are skipped in place by the packer
        ops.pack_input(x, self.trunk.input_buffer(B), self.trunk.halo[0],
                       index=index, transforms=transforms, nplanes=self.trunk.specs[0].cin)
        return B

    def head_params(self):
        p = self.net.params_of(self.head_name)
        w = p[0].reshape(-1)
        b0 = p[1] if len(p) > 1 else None
        return w, b0

    def head_grads(self):
        g = self.net.grads_of(self.head_name)
        return g[0].reshape(-1), (g[1] if len(g) > 1 else torch.zeros(1, device=self.net.device))

    def layer_offsets(self):
        """Start offset (elements) of each trunk conv layer's params in net.flat."""
        base = self.net.flat.data_ptr()
        return [(self.net.params_of(n)[0].data_ptr() - base) // 4 for n in self.conv_names]


class PolicyPlan(_TrunkPlan):
    def __init__(self, model, convs, head_conv, bias_layer, pass_layer=None):
        super(PolicyPlan, self).__init__(model, convs, head_conv)
        self.bias_name = bias_layer.name
        self.pass_name = pass_layer.name if pass_layer is not None else None
        self.head = PolicyHeadEngine(self.trunk, self.K, pass_logit=pass_layer is not None)

    def _pass_params(self):
        return self.net.params_of(self.pass_name) if self.pass_name else None

    def forward(self, x, index=None, transforms=None, clone=True):
        """Move probabilities [B, S*S (+1)]. clone=False returns the head's own output buffer
        (valid until the next forward of this plan; the search copies it to the host at once)."""
        B = self.prepare(x, index, transforms)
        self.trunk.forward(B)
        w, b0 = self.head_params()
        pb = self.net.params_of(self.bias_name)[0]
        out = self.head.forward(B, w, b0, pb, pass_params=self._pass_params())
        return out.clone() if clone else out

    @staticmethod
    def loss_mode(loss):
        if loss == "categorical_crossentropy":
            return 1
        return getattr(loss, "_rag_head_mode", None)

    def train_step(self, x, y, loss, sw=None, want_acc=False, labels=None, index=None,
                   transforms=None):
        mode = self.loss_mode(loss)
        if mode is None:
            return None
        if labels is None:
            # one-hot targets only (the reference's CE / REINFORCE targets); else generic path
            if not bool(((y.sum(1) == 1) & (y.max(1).values == 1)).all()):
                return None
            labels = y.argmax(1)
        B = self.prepare(x, index, transforms)
        norm = 1.0
        if sw is not None:
            norm = float((sw != 0).float().mean().clamp_min(1e-12))
        self.fwd_bwd(B, labels, sw, mode, 1.0 / (B * norm))
        lossv = float(self.head.loss[:B].mean()) / norm
        acc = float(self.head.hit[:B].mean()) if want_acc else None
        return lossv, acc

    def fwd_bwd(self, B, labels, sw, mode, gscale, on_layer_grads=None, metrics=None):
        """Forward + fused loss + full backward into net.flat_grad (no host syncs). metrics:
        fp32 [2] device accumulator of (loss sum, top-1 hits), updated in the head kernel."""
        self.trunk.forward(B, training=True)
        w, b0 = self.head_params()
        pb = self.net.params_of(self.bias_name)[0]
        self.head.forward(B, w, b0, pb, labels=labels, sweight=sw, mode=mode, gscale=gscale,
                          pass_params=self._pass_params(), acc=metrics)
        try:
            if self.pass_name:
                dW, db = self.net.grads_of(self.pass_name)
                self.head.pass_grads(B, dW, db)
            dw, db0 = self.head_grads()
            dpb = self.net.grads_of(self.bias_name)[0]
            self.head.backward(B, w, self.head.dz[:B], dw, db0, dpb)
        except BaseException:
            self.head.reset_metrics()  # a retrying caller's next forward must not raise
            raise
        dWs, dbs = self._grads()
        self.trunk.backward(B, dWs, dbs, on_layer_done=on_layer_grads)


class ValuePlan(_TrunkPlan):
    def __init__(self, model, convs, head_conv, dense1, dense2):
        super(ValuePlan, self).__init__(model, convs, head_conv)
        self.d1, self.d2 = dense1.name, dense2.name
        self.act1 = dense1.config.get("activation", "linear")
        self.head = ValueHeadEngine(self.trunk, self.K)

    def _mlp(self, z, params):
        W1, b1, W2, b2 = params
        return self._mlp_tail(z @ W1 + b1, W2, b2)

    def _mlp_tail(self, h, W2, b2):
        if self.act1 == "relu":
            h = torch.relu(h)
        elif self.act1 == "tanh":
            h = torch.tanh(h)
        return torch.tanh(h @ W2 + b2)

    def _dense_params(self):
        return self.net.params_of(self.d1) + self.net.params_of(self.d2)

    def forward(self, x, index=None, transforms=None):
        B = self.prepare(x, index, transforms)
        self.trunk.forward(B)
        w, b0 = self.head_params()
        z = self.head.conv_out(B, w, b0)
        W1, b1, W2, b2 = self._dense_params()
        if self.act1 in ops.MLP_ACTS:
            # inference: one fused HIP kernel instead of two library GEMMs + elementwise ops
            return ops.value_mlp_fwd(z, W1, b1, W2, b2, act=self.act1)
        return self._mlp(z, (W1, b1, W2, b2))

    def train_step(self, x, y, loss, sw=None, want_acc=False, index=None, transforms=None):
        if loss not in ("mse", "mean_squared_error"):
            return None
        B = self.prepare(x, index, transforms)
        lossv = self.fwd_bwd(B, y.reshape(B, -1), sw)
        return float(lossv), None

    def fwd_bwd(self, B, y, sw=None, on_layer_grads=None):
        self.trunk.forward(B, training=True)
        w, b0 = self.head_params()
        z = self.head.conv_out(B, w, b0)
        W1, b1, W2, b2 = self._dense_params()
        # the whole MLP head (forward, MSE loss, dW1 / db1 / dW2 / db2 / dz) on HIP kernels
        # (ops.value_mlp_train: head.hip forward partials + value_bwd.hip)
        gW1, gb1, gW2, gb2 = self.net.grads_of(self.d1) + self.net.grads_of(self.d2)
        dz = self.head.dz_buffer(B)
        yv = y.reshape(-1).float().contiguous()
        swv = sw.reshape(-1).float().contiguous() if sw is not None else None
        lossv = ops.value_mlp_train(z, W1, b1, W2, b2, yv, swv, self.act1, gW1, gb1, gW2, gb2,
                                    dz=dz).sum()
        dw, db0 = self.head_grads()
        self.head.backward_conv(B, w, dz, dw, db0)
        dWs, dbs = self._grads()
        self.trunk.backward(B, dWs, dbs, on_layer_done=on_layer_grads)
        return lossv.detach()


def _detect_resnet(model):
    """Match ResnetPolicy's functional graph (topologically ordered layer list)."""
    L = model.layers
    S = model.input_shape[-1] if model.input_shape else None
    if not S or S > 25 or len(L) < 8 or L[0].class_name != "InputLayer":
        return None

    def conv(ld, src, ks=None):
        return (_conv_ok(ld) and ld.inbound == [src] and
                ld.config.get("activation", "linear") == "linear" and
                (ks is None or ld.config["nb_row"] == ks))

    def bn_ok(ld, src):
        c = ld.config
        return (ld.class_name == "BatchNormalization" and ld.inbound == [src] and
                c.get("mode", 0) == 0 and c.get("axis", -1) in (-1, 3))

    def act(ld, src, name):
        return (ld.class_name == "Activation" and ld.inbound == [src] and
                ld.config["activation"] == name)

    if not conv(L[1], L[0].name):
        return None
    convs, bns, units = [L[1]], [], []
    cur, i = L[1].name, 2
    while i < len(L) and L[i].class_name == "BatchNormalization":
        path, n = cur, 0
        while i + 2 < len(L) and bn_ok(L[i], path) and act(L[i + 1], L[i].name, "relu") and \
                conv(L[i + 2], L[i + 1].name) and L[i + 2].config["nb_row"] <= 7:
            bns.append(L[i])
            convs.append(L[i + 2])
            path = L[i + 2].name
            n += 1
            i += 3
        m = L[i] if i < len(L) else None
        if n == 0 or m is None or m.class_name != "Merge" or \
                m.config.get("mode", "sum") != "sum" or sorted(m.inbound) != sorted([cur, path]):
            return None
        units.append(n)
        cur, i = m.name, i + 1
    rest = L[i:]
    pl = rest[4] if len(rest) == 6 and rest[4].class_name == "PassLogit" and \
        rest[4].inbound == [rest[3].name] else None
    if not units or len(rest) != (6 if pl is not None else 5) or \
            not act(rest[0], cur, "relu") or \
            not conv(rest[1], rest[0].name, 1) or rest[1].config["nb_filter"] != 1 or \
            rest[2].class_name != "Flatten" or rest[3].class_name != "Bias" or \
            not act(rest[-1], rest[-2].name, "softmax"):
        return None
    K = L[1].config["nb_filter"]
    if any(c.config["nb_filter"] != K for c in convs):
        return None
    return ResnetPlan(model, convs, bns, units, rest[1], rest[3], pl)


class ResnetPlan(PolicyPlan):
    """ResnetPolicy on the HIP engine: ResTrunk (column BN + ReLU kernels, residual conv
    epilogue) + the same fused policy head / loss as PolicyPlan. Training steps use batch
    statistics (and update the running averages); forward / evaluation use the running ones,
    like Keras' learning phase."""

    def __init__(self, model, convs, bns, units, head_conv, bias_layer, pass_layer=None):
        net = model.net
        self.model, self.net = model, net
        specs = []
        for ld in convs:
            W = net.params_of(ld.name)[0]
            specs.append(ConvSpec(ld.config["nb_row"], W.shape[1], W.shape[0], False))
        bspecs = [BNSpec(ld.config.get("epsilon", 1e-3), ld.config.get("momentum", 0.99),
                         net.params_of(ld.name), net.grads_of(ld.name)) for ld in bns]
        self.S = model.input_shape[-1]
        self.trunk = ResTrunk(specs, units, bspecs, self.S, net.device)
        self.conv_names = [ld.name for ld in convs]
        self.head_name = head_conv.name
        self.K = specs[-1].cout
        net._sgd_fold = self.sgd_fold  # the optimizer's step folded into the weight repack
        self.bias_name = bias_layer.name
        self.pass_name = pass_layer.name if pass_layer is not None else None
        self.head = PolicyHeadEngine(self.trunk, self.K, pass_logit=pass_layer is not None)
