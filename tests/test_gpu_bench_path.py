"""The exact benchmark path pinned against fp32 PyTorch.

* One SL training step of the north-star policy (48 planes -> 5x5 conv 192, 11 x 3x3 conv 192,
  1x1 head + position bias + softmax; B = 256) through SupervisedTrainer — the bench.py path
  with the default kernels: deferred fp16 block-scaled wgrad partial slabs reduced inside the
  next dgrad launch — against fp32 autograd of the same network on the same batch. The
  reference consumes bf16-rounded weights and bf16-rounded layer inputs (what the MFMA kernels
  read); everything else, including all accumulation and the whole backward, is fp32.
* The same step on 2 data-parallel ranks (gloo, both on this GPU, launched as child processes)
  leaves bit-identical replicas whose one-step update equals the single-process update on the
  concatenated batch (reference: supervised_policy_trainer.py:249-250 trains one replica).
* The value-net train step against fp32 autograd on the same bf16-rounded trunk inputs.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES, VALUE_FEATURES
from rocalphago_amd.models import kerasish as K
from rocalphago_amd.models.policy import CNNPolicy
from rocalphago_amd.models.value import CNNValue
from rocalphago_amd.training.data import DeviceDataset
from rocalphago_amd.training.supervised import SupervisedTrainer

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bf(t):
    return t.to(torch.bfloat16).float()


def _rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


class _Inject(torch.autograd.Function):
    """Forward: the kernels' own stored activation of a layer (so the next layer consumes
    exactly what the MFMA kernels consumed); backward: the ReLU derivative from that same
    activation, applied to the fp32 gradient."""

    @staticmethod
    def forward(ctx, pre, act, store_bf16):
        ctx.save_for_backward(act)
        ctx.store_bf16 = store_bf16
        return act.clone()

    @staticmethod
    def backward(ctx, g):
        act, = ctx.saved_tensors
        g = g * (act > 0).to(g.dtype)
        # the kernels keep dL/d(pre-activation) of every layer in bf16 buffers
        return (_bf(g) if ctx.store_bf16 else g), None, None


def _wino_corr(x, w):
    """3x3 'same' correlation of x [B, C, H, W] with w [N, C, 3, 3] computed the way
    conv_wino.hip does: Winograd F(2,3) along the width, the transformed inputs
    V = (d0 - d2, d1 + d2, d2 - d1, d1 - d3) and weights U = (g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2)
    each rounded to bf16 once (U from the fp32 masters), then fp32 products and sums."""
    B, C, H, W = x.shape
    T = (W + 1) // 2
    xp = F.pad(x, (1, 2 * T + 1 - W, 1, 1))
    d = [xp[..., k:k + 2 * T:2] for k in range(4)]
    V = [_bf(d[0] - d[2]), _bf(d[1] + d[2]), _bf(d[2] - d[1]), _bf(d[1] - d[3])]
    g0, g1, g2 = w[..., 0], w[..., 1], w[..., 2]
    U = [_bf(g0), _bf((g0 + g1 + g2) / 2), _bf((g0 - g1 + g2) / 2), _bf(g2)]
    M = [F.conv2d(V[q], U[q].unsqueeze(-1)) for q in range(4)]
    y = torch.stack([M[0] + M[1] + M[2], M[1] - M[2] - M[3]], -1)
    return y.reshape(B, -1, H, 2 * T)[..., :W]


class _WinoConv(torch.autograd.Function):
    """3x3 conv on bf16 weights whose forward (``fwd``) and / or input gradient (``dgrad``: with
    the flipped, transposed weights) are computed the Winograd way (_wino_corr); weight / bias
    gradients plain fp32."""

    @staticmethod
    def forward(ctx, x, W, b, fwd, dgrad):
        ctx.save_for_backward(x, W)
        ctx.dgrad = dgrad
        if fwd:
            return _wino_corr(x, W) + b.view(1, -1, 1, 1)
        return F.conv2d(x, _bf(W), b, padding=1)

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        if ctx.dgrad:
            gx = _wino_corr(g, W.flip(2, 3).transpose(0, 1))
        else:
            gx = torch.nn.grad.conv2d_input(x.shape, _bf(W), g, padding=1)
        gw = torch.nn.grad.conv2d_weight(x, W.shape, g, padding=1)
        return gx, gw, g.sum((0, 2, 3)), None, None


def _trunk_ref(x, Ws, bs, acts=None, store_bf16=True, wino=None):
    """fp32 trunk on bf16-rounded weights and layer inputs (autograd through the roundings is
    the identity: straight-through). ``acts``: the kernels' stored activations per layer
    (NCHW fp32), injected as each layer's output — the backward is then fp32 autograd of the
    exact forward point the kernels differentiated. ``wino``: (forward, dgrad) per-layer flags
    of the layers the trunk ran through conv_wino.hip, computed the Winograd way here (the
    forward only without ``acts``)."""
    h = x
    for l, (W, b) in enumerate(zip(Ws, bs)):
        hin = h + (_bf(h) - h).detach()
        Wq = W + (_bf(W) - W).detach()
        if wino is not None and (wino[0][l] or wino[1][l]):
            pre = _WinoConv.apply(hin, W, b, acts is None and wino[0][l], wino[1][l])
        else:
            pre = F.conv2d(hin, Wq, b, padding=W.shape[-1] // 2)
        h = F.relu(pre) if acts is None else _Inject.apply(pre, acts[l], store_bf16)
    return h + (_bf(h) - h).detach()


def _gpu_acts(plan, B):
    from rocalphago_amd.ops import hipops as ops
    out = []
    for a, s in zip(plan.trunk.acts[1:], plan.trunk.specs):
        out.append(ops.unpack(a[:B], s.cout, (a.shape[1] - plan.S) // 2))
    return out


@pytest.mark.parametrize("augment,defer", [(False, True), (True, True), (False, False)])
def test_north_star_sl_step_matches_fp32(cuda, augment, defer, monkeypatch):
    """Gradients of one bench-path step vs fp32 autograd, two references:
    (a) fp32 autograd at the kernels' own forward point (their stored bf16 activations injected
        as each layer's output, ReLU masks from them, dL/d(pre-activation) rounded to bf16 where
        the kernels store it) — pins the whole backward arithmetic: head, dgrad, fp32
        accumulation, fp16 block-scaled partial slabs reduced inside the next dgrad launch.
        Every tensor within 2e-2; Winograd dgrads (when the trunk runs them) are computed as
        conv_wino.hip computes them (bf16 V and U, _wino_corr). Without the bf16 storage
        rounding the top layer's bias gradient (a sum that cancels to a few % of its terms at
        init) differs by ~5 %, and without the Winograd roundings the top layers' weight
        gradients by ~3.6 % (same cancellation: ~0.35 % noise in g, amplified ~10x).
    (b) an independent fp32 forward + backward (bf16-rounded weights / layer inputs) with the
        Winograd layers' forward (and dgrad) rounded as the kernels round them — within 0.25.
        Its forward activations differ from the kernels' by 0.2-0.6 % (accumulation order
        changes bf16 roundings, scripts/dbg/bench_path_err.py), and at random init the 12-layer
        trunk's activations are nearly constant over the board, so the gradient
        sum_p x(p) (p(p) - y(p)) cancels to a few % of its terms and amplifies that into ~12 %
        per tensor (3 layers: 1-4 %; identical with fp32 partial slabs and without deferred
        reductions, i.e. not a kernel error).
    (c) the same with plain direct-convolution arithmetic everywhere — within 0.4: the Winograd
        roundings (bf16 V and U, ~0.3 % relative per layer against ~0.2 % for the direct kernel)
        go through the same amplification (0.28 measured on MI355X with Winograd dgrads too).
    ``augment``: the bench's random dihedral augmentation (all 8 transforms, drawn by the
    sl_batch kernel and applied while packing the input) -- the reference applies the same
    per-sample transforms to the planes and the targets with numpy. ``defer=False``
    (HipTrunk.DEFER_REDUCE False): the wgrad reductions run as their own launches and the
    dgrads of the Winograd layers run Winograd too."""
    if not defer:
        from rocalphago_amd.models.engine import HipTrunk
        monkeypatch.setattr(HipTrunk, "DEFER_REDUCE", False)
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=12, device=cuda,
                    seed=1234)
    model = pol.model
    model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.003),
                  metrics=["accuracy"])
    ds = DeviceDataset.synthetic(1024, 48, 19, cuda, seed=17)
    from rocalphago_amd.ops import hipops as ops
    from rocalphago_amd.training.data import TRANSFORM_NAMES, apply_transform_np
    tr = SupervisedTrainer(model, ds, 256, TRANSFORM_NAMES if augment else ["noop"], None,
                           seed=5)
    plan = tr.plan
    assert plan is not None and len(plan.conv_names) == 12
    net = model.net
    params = {n: [p.detach().clone() for p in net.params_of(n)]
              for n in plan.conv_names + [plan.head_name, plan.bias_name]}
    g = torch.Generator(device=cuda)
    g.manual_seed(3)
    idx = torch.randint(0, ds.N, (256,), generator=g, device=cuda)
    # the transforms and transformed targets the step will draw (a pure function of the
    # trainer seed and the optimizer iteration, batch.hip)
    tf, labels = ops.sl_batch(idx.long().contiguous(), ds.labels, ds.tf_table, tr.sym, tr.seed,
                              getattr(model.optimizer, "iterations", 0))
    tf, labels = tf.clone(), labels.clone()
    tr.step(idx)
    torch.cuda.synchronize()
    got = {n: [t.detach().clone() for t in net.grads_of(n)] for n in params}
    acts = _gpu_acts(plan, 256)
    xs = ds.states[idx].cpu().numpy()
    tfs = tf.cpu().numpy()
    if augment:
        assert len(set(tfs.tolist())) == 8  # every transform drawn in a batch of 256
    x = torch.from_numpy(np.stack([apply_transform_np(xs[b], int(tfs[b]))
                                   for b in range(256)]).astype(np.float32)).to(cuda)
    # the 3x3 192 -> 192 layers run forward (and dgrad, unless it carries a deferred wgrad
    # reduction) through the Winograd kernel at B = 256; references (a) and (b) compute them the
    # same way (_wino_corr), the others do not
    wf = plan.trunk.wino_plan(256)
    assert wf == [False] + [True] * 11
    assert plan.trunk.wino_dgrad == (not defer)
    wino = (wf, [w and plan.trunk.wino_dgrad for w in wf])
    cases = (("kernels' forward point, bf16-stored grads", True, True, True, 2e-2),
             ("kernels' forward point, fp32 grads", True, False, False, 0.1),
             ("independent fp32, Winograd roundings", False, False, True, 0.25),
             ("independent fp32, direct arithmetic", False, False, False, 0.4))
    for label, inject, store, wi, bound in cases:
        leaf = {n: [p.clone().requires_grad_(True) for p in ps] for n, ps in params.items()}
        h = _trunk_ref(x, [leaf[n][0] for n in plan.conv_names],
                       [leaf[n][1] for n in plan.conv_names], acts if inject else None, store,
                       wino if wi else None)
        hw, hb = leaf[plan.head_name]
        z = F.conv2d(h, hw, hb).reshape(256, -1) + leaf[plan.bias_name][0]
        loss = F.cross_entropy(z, labels)
        loss.backward()
        errs = {}
        for n in params:
            for k, (a, p) in enumerate(zip(got[n], leaf[n])):
                if n == plan.head_name and k == 1:
                    # the head's scalar bias: softmax gradients sum to zero over the board, so its
                    # true gradient is 0 up to rounding noise — compare against the batch scale
                    errs["%s/%d" % (n, k)] = float((a - p.grad).abs().max()) / 1e-3
                    continue
                errs["%s/%d" % (n, k)] = _rel(a, p.grad)
        worst = max(errs.values())
        print("[%s] per-tensor gradient rel. error (max %.3g):" % (label, worst),
              " ".join("%s=%.2g" % kv for kv in errs.items()))
        assert worst <= bound, (label, errs)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_two_ranks_one_step_matches_single_process(cuda):
    env = dict(os.environ, RAG_DIST_BACKEND="gloo", DP_CHECK_STEPS="1", DP_CHECK_TOL="1e-3",
               OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dp_replica_job.py")]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-3000:]
    import json
    res = json.loads(lines[-1])
    print(res)
    assert res["replicas_identical"]
    assert res["update_rel_diff_vs_single_process"] <= 1e-3


def test_value_step_matches_fp32(cuda):
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    val = CNNValue(VALUE_FEATURES, board=19, filters_per_layer=64, layers=5, device=cuda,
                   seed=7)
    model = val.model
    model.compile(loss="mse", optimizer=K.SGD(lr=0.01))
    plan = model._plan_for()
    assert plan is not None
    net = model.net
    names = plan.conv_names + [plan.head_name, plan.d1, plan.d2]
    params = {n: [p.detach().clone() for p in net.params_of(n)] for n in names}
    rng = np.random.RandomState(2)
    B = 64
    X = torch.from_numpy((rng.rand(B, 49, 19, 19) > 0.65).astype(np.float32)).to(cuda)
    Y = torch.from_numpy(rng.uniform(-1, 1, (B, 1)).astype(np.float32)).to(cuda)
    plan.train_step(X, Y, "mse")
    torch.cuda.synchronize()
    got = {n: [t.detach().clone() for t in net.grads_of(n)] for n in names}
    leaf = {n: [p.clone().requires_grad_(True) for p in ps] for n, ps in params.items()}
    h = _trunk_ref(X, [leaf[n][0] for n in plan.conv_names],
                   [leaf[n][1] for n in plan.conv_names], _gpu_acts(plan, B))
    hw, hb = leaf[plan.head_name]
    z = F.conv2d(h, hw, hb).reshape(B, -1)
    W1, b1 = leaf[plan.d1]
    W2, b2 = leaf[plan.d2]
    a = z @ W1 + b1
    a = {"relu": F.relu, "tanh": torch.tanh}.get(plan.act1, lambda t: t)(a)
    v = torch.tanh(a @ W2 + b2)
    loss = ((v - Y) ** 2).mean()
    loss.backward()
    errs = {}
    for n in names:
        for k, (g_, p) in enumerate(zip(got[n], leaf[n])):
            errs["%s/%d" % (n, k)] = _rel(g_, p.grad)
    print("value grads rel. error:", " ".join("%s=%.2g" % kv for kv in errs.items()))
    assert max(errs.values()) <= 2e-2, errs
