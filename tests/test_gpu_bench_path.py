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


def _trunk_ref(x, Ws, bs, acts=None, store_bf16=True):
    """fp32 trunk on bf16-rounded weights and layer inputs (autograd through the roundings is
    the identity: straight-through). ``acts``: the kernels' stored activations per layer
    (NCHW fp32), injected as each layer's output — the backward is then fp32 autograd of the
    exact forward point the kernels differentiated."""
    h = x
    for l, (W, b) in enumerate(zip(Ws, bs)):
        hin = h + (_bf(h) - h).detach()
        Wq = W + (_bf(W) - W).detach()
        pre = F.conv2d(hin, Wq, b, padding=W.shape[-1] // 2)
        h = F.relu(pre) if acts is None else _Inject.apply(pre, acts[l], store_bf16)
    return h + (_bf(h) - h).detach()


def _gpu_acts(plan, B):
    from rocalphago_amd.ops import hipops as ops
    out = []
    for a, s in zip(plan.trunk.acts[1:], plan.trunk.specs):
        out.append(ops.unpack(a[:B], s.cout, (a.shape[1] - plan.S) // 2))
    return out


@pytest.mark.parametrize("augment", [False, True])
def test_north_star_sl_step_matches_fp32(cuda, augment):
    """Gradients of one bench-path step vs fp32 autograd, two references:
    (a) fp32 autograd at the kernels' own forward point (their stored bf16 activations injected
        as each layer's output, ReLU masks from them, dL/d(pre-activation) rounded to bf16 where
        the kernels store it) — pins the whole backward arithmetic: head, dgrad, fp32
        accumulation, fp16 block-scaled partial slabs reduced inside the next dgrad launch.
        Every tensor within 2e-2. Without the bf16 storage rounding the top layer's bias
        gradient (a sum that cancels to a few % of its terms at init) differs by ~5 %.
    (b) an independent fp32 forward + backward (bf16-rounded weights / layer inputs) — within
        0.25. Its forward activations differ from the kernels' by 0.2-0.6 % (accumulation order
        changes bf16 roundings, scripts/dbg/bench_path_err.py), and at random init the 12-layer
        trunk's activations are nearly constant over the board, so the gradient
        sum_p x(p) (p(p) - y(p)) cancels to a few % of its terms and amplifies that into ~12 %
        per tensor (3 layers: 1-4 %; identical with fp32 partial slabs and without deferred
        reductions, i.e. not a kernel error).
    ``augment``: the bench's random dihedral augmentation (all 8 transforms, drawn by the
    sl_batch kernel and applied while packing the input) -- the reference applies the same
    per-sample transforms to the planes and the targets with numpy."""
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
    cases = (("kernels' forward point, bf16-stored grads", True, True, 2e-2),
             ("kernels' forward point, fp32 grads", True, False, 0.1),
             ("independent fp32", False, False, 0.25))
    for label, inject, store, bound in cases:
        leaf = {n: [p.clone().requires_grad_(True) for p in ps] for n, ps in params.items()}
        h = _trunk_ref(x, [leaf[n][0] for n in plan.conv_names],
                       [leaf[n][1] for n in plan.conv_names], acts if inject else None, store)
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
