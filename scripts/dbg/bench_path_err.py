"""Diagnose the SL bench path vs fp32 autograd: per-layer activation / gradient errors for the
north-star policy (or a shallower one), with the wgrad partial format and deferral from env."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES  # noqa: E402
from rocalphago_amd.models import kerasish as K  # noqa: E402
from rocalphago_amd.models.policy import CNNPolicy  # noqa: E402
from rocalphago_amd.ops import hipops as ops  # noqa: E402
from rocalphago_amd.training.data import DeviceDataset  # noqa: E402
from rocalphago_amd.training.supervised import SupervisedTrainer  # noqa: E402


def bf(t):
    return t.to(torch.bfloat16).float()


def rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


def main():
    layers = int(os.environ.get("L", "12"))
    B = int(os.environ.get("B", "256"))
    torch.backends.cudnn.allow_tf32 = False
    dev = torch.device("cuda")
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=layers, device=dev,
                    seed=1234)
    model = pol.model
    model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.003))
    ds = DeviceDataset.synthetic(1024, 48, 19, dev, seed=17)
    tr = SupervisedTrainer(model, ds, B, ["noop"], None, seed=5)
    plan = tr.plan
    net = model.net
    names = plan.conv_names + [plan.head_name, plan.bias_name]
    params = {n: [p.detach().clone() for p in net.params_of(n)] for n in names}
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    idx = torch.randint(0, ds.N, (B,), generator=g, device=dev)
    tr.step(idx)
    torch.cuda.synchronize()
    got = {n: [t.detach().clone() for t in net.grads_of(n)] for n in names}
    acts = [ops.unpack(a[:B], a.shape[-1], (a.shape[1] - 19) // 2) for a in plan.trunk.acts[1:]]
    leaf = {n: [p.clone().requires_grad_(True) for p in ps] for n, ps in params.items()}
    h = ds.states[idx].float()
    ref_acts = []
    for n in plan.conv_names:
        W, b = leaf[n]
        hin = h + (bf(h) - h).detach()
        Wq = W + (bf(W) - W).detach()
        h = F.relu(F.conv2d(hin, Wq, b, padding=W.shape[-1] // 2))
        h.retain_grad()
        ref_acts.append(h)
    hq = h + (bf(h) - h).detach()
    hw, hb = leaf[plan.head_name]
    z = F.conv2d(hq, hw, hb).reshape(B, -1) + leaf[plan.bias_name][0]
    loss = F.cross_entropy(z, ds.labels[idx])
    loss.backward()
    out = {"layers": layers, "B": B, "env": {k: v for k, v in os.environ.items()
                                             if k.startswith("RAG_")}}
    out["act_rel"] = [round(rel(a[:, :r.shape[1]], r.detach()), 5) for a, r in
                      zip(acts, ref_acts)]
    out["act_norm"] = [round(float(r.detach().norm()), 4) for r in ref_acts]
    out["grad_rel"] = {n: [round(rel(a, p.grad), 5) for a, p in zip(got[n], leaf[n])]
                       for n in names}
    out["grad_norm"] = {n: [float("%.3g" % float(p.grad.norm())) for p in leaf[n]] for n in names}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
