"""DP replica check on the real HIP training path, run by tests/test_gpu_bench_path.py under
torch.distributed.run (on one GPU with RAG_DIST_BACKEND=gloo):

  * every rank trains the 192-filter SL policy (conv_tap / wgrad_slab kernels, the wgrad
    reductions deferred into the dgrad launches, layer-bucketed gradient all-reduce) on its own
    slice of each global batch;
  * rank 0 checks that all replicas hold bit-identical weights afterwards, and compares the
    weight update with a single-process run on the concatenated global batch (same kernels,
    batch 2x: bf16 summation order differs, so a relative tolerance).

Prints one JSON line on rank 0 and exits non-zero on a mismatch.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES  # noqa: E402
from rocalphago_amd.models import kerasish as K  # noqa: E402
from rocalphago_amd.models.policy import CNNPolicy  # noqa: E402
from rocalphago_amd.parallel.dp import DPContext  # noqa: E402
from rocalphago_amd.training.data import DeviceDataset  # noqa: E402
from rocalphago_amd.training.supervised import SupervisedTrainer  # noqa: E402

STEPS, LOCAL_B = int(os.environ.get("DP_CHECK_STEPS", "1")), 32


def make(dev):
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=4, device=dev,
                    seed=21)
    pol.model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.05),
                      metrics=["accuracy"])
    return pol.model


def main():
    dp = DPContext()
    dev = dp.device
    ds = DeviceDataset.synthetic(STEPS * LOCAL_B * dp.world, 48, 19, dev, seed=5)
    model = make(dev)
    dp.broadcast_model(model)
    start = model.net.flat.detach().clone()
    tr = SupervisedTrainer(model, ds, LOCAL_B, ["noop"], dp, seed=0)
    assert tr.plan is not None, "HIP plan not active"
    gb = LOCAL_B * dp.world
    for s in range(STEPS):
        tr.step(torch.arange(s * gb + dp.rank * LOCAL_B, s * gb + (dp.rank + 1) * LOCAL_B,
                             device=dev))
    torch.cuda.synchronize()
    flat = model.net.flat.detach().clone()
    allw = [torch.empty_like(flat) for _ in range(dp.world)]
    dist.all_gather(allw, flat)
    ok = True
    out = {"world": dp.world, "backend": dist.get_backend()}
    if dp.is_root:
        out["replicas_identical"] = all(torch.equal(allw[0], w) for w in allw[1:])
        ok &= out["replicas_identical"]
    dp.shutdown()
    if dp.is_root:
        ref = make(dev)
        ref.net.flat.data.copy_(start)
        ref.net.bump()
        rt = SupervisedTrainer(ref, ds, gb, ["noop"], None, seed=0)
        for s in range(STEPS):
            rt.step(torch.arange(s * gb, (s + 1) * gb, device=dev))
        torch.cuda.synchronize()
        d_dp = (allw[0] - start).double()
        d_ref = (ref.net.flat.detach() - start).double()
        rel = float((d_dp - d_ref).norm() / d_ref.norm())
        out["update_rel_diff_vs_single_process"] = rel
        out["update_norm"] = float(d_ref.norm())
        ok &= rel < float(os.environ.get("DP_CHECK_TOL", "1e-3")) and float(d_ref.norm()) > 0
        out["ok"] = bool(ok)
        print(json.dumps(out), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
