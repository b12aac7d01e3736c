"""Per-step wall time of the first SL training steps (bench.py's model and trainer): how many
steps the step time takes to settle after start-up."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.training.data import TRANSFORM_NAMES, DeviceDataset
    from rocalphago_amd.training.supervised import SupervisedTrainer
    dev = torch.device("cuda")
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=13, device=dev,
                    seed=1234)
    pol.model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.003), metrics=["accuracy"])
    ds = DeviceDataset.synthetic(16384, 48, 19, dev, seed=17)
    tr = SupervisedTrainer(pol.model, ds, 256, TRANSFORM_NAMES, None, seed=5)
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    ts = []
    for k in range(60):
        idx = torch.randint(0, ds.N, (256,), device=dev, generator=gen)
        torch.cuda.synchronize()
        t = time.perf_counter()
        tr.step(idx)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    print("ms per step:", " ".join("%.2f" % x for x in ts))


if __name__ == "__main__":
    main()
