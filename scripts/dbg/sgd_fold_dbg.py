"""Which parameters differ between the folded SGD step and sgd_kernel + repack (ResNet)."""
import numpy as np
import torch

from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
from rocalphago_amd.models import kerasish as KZ
from rocalphago_amd.models.policy import ResnetPolicy

rs = np.random.RandomState(4)
B = 256
X = (rs.rand(B, 48, 19, 19) > 0.6).astype(np.uint8)
Y = np.zeros((B, 361), np.float32)
Y[np.arange(B), rs.randint(0, 361, B)] = 1
out = []
for fold in (True, False, False):
    pol = ResnetPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=128, layers=5,
                       device=torch.device("cuda"), seed=9)
    m = pol.model
    m.compile(loss="categorical_crossentropy", optimizer=KZ.SGD(lr=0.05))
    plan = m._plan_for()
    if not fold:
        m.net._sgd_fold = None
    init = m.net.flat.clone()
    for _ in range(int(__import__("sys").argv[1]) if len(__import__("sys").argv) > 1 else 1):
        m.train_on_batch(X, Y)
    torch.cuda.synchronize()
    out.append((m.net.flat.clone(), init, [v.clone() for v in m.net._views], getattr(plan, "folded_steps", 0)))
names = m.net.weight_names
print("init equal", torch.equal(out[0][1], out[1][1]), "folded", out[0][3], out[1][3])
for k, (nm, a, b, c) in enumerate(zip(names, out[0][2], out[1][2], out[2][2])):
    d = (a - b).abs().max().item()
    d2 = (b - c).abs().max().item()
    print(nm, tuple(a.shape), "fold-vs-plain %.3g" % d, "plain-vs-plain %.3g" % d2, "scale %.3g" % b.abs().max().item())
