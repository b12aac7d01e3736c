import numpy as np, torch, sys
sys.path.insert(0, ".")
from tests.test_gpu_sampling import _positions
from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
from rocalphago_amd.models.policy import CNNPolicy
from rocalphago_amd.ops.features import GpuFeatures
from rocalphago_amd.ops import hipops as ops
gpu = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=64, layers=4, device="cuda", seed=4)
gpu.model.set_weights([w * 8 for w in gpu.model.get_weights()])
states = _positions(8, seed=1)
gf = GpuFeatures(DEFAULT_FEATURES, "cuda")
sens = torch.empty((8, 361), dtype=torch.uint8, device="cuda")
xg = gf([s.native for s in states], sens_out=sens)
xc = gpu.preprocessor.states_to_tensor_u8(states)
print("feat diff", (xg.cpu().numpy() != xc).sum(), "per plane", (xg.cpu().numpy() != xc).sum(axis=(0,2,3)))
pg = gpu.forward_device(xg).cpu().numpy()
pc = gpu.forward(xc)
print("prob diff", np.abs(pg - pc).max())
mv = ops.sample_moves(torch.from_numpy(pg).cuda(), sens, 1.0, torch.ones(8, dtype=torch.uint8, device="cuda"), 1).cpu().numpy()
for i, st in enumerate(states):
    legal = st.get_legal_moves(include_eyes=False)
    idx = [x * 19 + y for x, y in legal]
    best = idx[int(np.argmax(pc[i][idx]))]
    print(i, mv[i], best, pg[i][mv[i]] if mv[i] >= 0 else None, pc[i][best], sens[i].sum().item(), len(idx))
