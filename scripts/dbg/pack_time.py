"""Per-part timing of the one-launch weight update (pack_step) on the SL trunk: the whole
launch, its pack_trunk rows alone, its wino_pack rows alone, and the separate kernels (CUDA
events over 200 launches each, with the SGD fold on a scratch flat buffer)."""
import torch

from rocalphago_amd.models.engine import ConvSpec, HipTrunk
from rocalphago_amd.ops import hipops as ops


def main():
    dev = torch.device("cuda")
    specs = [ConvSpec(5, 48, 192, True)] + [ConvSpec(3, 192, 192, True)] * 11 + \
        [ConvSpec(1, 192, 1, False)]
    sizes = [s.cout * s.cin * s.ks * s.ks + s.cout for s in specs]
    n = 1024 + sum(sizes)
    flat = torch.randn(n, device=dev) * 0.01
    grad = torch.randn(n, device=dev) * 1e-6
    ws, bs, p = [], [], 1024
    for s in specs:
        k = s.cout * s.cin * s.ks * s.ks
        ws.append(flat[p:p + k].view(s.cout, s.cin, s.ks, s.ks))
        bs.append(flat[p + k:p + k + s.cout])
        p += k + s.cout
    tr = HipTrunk(specs, 19, dev)
    tr.sync_weights(ws, bs, 1)
    goff = (grad.data_ptr() - flat.data_ptr()) // 4
    sgd = (goff, 1e-9, 0.0)
    nw = sum(tr._wino)
    width = max(8 * tr._wpack_tiles, tr._pack_total)
    L = len(specs)
    cases = {
        "pack_step all": lambda: ops.pack_step(tr._wpack_table, nw, tr._pack_table, L,
                                               tr._pack_nfull, tr._pack_taps, width, sgd=sgd,
                                               flat=flat, rest=[(0, 1024)]),
        "pack_step trunk rows": lambda: ops.pack_step(None, 0, tr._pack_table, L, tr._pack_nfull,
                                                      tr._pack_taps, width, sgd=sgd),
        "pack_step wino rows": lambda: ops.pack_step(tr._wpack_table, nw, None, 0, 0, 1, width,
                                                     sgd=sgd),
        "wino_pack": lambda: ops.wino_pack(tr._wpack_table, nw, tr._wpack_tiles, sgd=sgd),
        "pack_trunk": lambda: ops.pack_trunk(tr._pack_table, L, tr._pack_total, tr._pack_nfull,
                                             sgd=sgd),
        "sgd rest": lambda: ops.sgd_(flat[:1024], grad[:1024], 1e-9),
    }
    for name, fn in cases.items():
        for _ in range(20):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(5):
            a.record()
            for _ in range(200):
                fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1000 / 200)
        print("%-22s %7.1f us per launch (best of 5 x 200)" % (name, min(ts)), flush=True)


if __name__ == "__main__":
    main()
