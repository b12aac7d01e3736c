"""Diagnostic: GPU ladder planes on the leaf boards of a real search (odd wave sizes, early and
late positions), checked against the native search after every wave."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch

from rocalphago_amd._native import engine
from rocalphago_amd.engine.gamestate import GameState
from rocalphago_amd.ops.features import gpu_ladders

rg = engine()


def main():
    dev = torch.device("cuda")
    rp = rg.RolloutPolicy()
    rs = np.random.RandomState(0)
    work = None
    checked = 0
    for start in (0, 1, 2, 60, 200):
        st = GameState()
        for k in range(start):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            st.do_move(None if mv < 0 else divmod(mv, 19))
        s = rg.Search(st.native, 8)
        s.lmbda = 0.0
        for w in range(12):
            wid, n = s.select(int(rs.choice([1, 7, 255, 256, 131])))
            if n == 0:
                continue
            boards = s.leaf_boards(wid)
            colors, _, meta, _, want = rg.gpu_feature_inputs(boards, True, 8)
            c = torch.from_numpy(colors).to(dev)
            m = torch.from_numpy(meta).to(dev)
            got, work = gpu_ladders(c, m, 19, work=work)
            torch.cuda.synchronize()
            got = got.cpu().numpy()
            assert np.array_equal(got, want), (start, w, n)
            checked += n
            P = 361
            s.backup_value(wid, np.full((n, P), 1.0 / P, np.float32), np.zeros(n, np.float32),
                           None)
        print("start", start, "ok", flush=True)
    print("checked", checked, "leaves")


if __name__ == "__main__":
    main()
