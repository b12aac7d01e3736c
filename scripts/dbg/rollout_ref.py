"""Bit-exactness guard for rollout kernel rewrites: fixed positions + seed -> winners/lengths.

  python scripts/dbg/rollout_ref.py save  OUT.npz   # record with the current kernel
  python scripts/dbg/rollout_ref.py check REF.npz   # compare the current kernel to a record
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch

from rocalphago_amd._native import engine
from rocalphago_amd.engine.gamestate import GameState
from rocalphago_amd.search.gpu_rollout import GpuRollouts


def states(n=384, seed=5):
    rg = engine()
    rp = rg.RolloutPolicy()
    rs = np.random.RandomState(seed)
    out = []
    for i in range(n):
        st = GameState()
        for _ in range(int(rs.randint(0, 200))):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            st.do_move(None if mv < 0 else divmod(mv, 19))
            if st.is_end_of_game:
                break
        out.append(st)
    return out, rp


def main():
    mode, path = sys.argv[1], sys.argv[2]
    sts, rp = states()
    gr = GpuRollouts(rp, torch.device("cuda"))
    w, ln = gr.run(sts, R=4, limit=500, seed=123)
    lg = gr.initial_logits(sts[:64])
    if mode == "save":
        np.savez(path, w=w, ln=ln, lg=lg)
        print("saved", w.shape, float(ln.mean()))
    else:
        ref = np.load(path)
        same_w = np.array_equal(ref["w"], w)
        same_l = np.array_equal(ref["ln"], ln)
        same_g = np.array_equal(ref["lg"], lg)
        print("winners equal", same_w, "lengths equal", same_l, "logits equal", same_g,
              "mean length", float(ln.mean()), "ref", float(ref["ln"].mean()))
        if not (same_w and same_l and same_g):
            sys.exit(1)


if __name__ == "__main__":
    main()
