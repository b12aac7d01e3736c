"""SGF -> HDF5 conversion throughput (games/s and positions/s): the bulk native converter at
1..N threads against the python replay, on copies of the reference fixture games (48 planes,
19x19; the reference itself converts one game at a time in python, game_converter.py:102-140)."""
import argparse
import glob
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rocalphago_amd.features.converter import GameConverter  # noqa: E402
from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES  # noqa: E402

REF = "/root/reference/tests/test_data/sgf"


def _synthetic_games(d, n):
    import numpy as np
    from rocalphago_amd._native import engine
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.utils.go_util import save_gamestate_to_sgf
    rp = engine().RolloutPolicy()
    rs = np.random.RandomState(0)
    out = []
    for g in range(n):
        st = GameState()
        for _ in range(int(rs.randint(150, 300))):
            mv = rp.sample(st.native, int(rs.randint(1 << 30)))
            st.do_move(None if mv < 0 else divmod(mv, 19))
            if st.is_end_of_game:
                break
        name = "synthetic%d.sgf" % g
        save_gamestate_to_sgf(st, d, name)
        out.append(os.path.join(d, name))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=40)
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--sgf-dir", default=REF)
    args = ap.parse_args()
    d = tempfile.mkdtemp()
    src = sorted(glob.glob(os.path.join(args.sgf_dir, "*.sgf")))
    if not src:  # no fixture games here: rollout-policy self-play games of 150-300 moves
        src = _synthetic_games(d, 5)
    try:
        files = []
        for k in range(args.copies):
            for f in src:
                dst = os.path.join(d, "%03d_%s" % (k, os.path.basename(f)))
                shutil.copy(f, dst)
                files.append(dst)
        conv = GameConverter(list(DEFAULT_FEATURES))
        out = {"games": len(files), "features": 48}
        npos = sum(len(conv._python_game(f, 19)[1]) for f in files[:len(src)])
        # end to end (parse, replay, features, LZF, HDF5) for every path; threads 0 = the
        # per-game Python replay on the first copy of the games
        t = time.perf_counter()
        conv.sgfs_to_hdf5(files[:len(src)], os.path.join(d, "py.h5"), nthreads=0, batch=64)
        dt = time.perf_counter() - t
        out["python_games_per_s"] = round(len(src) / dt, 2)
        out["python_positions_per_s"] = round(npos / dt, 1)
        for nt in [int(x) for x in args.threads.split(",")]:
            t = time.perf_counter()
            conv.sgfs_to_hdf5(files, os.path.join(d, "o%d.h5" % nt), nthreads=nt, batch=64)
            dt = time.perf_counter() - t
            out["native_games_per_s_t%d" % nt] = round(len(files) / dt, 2)
            size = os.path.getsize(os.path.join(d, "o%d.h5" % nt))
            out["native_positions_per_s_t%d" % nt] = round(npos * args.copies / dt, 1)
            out["hdf5_bytes"] = size
        print(json.dumps(out))
    finally:
        shutil.rmtree(d)


if __name__ == "__main__":
    main()
