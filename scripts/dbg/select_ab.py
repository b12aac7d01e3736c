"""A/B of Search.batched_select on the null evaluator: python scripts/dbg/select_ab.py THREADS 0|1"""
import time, sys, numpy as np
from rocalphago_amd._native import engine
from rocalphago_amd.engine.gamestate import GameState
from benchmarks.mcts_null_bench import NullEvaluator
rg = engine()
st = GameState()
th = int(sys.argv[1]); batched = sys.argv[2] == "1"
ev = NullEvaluator(nthreads=th)
for rep in range(3):
    s = rg.Search(st.native, th); s.lmbda = 0.5; s.batched_select = batched
    tsel = tb = 0; t0 = time.perf_counter()
    while s.root_visits < 32768:
        a = time.perf_counter()
        wid, n = s.select(512)
        b = time.perf_counter()
        boards = s.leaf_boards(wid)
        pri, val, sens = ev(boards)
        c = time.perf_counter()
        s.backup_value(wid, pri, val, sens); s.backup_rollout(wid, np.zeros(n, np.float32))
        tb += time.perf_counter() - c; tsel += b - a
    print(batched, th, "select us/sim %.3f backup %.3f  timers %s coll %d nodes %d" % (tsel/s.sims*1e6, tb/s.sims*1e6, s.timers, s.collisions, s.num_nodes))
