"""Same-box A/B of the SGD step folded into the trunk's weight repack: runs bench.py with
kerasish.SGD.FOLD set from the first argument (1 / 0); the other arguments go to bench.py.

    python scripts/dbg/fold_ab.py 0 --no-mcts --steps 60 --warmup 10
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    from rocalphago_amd.models import kerasish
    kerasish.SGD.FOLD = sys.argv[1] != "0"
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
    runpy.run_path(sys.argv[0], run_name="__main__")
