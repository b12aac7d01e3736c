"""Same-box A/B of the one-launch weight update (engine._PackedConvs.ONE_LAUNCH: pack_step
against wino_pack + pack_trunk + sgd_kernel): runs bench.py with ONE_LAUNCH set from the first
argument (1 / 0); the other arguments go to bench.py.

    python scripts/dbg/pack_ab.py 0 --no-mcts --steps 60 --warmup 10
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    from rocalphago_amd.models import engine
    engine._PackedConvs.ONE_LAUNCH = sys.argv[1] != "0"
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
    runpy.run_path(sys.argv[0], run_name="__main__")
