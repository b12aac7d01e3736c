"""Per-step time of every training step in a rocprofv3 kernel trace (steps delimited by the
input-packing kernel), with the summed time of the 3x3 Winograd forward launches of each step:
shows whether early steps are slower and whether every kernel slows alike (clock ramp) or only
some (a software warm-up).

    python scripts/dbg/step_ramp_trace.py gpurun_out/<job>/trace/sl_results.db
"""
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from step_kernels import load  # noqa: E402


def main(path, marker="pack_input"):
    ks = load(path)
    starts = [s for s, e, n in ks if marker in n]
    for i, (a, b) in enumerate(zip(starts, starts[1:])):
        wino = sum(e - s for s, e, n in ks if a <= s < b and "conv_wino" in n)
        nw = sum(1 for s, e, n in ks if a <= s < b and "conv_wino" in n)
        wg = sum(e - s for s, e, n in ks if a <= s < b and "wgrad_slab_kernel" in n)
        print("step %3d  %8.1f us   wino %7.1f us (%d)   wgrad %7.1f us" % (
            i, (b - a) / 1e3, wino / 1e3, nw, wg / 1e3))


if __name__ == "__main__":
    main(*sys.argv[1:])
