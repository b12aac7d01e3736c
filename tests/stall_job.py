"""A minimal data-parallel loop with the same failure detection as bench.py (gloo, CPU): every
rank heart-beats per step into the rank watchdog and all-reduces a gradient-sized buffer;
RAG_STALL=rank:step makes one rank hang before its all-reduce. Launched by
tests/test_watchdog.py under torch.distributed.run."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.parallel.watchdog import RankWatchdog, inject_stall
    limit = float(os.environ.get("RAG_TEST_STALL_LIMIT", "6"))
    dp = DPContext(device="cpu", timeout_s=int(limit) + 60)
    wd = RankWatchdog(dp.rank, dp.world, limit, phase="sl-timed", publish_s=0.2)
    g = torch.ones(1 << 16)
    for k in range(40):
        inject_stall(dp.rank, k)
        wd.beat(2 * k)
        dp.allreduce_sum_(g)
        wd.beat(2 * k + 1)
        time.sleep(0.02)
    wd.stop()
    print("rank %d done" % dp.rank, flush=True)
    dp.shutdown()


if __name__ == "__main__":
    main()
