"""Per-rank training observability: a JSONL stream of step time, exposed
all-reduce time and HBM use, written by every rank to ``<out>/metrics.rank<r>.jsonl``.

The reference only writes per-epoch loss/accuracy into metadata.json
(/root/reference/AlphaGo/training/supervised_policy_trainer.py:48-73). Here each rank also
reports, per logging interval:

* ``step_ms``        mean wall time per optimizer step (host clock, synchronised at the interval
                     boundary only — no per-step host syncs on the hot path);
* ``allreduce_wait_ms`` mean time the compute stream stalled waiting for the gradient all-reduce
                     (HIP events around ``BucketedAllReduce.finish``: the part of the collective
                     not hidden behind backward);
* ``hbm_max_gb``     ``torch.cuda.max_memory_allocated`` of the rank's device.

Nothing here issues a collective, so ranks may log at different moments.
"""
import json
import os
import time

import torch


class CommTimer(object):
    """Records (start, end) event pairs on the current stream around the exposed part of each
    step's gradient all-reduce. Pairs are resolved as they complete (a bounded ring: once more
    than ``ring`` pairs are outstanding the oldest is waited for), so a long epoch keeps O(ring)
    events alive instead of two per step until ``pop``."""

    def __init__(self, device, ring=64):
        self.cuda = torch.device(device).type == "cuda"
        self.pairs = []
        self.ring = int(ring)
        self.done_ms = 0.0
        self.done_n = 0
        self.host_ms = 0.0
        self.host_n = 0
        self._t = None

    def start(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.pairs.append([e, None])
        else:
            self._t = time.perf_counter()

    def stop(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.pairs[-1][1] = e
            self._resolve(block=len(self.pairs) > self.ring)
        elif self._t is not None:
            self.host_ms += (time.perf_counter() - self._t) * 1e3
            self.host_n += 1
            self._t = None

    def _resolve(self, block=False):
        """Fold completed pairs (oldest first) into the running total; with ``block`` wait for
        the oldest pair so the ring stays bounded."""
        while self.pairs and self.pairs[0][1] is not None:
            a, b = self.pairs[0]
            if not b.query():
                if not block:
                    return
                b.synchronize()
            block = False
            self.done_ms += a.elapsed_time(b)
            self.done_n += 1
            self.pairs.pop(0)

    def pending(self):
        return len(self.pairs)

    def pop(self):
        """(total exposed all-reduce ms, number of steps) since the last pop (synchronises on the
        last event)."""
        if self.pairs and self.pairs[-1][1] is not None:
            self.pairs[-1][1].synchronize()
        self._resolve()
        ms, n = self.done_ms + self.host_ms, self.done_n + self.host_n
        self.done_ms = self.host_ms = 0.0
        self.done_n = self.host_n = 0
        return ms, n


class RankMetrics(object):
    """Appends one JSON line per ``log`` call to ``<out_dir>/metrics.rank<rank>.jsonl``."""

    def __init__(self, out_dir, rank, world, device):
        self.path = os.path.join(out_dir, "metrics.rank%d.jsonl" % rank) if out_dir else None
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        self.comm = CommTimer(self.device)
        self._t0 = time.perf_counter()
        self._steps = 0

    def step_done(self, n=1):
        self._steps += n

    def log(self, **extra):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        dt = now - self._t0
        comm_ms, ncomm = self.comm.pop()
        rec = {"rank": self.rank, "world": self.world, "steps": self._steps,
               "step_ms": round(dt * 1e3 / max(self._steps, 1), 4),
               "allreduce_wait_ms": round(comm_ms / max(ncomm, 1), 4) if ncomm or comm_ms else 0.0,
               "time": round(time.time(), 3)}
        if self.device.type == "cuda":
            rec["hbm_max_gb"] = round(torch.cuda.max_memory_allocated(self.device) / 2 ** 30, 4)
        rec.update(extra)
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(rec) + "\n")
        self._t0, self._steps = now, 0
        return rec
