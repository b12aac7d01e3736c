"""Per-rank stall watchdog for multi-process GPU jobs (SURVEY §5.3 failure detection, §5.8).

A rank that stops making progress (a hung collective, a wedged kernel, a peer that died) must
not turn a multi-GPU run into a silent hang: every rank runs a ``RankWatchdog`` thread, the hot
loop calls ``beat(step)`` and the watchdog, when no beat arrives for ``limit_s`` seconds, prints
one diagnostic line per rank to stderr and ends the process with a non-zero status
(``os._exit(STALL_EXIT)``, so a thread stuck inside a collective cannot block the exit).

The diagnostic names the *stalled* rank(s), not just "timeout": each rank publishes its
heartbeat (phase, step, wall time) into the job's c10d key-value store (the TCPStore that
torchrun's rendezvous already runs on MASTER_ADDR), throttled to one store write per
``publish_s``; a timed-out rank reads every rank's last heartbeat and reports the ranks whose
step is behind (or that never published), e.g.

  [watchdog] rank 0: no progress for 12.0s in 'sl-dp' (last step 3); stalled rank(s): [1]
             heartbeats: r0=sl-dp:4@11.9s r1=sl-dp:2@12.0s

The store read has its own short timeout, so a dead store never delays the exit.
"""
import os
import sys
import threading
import time

STALL_EXIT = 3


def _default_store():
    try:
        import torch.distributed as dist
        if not dist.is_initialized():
            return None
        from torch.distributed import distributed_c10d as c10d
        return c10d._get_default_store()
    except Exception:  # noqa: BLE001 - no store: local diagnostics only
        return None


class RankWatchdog(object):
    def __init__(self, rank, world, limit_s, phase="init", publish_s=1.0, store=None,
                 stream=None, on_stall=None):
        self.rank, self.world = int(rank), int(world)
        self.limit_s = float(limit_s)
        self.publish_s = float(publish_s)
        self.phase = phase
        self.step = -1
        self.store = store if store is not None else _default_store()
        self.stream = stream or sys.stderr
        self.on_stall = on_stall  # tests: called with the message instead of exiting
        self.t0 = time.time()
        self.last = time.time()
        self._published = 0.0
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, name="rank-watchdog", daemon=True)
        self._th.start()
        self._publish(force=True)

    # ---------------------------------------------------------------- hot loop side
    def beat(self, step=None, phase=None):
        if phase is not None:
            self.phase = phase
        if step is not None:
            self.step = int(step)
        self.last = time.time()
        self._publish()

    def set_phase(self, phase, limit_s=None):
        if limit_s is not None:
            self.limit_s = float(limit_s)
        self.beat(-1, phase)
        self._publish(force=True)

    def stop(self):
        self._stop.set()

    # ---------------------------------------------------------------- internals
    def _publish(self, force=False):
        if self.store is None:
            return
        now = time.time()
        if not force and now - self._published < self.publish_s:
            return
        self._published = now
        try:
            self.store.set("rag/hb/%d" % self.rank,
                           "%s:%d:%.3f" % (self.phase, self.step, now - self.t0))
        except Exception:  # noqa: BLE001 - heartbeats are best effort
            pass

    def heartbeats(self):
        """{rank: (phase, step, seconds since that rank's start) or None} from the store."""
        out = {}
        if self.store is None:
            return out
        try:
            self.store.set_timeout(__import__("datetime").timedelta(seconds=2))
        except Exception:  # noqa: BLE001
            pass
        for r in range(self.world):
            try:
                if not self.store.check(["rag/hb/%d" % r]):
                    out[r] = None
                    continue
                v = self.store.get("rag/hb/%d" % r).decode()
                ph, st, t = v.rsplit(":", 2)
                out[r] = (ph, int(st), float(t))
            except Exception:  # noqa: BLE001
                out[r] = None
        return out

    def stalled_ranks(self, hb):
        """Ranks behind the furthest one: no heartbeat, an earlier phase-local step, or (same
        step) the oldest heartbeat."""
        known = {r: v for r, v in hb.items() if v is not None}
        missing = sorted(r for r, v in hb.items() if v is None)
        if not known:
            return missing
        top = max(v[1] for v in known.values())
        behind = sorted(r for r, v in known.items() if v[1] < top)
        if not behind and not missing and len(known) > 1:
            # everyone at the same step: the rank whose last beat is oldest stopped first
            oldest = min(known.items(), key=lambda kv: kv[1][2])[0]
            behind = [oldest]
        return sorted(set(behind) | set(missing))

    def _run(self):
        while not self._stop.wait(0.25):
            idle = time.time() - self.last
            if idle < self.limit_s:
                continue
            # this rank's exact state, then a moment for the other ranks' watchdogs (they stall
            # together) to publish theirs: the throttled heartbeats may be up to publish_s old
            self._publish(force=True)
            time.sleep(min(2.0, 2 * self.publish_s))
            hb = self.heartbeats()
            stalled = self.stalled_ranks(hb) if hb else [self.rank]
            beats = " ".join("r%d=%s" % (r, "none" if v is None else "%s:%d@%.1fs" % v)
                             for r, v in sorted(hb.items()))
            msg = ("[watchdog] rank %d: no progress for %.1fs in '%s' (last step %d); "
                   "stalled rank(s): %s%s" % (self.rank, idle, self.phase, self.step, stalled,
                                              ("\n[watchdog]   heartbeats: " + beats)
                                              if beats else ""))
            if self.on_stall is not None:
                self.on_stall(msg)
                return
            try:
                self.stream.write(msg + "\n")
                self.stream.flush()
            finally:
                os._exit(STALL_EXIT)


def inject_stall(rank, step):
    """Fault injection for the failure-detection tests and rehearsals: when the environment
    names this rank and step (RAG_STALL="rank:step[:seconds]"), stop here (sleep, default an
    hour) as a rank whose peer collective never arrives would."""
    spec = os.environ.get("RAG_STALL")
    if not spec:
        return
    parts = spec.split(":")
    if int(parts[0]) != int(rank) or int(parts[1] if len(parts) > 1 else 0) != int(step):
        return
    time.sleep(float(parts[2]) if len(parts) > 2 else 3600.0)
