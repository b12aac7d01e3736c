"""GPU fast rollouts (csrc/hip/rollout.hip): thousands of playouts per launch, one wavefront per
game, on side HIP streams so they overlap the policy/value network pass of the same wave.

A playout is ~430 strictly sequential moves, so one launch lasts as long as its slowest game
(milliseconds) however few games it holds. Launches of consecutive search waves therefore go to a
small ring of streams (separate hardware queues) and run concurrently; on one stream they would
serialise and cap the search at one wave of rollouts per playout latency."""
import ctypes

import numpy as np
import torch

from ..ops.hipops import _check, _lib, _ptr


class _Pending(object):
    """One launch's winners, copied to pinned host memory on the rollout's own stream: reading
    them waits for that stream only. (A ``.cpu()`` here ran on the main stream and so waited for
    every network wave queued there, stalling the search pipeline at each rollout backup.)"""

    def __init__(self, event, host_winners, n, R):
        self.event = event
        self.host = host_winners
        self.n = n
        self.R = R

    def done(self):
        return self.event.query()

    def result(self):
        """Mean result per leaf from BLACK's point of view, numpy float32 [n]."""
        self.event.synchronize()
        w = self.host.numpy().reshape(self.n, self.R).astype(np.float32)
        return w[:, 0].copy() if self.R == 1 else w.mean(1, dtype=np.float32)


class _Group(object):
    """Rollouts of several search waves launched together (RolloutBatcher)."""

    def __init__(self):
        self.colors, self.meta = [], []
        self.games = 0
        self.pending = None
        self._res = None

    def result(self):
        if self._res is None:
            self._res = self.pending.result()
        return self._res


class _Slice(object):
    """One wave's share of a group: the _Pending interface (done / result)."""

    def __init__(self, batcher, group, off, n):
        self.batcher, self.group, self.off, self.n = batcher, group, off, n

    def done(self):
        return self.group.pending is not None and self.group.pending.done()

    def result(self):
        if self.group.pending is None:
            self.batcher.flush()
        return self.group.result()[self.off:self.off + self.n]


class RolloutBatcher(object):
    """Launches the rollouts of ``group`` consecutive search waves as one kernel.

    A launch lasts as long as its longest playout (~430 sequential moves) whether it holds 256 or
    1024 games — a 256-leaf wave fills only 64 CUs — and launches of different waves overlap only
    as far as the hardware queues allow. Grouping waves multiplies the rollouts per queue slot;
    a wave's rollouts start at most one wave later, which the asynchronous rollout backup of
    APV-MCTS absorbs."""

    def __init__(self, rollouts, group=2):
        self.gr = rollouts
        self.k = max(1, int(group))
        self.cur = None
        self.args = None

    def add(self, search, wave, R, limit, seed):
        colors, meta = search.rollout_inputs(wave)
        if self.cur is None:
            self.cur = _Group()
            b = search.root_board
            self.args = (b.size, b.komi, R, limit, seed)
        g = self.cur
        sl = _Slice(self, g, g.games, colors.shape[0])
        g.colors.append(colors)
        g.meta.append(meta)
        g.games += colors.shape[0]
        if len(g.colors) >= self.k:
            self.flush()
        return sl

    def flush(self):
        g, self.cur = self.cur, None
        if g is None:
            return
        S, komi, R, limit, seed = self.args
        colors = np.concatenate(g.colors) if len(g.colors) > 1 else g.colors[0]
        meta = np.concatenate(g.meta) if len(g.meta) > 1 else g.meta[0]
        ev, _, _, _, host = self.gr._launch(colors, meta, S, komi, R, limit, seed)
        g.pending = _Pending(ev, host, colors.shape[0], R)


# moves per rollout launch (rag_rollouts' sliced mode: the games are parked in HBM between
# launches, so no launch holds a CU for a whole playout); 0 = one launch per playout. With
# 8-wave rollout groups, 4 / 8 / 16 moves measured 138.6-140.2k / 140.7-141.7k / 139.1-142.6k
# sims/s (three alternating runs each, one box): the same within the spread. The conv launches
# that overlap a rollout slice ran 1.55x / 2.7x / ~4x the median, against 9.6x for one launch per
# playout (profiles/mcts_rollout_interference_r6.txt)
DEFAULT_SLICE = 4
# torch stream priority of the rollout streams (larger = lower; 0 = default)
DEFAULT_PRIORITY = 0


class GpuRollouts(object):
    def __init__(self, policy, device=None, nstreams=6, priority=None, slice_moves=None):
        """nstreams: ring of rollout streams (hardware queues); priority: torch stream priority
        (larger = lower; 0 = default); slice_moves: moves per launch (None: DEFAULT_SLICE, 0:
        one launch per playout)."""
        self.device = torch.device(device or "cuda")
        self.slice = DEFAULT_SLICE if slice_moves is None else int(slice_moves)
        if priority is None:
            priority = DEFAULT_PRIORITY
        self.streams = [torch.cuda.Stream(self.device, priority=priority)
                        for _ in range(max(1, nstreams))]
        self._next = 0
        self.set_policy(policy)

    def set_policy(self, policy):
        self.w = torch.tensor(np.asarray(policy.weights, np.float32), device=self.device)
        self.pattern = torch.tensor(np.asarray(policy.pattern, np.float32), device=self.device)
        # the side streams must see the uploaded weights (later launches do not wait for the
        # main stream)
        for st in self.streams:
            st.wait_stream(torch.cuda.current_stream(self.device))

    def _launch(self, colors, meta, S, komi, R, limit, seed, length=False, dbg=False):
        n = colors.shape[0]
        games = n * R
        # everything the kernel touches is allocated / staged on the side stream itself, so the
        # launch does not wait for the network work queued on the main stream
        stream = self.streams[self._next]
        self._next = (self._next + 1) % len(self.streams)
        with torch.cuda.stream(stream):
            winners = torch.empty(games, dtype=torch.int8, device=self.device)
            lengths = torch.empty(games, dtype=torch.int16, device=self.device) \
                if length else None
            logits = torch.empty(games, S * S, dtype=torch.float32, device=self.device) \
                if dbg else None
            c = torch.from_numpy(np.ascontiguousarray(colors, np.int8)).pin_memory() \
                .to(self.device, non_blocking=True)
            m = torch.from_numpy(np.ascontiguousarray(meta, np.int32)).pin_memory() \
                .to(self.device, non_blocking=True)
            park, sl = None, 0
            if self.slice > 0 and not dbg and limit > self.slice:
                # the parked games (allocated on this stream: reused only after the launches)
                park = torch.empty(games * int(_lib().rag_rollout_park_bytes(S)),
                                   dtype=torch.uint8, device=self.device)
                sl = self.slice
            _check(_lib().rag_rollouts(_ptr(c), _ptr(m), n, R, S, float(komi), int(limit),
                                       _ptr(self.w), _ptr(self.pattern),
                                       ctypes.c_uint(seed & 0xFFFFFFFF), _ptr(winners),
                                       _ptr(lengths), _ptr(logits),
                                       ctypes.c_void_p(stream.cuda_stream), _ptr(park), sl),
                   "rollouts")
            host = torch.empty(games, dtype=torch.int8, pin_memory=True)
            host.copy_(winners, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        return ev, winners, lengths, logits, host

    def launch(self, search, wave, R, limit, seed=1):
        """Start R playouts for every leaf of a native Search wave (non-blocking)."""
        colors, meta = search.rollout_inputs(wave)
        b = search.root_board
        ev, _, _, _, host = self._launch(colors, meta, b.size, b.komi, R, limit, seed)
        return _Pending(ev, host, colors.shape[0], R)

    # ---------------------------------------------------------------- direct use / tests
    @staticmethod
    def encode(states):
        """GameStates -> (colors [n, S*S] int8, meta [n, 8] int32)."""
        S = states[0].size
        colors = np.zeros((len(states), S * S), np.int8)
        meta = np.zeros((len(states), 8), np.int32)
        for i, st in enumerate(states):
            b = st.native
            colors[i] = np.asarray(b.board(), np.int8).reshape(-1)
            l1, l2 = b.last_moves
            meta[i] = [b.current_player, b.ko, l1, l2, b.passes_black, b.passes_white,
                       b.move_count, int(b.end_of_game)]
        return colors, meta

    def run(self, states, R=1, limit=500, seed=1):
        """(winners [n, R] int8, lengths [n, R] int16) as numpy."""
        colors, meta = self.encode(states)
        ev, _, ln, _, host = self._launch(colors, meta, states[0].size, states[0].komi, R, limit,
                                          seed, length=True)
        ev.synchronize()
        n = len(states)
        with torch.cuda.stream(self.streams[0]):  # lengths: read after the launch's own event
            torch.cuda.current_stream().wait_event(ev)
            lens = ln.view(n, R).cpu().numpy()
        return host.numpy().reshape(n, R).copy(), lens

    def initial_logits(self, states):
        """Debug: candidate logits at each state's position ([n, S*S], -inf = not a legal
        candidate), for parity with RolloutPolicy.candidates."""
        colors, meta = self.encode(states)
        ev, _, _, lg, _ = self._launch(colors, meta, states[0].size, states[0].komi, 1, 0, 1,
                                       dbg=True)
        ev.synchronize()
        return lg.cpu().numpy()
