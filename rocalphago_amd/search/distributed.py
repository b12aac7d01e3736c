"""APV-MCTS on several GPUs of one node (the reference's ParallelMCTS is
an empty stub, /root/reference/AlphaGo/mcts.py:219-220, and its search one sequential tree,
/root/reference/AlphaGo/mcts.py:191-206). One process per GPU.

DistributedMCTS (``bench.py --gpus N``, ``benchmarks/mcts_bench.py --distributed``) is ONE search:

  * rank 0 owns the only tree (the native ``_rocgo.Search``) and runs the master loop natively
    (csrc/mcts/master.hpp ``run_master``, GIL released): for every GPU with room it selects a
    wave of leaves (parallel descents with virtual loss, no leaf boards built), writes each leaf
    as its move path from the root into that GPU's slot of a shared-memory channel, and backs up
    whatever values / rollout results came back — straight from the shared slots;
  * every rank (rank 0 too, on a second thread, for its ``master_share`` of the leaves) serves
    its slots (``serve``): it replays the paths on its own copy of the root board
    (``Search.load_paths``: the boards the tree would have built, superko history included),
    runs the HIP feature kernel and both networks on its GPU (the single-GPU search's packed-wave
    path), starts the wave's fast rollouts on its rollout streams, and writes priors, values and
    sensible masks, later the rollout results, back into the slot;
  * ranks never exchange anything but these slots: no collective per wave or round, no device
    staging of host data, no Python on rank 0's round loop. The root position reaches the other
    ranks as its game record in the channel header.

Throughput vs. search quality: every GPU keeps ``depth`` waves waiting for values and up to
``nslots`` waves holding virtual loss until their rollouts return, so N GPUs keep N times the
leaves of one GPU in flight — a wider search for the same budget. search/efficiency.py measures
what that costs (budget efficiency against one tree with the same total budget) and
``benchmarks/search_efficiency.py --effective`` picks the per-GPU wave / depth with the best
effective rate (simulations/s x efficiency); profiles/search_efficiency_r6.json.

The channel is POSIX shared memory, so all ranks must share one host (the bench's 8-GPU node);
the tree, like the reference's, is host-resident, and leaves travel host-to-host.

SharedRootMCTS (``mode="shared"``) — every rank runs the full single-GPU pipelined search on the
same position and the ranks all-reduce the statistics their trees added at the root's children
after every wave. Measured: the N trees expand the same nodes (duplication N with a
deterministic evaluator), so the job searches like ONE rank (efficiency 1/N) and its N-fold
simulations/s over-credit the search; the bench reports its live duplication. Kept for
comparison.
"""
import collections
import math
import os
import socket
import threading
import time
import uuid

import numpy as np
import torch
import torch.distributed as dist

from .._native import engine as _engine
from ..engine import gamestate as go
from ..engine.gamestate import PASS_MOVE
from .apv import ParallelMCTS, _Slots

_rg = _engine()


def open_channel(dp, nslots, cap, S, PW, stride):
    """The search's shared-memory channel: created by rank 0, attached by the others (one object
    broadcast for its name). Collective over ``dp`` (None / disabled: one process)."""
    world = dp.world if dp is not None and dp.enabled else 1
    rank = dp.rank if dp is not None and dp.enabled else 0
    if world > 1:
        hosts = [None] * world
        dist.all_gather_object(hosts, socket.gethostname())
        if len(set(hosts)) > 1:
            raise RuntimeError("DistributedMCTS: the ranks span hosts %s; its leaf channel is "
                               "shared memory (one node)" % sorted(set(hosts)))
    ch = None
    name = None
    if rank == 0:
        tag = "rag_mcts_%d_%s" % (os.getpid(), uuid.uuid4().hex[:12])
        try:
            name = "/" + tag
            ch = _rg.SearchChannel(name, True, world, nslots, cap, S * S, PW, stride)
        except RuntimeError:
            # /dev/shm too small (containers often give it 64 MB): a mapped file instead
            import tempfile
            name = os.path.join(tempfile.gettempdir(), tag)
            ch = _rg.SearchChannel(name, True, world, nslots, cap, S * S, PW, stride)
    if world > 1:
        obj = [name]
        dist.broadcast_object_list(obj, 0)
        if rank != 0:
            ch = _rg.SearchChannel(obj[0], False)
        dp.barrier()
    ch.unlink()  # every rank mapped it: the name goes, the memory stays while mapped
    return ch


class _ZNow(object):
    """Rollout results that are ready at once (null rollouts)."""

    def __init__(self, n):
        self.z = np.zeros(n, np.float32)

    def done(self):
        return True

    def result(self):
        return self.z


class _ZCpu(object):
    """Native CPU rollouts of a worker wave (Search.start_rollouts), BLACK's view on result()."""

    def __init__(self, ws, wid):
        self.ws, self.wid = ws, wid

    def done(self):
        return True

    def result(self):
        return self.ws.rollout_black_z(self.wid)


def _done(handle):
    """Has a value handle's device work finished (CPU handles: always)?"""
    slot = getattr(handle, "slot", None)
    ev = slot.event if slot is not None else getattr(handle, "event", None)
    return True if ev is None else ev.query()


class DistributedMCTS(ParallelMCTS):
    """One search tree on rank 0, leaf evaluation on every rank of ``dp`` (module doc).

    Call ``get_move(state)`` on EVERY rank (all return the same move; only rank 0's ``state`` is
    read, the others may pass None) and ``update_with_move(move)`` on every rank after playing
    it; ``stop()`` on rank 0 releases the other ranks (their get_move / serve returns None).

    depth: waves per GPU waiting for their values; rollout_slots: further waves per GPU that
    hold virtual loss until their rollouts return (default: one GPU rollout group); batch: leaves
    per wave and GPU; master_share: rank 0's wave relative to the others' (its host also runs the
    tree); rollout_delay: CPU rollouts are returned only this many waves later (the search
    efficiency study's stand-in for the GPU's rollout latency)."""

    # moves per GPU rollout launch on a serving GPU: its rollout groups are small (6 waves of
    # 128-256 leaves), and 4- or 16-move slices cost it 8-15 % of its serving rate against 64
    # (wave 128: 74.3-74.6k / 69.6-74.1k / 80.9-82.7k sims/s, profiles/mcts_wave_rates_r6.json);
    # the single-GPU search's 8-wave groups of 512 take gpu_rollout.DEFAULT_SLICE (4)
    ROLLOUT_SLICE = 64

    def __init__(self, policy=None, value=None, rollout=None, dp=None, depth=2,
                 rollout_slots=None, master_share=1.0, rollout_delay=0, max_path=127,
                 board=None, stall_s=120.0, force_master=False, worker_threads=None, **kw):
        kw.setdefault("pipeline", 3)
        # GPU rollout launches of 6 waves per serving GPU: the geometry its serving rates and the
        # effective-throughput table were measured at (profiles/mcts_wave_rates_r6.json); the
        # single-GPU search launches 8 (ParallelMCTS)
        kw.setdefault("rollout_group", 6)
        super(DistributedMCTS, self).__init__(policy, value, rollout, dp=None, **kw)
        self.ddp = dp
        # host threads of this rank's leaf builder (path replay, input packing, ladder reads);
        # ``nthreads`` sizes rank 0's tree pool
        self.worker_threads = int(worker_threads or self.nthreads)
        self.world = dp.world if dp is not None and dp.enabled else 1
        self.rank = dp.rank if dp is not None and dp.enabled else 0
        self.force_master = bool(force_master)
        self.depth = max(1, int(depth))
        net = policy if policy is not None else value
        if board is None:
            board = net.model.input_shape[-1] if hasattr(net, "model") else 19
        self.S = int(board)
        gpu_dev = None
        inner = getattr(getattr(net, "model", None), "net", None)
        if inner is not None and inner.device.type == "cuda":
            gpu_dev = inner.device
        self.gpu = gpu_dev
        if rollout_slots is None:
            rollout_slots = (self.rollout_group if gpu_dev is not None else 0) + int(rollout_delay)
        self.rollout_slots = int(rollout_slots) if self.lmbda > 0 else 0
        self.rollout_delay = int(rollout_delay)
        self.nslots = self.depth + self.rollout_slots + 1
        from ..models.policy import has_pass_logit
        P = self.S * self.S
        self.PW = P + (1 if has_pass_logit(policy) else 0)
        self.master_share = float(master_share)
        b = int(self.batch)
        self.batches = [max(0, int(round(b * self.master_share)))] + [b] * (self.world - 1) \
            if self.world > 1 else [b]
        self.stall_s = float(stall_s)
        self.worker_rollouts = "gpu" if gpu_dev is not None else "native"
        # search/efficiency.py: answer a wave only once `depth` waves (values) / rollout_delay
        # further waves (rollouts) were received, or after idle_us without a request — the
        # GPU pipeline's leaves in flight, deterministically, with instant CPU evaluations
        self.emulate_latency = False
        self.idle_us = 20
        # no request for this long: launch a partial GPU rollout group (the search is ending)
        self.flush_s = 0.002
        self.chan = None
        if self.world > 1 or self.force_master:
            self.chan = open_channel(dp, self.nslots, max(self.batches), self.S, self.PW,
                                     int(max_path) + 1)
            self._wk = 0
            self._wseq = [0] * self.nslots
            self._wcmd = self.chan.cmd()[0]
        self._views = None
        self._ws = None
        self._wslots = None
        self._batcher = None
        self._err = None
        self.rank_leaves = 0
        self.leaves_per_rank = np.zeros(self.world, np.int64)
        self.master_stats = {}

    # ------------------------------------------------------------------ rank 0: the search
    def get_move(self, state):
        if self.chan is None:
            return super(DistributedMCTS, self).get_move(state)  # one GPU: the local pipeline
        if self.rank != 0:
            return self.serve()
        s = self.search(state)
        a = s.best_move()
        self.chan.post_cmd(_rg.CHAN_CMD_MOVE, int(a))
        self._join_local()
        return PASS_MOVE if a < 0 else divmod(int(a), state.size)

    def search(self, state, n_playout=None):
        """Rank 0: grow the tree by ``n_playout`` simulations through the channel (the master
        loop is native; rank 0's own share is served by a second thread meanwhile)."""
        if self.chan is None:
            return super(DistributedMCTS, self).search(state, n_playout)
        s = self._sync_root(state)
        if state.size != self.S:
            raise ValueError("DistributedMCTS was built for %dx%d boards" % (self.S, self.S))
        self._write_root(state, s)
        self._local_state = state
        self._local = None
        if self.batches[0] > 0:
            self._local = threading.Thread(target=self._serve_local, name="rag-serve-0",
                                           daemon=True)
            self._local.start()
        try:
            st = _rg.run_master(s, self.chan, list(self.batches), self.depth, self.nslots,
                                int(n_playout or self.n_playout), self.seed, self.stall_s)
        except BaseException as e:
            self.chan.abort("rank 0 master: %s" % str(e)[:100])
            self._join_local()
            if self._err is not None:
                raise self._err
            raise
        self.leaves_per_rank += np.asarray(st["leaves"], np.int64)
        self.stats["waves"] += int(st["waves"])
        self.stats["sims"] += int(st["sims"])
        for k in ("t_select", "t_ship", "t_value", "t_rollout", "t_idle", "wall"):
            self._acc(k, float(st[k]))
        self.master_stats = st
        return s

    def _serve_local(self):
        try:
            self.serve(0)
        except BaseException as e:  # the master loop aborts on the channel flag
            self._err = e
            self.chan.abort("rank 0 serving thread: %s" % str(e)[:100])

    def _join_local(self):
        if getattr(self, "_local", None) is not None:
            self._local.join()
            self._local = None

    def _write_root(self, state, s):
        """The root's game record into the channel header (read by ranks that rebuild it)."""
        meta = self.chan.view(0, 0, "root_meta")
        mv = self.chan.view(0, 0, "root_moves")
        size = state.size
        flat = [-1 if m is PASS_MOVE else m[0] * size + m[1] for m in state.history]
        hc = [m[0] * size + m[1] for m in getattr(state, "handicaps", [])]
        rec = hc + flat
        if len(rec) > mv.shape[0]:
            raise ValueError("game record longer than the channel's root record")
        mv[:len(rec)] = rec
        meta[:] = [len(flat), len(hc), size, int(bool(state.enforce_superko)),
                   int(round(state.komi * 2)), np.int64(np.uint64(s.root_board.hash).view(
                       np.int64)), int(state.current_player), 0]

    def stop(self):
        """Rank 0: release the serving ranks, its own serving thread included (serve() returns
        None)."""
        if self.chan is not None and self.rank == 0:
            self.chan.post_cmd(_rg.CHAN_CMD_STOP, 0)
            self._join_local()

    def update_with_move(self, last_move):
        if self.rank == 0:
            super(DistributedMCTS, self).update_with_move(last_move)

    def leaf_counts(self):
        """Leaves evaluated by each rank (rank 0 knows them all; the others their own)."""
        if self.rank == 0:
            return self.leaves_per_rank.astype(np.float64)
        c = np.zeros(self.world)
        c[self.rank] = self.rank_leaves
        return c

    # ------------------------------------------------------------------ every rank: serving
    def _worker_search(self, root):
        """This rank's leaf builder: a native Search whose waves are loaded from path records
        (its own tree is never grown)."""
        ws = self._ws
        if ws is None:
            ws = self._ws = _rg.Search(root, self.worker_threads)
        elif ws.root_board.hash != root.hash or \
                ws.root_board.current_player != root.current_player:
            ws.reset(root)
        ws.keyed_rollouts = bool(getattr(self, "keyed_rollouts", False))
        ws.rollout_limit = self.rollout_limit
        ws.seed = self.seed
        ws.set_rollout_policy(self.rollout)
        return ws

    def _root_for(self, rhash):
        """The board whose hash the master's request carries: rank 0's own state, else the
        position replayed from the channel's root record."""
        st = getattr(self, "_local_state", None) if self.rank == 0 else None
        if st is not None and np.uint64(st.native.hash) == np.uint64(rhash):
            return st.native
        cached = getattr(self, "_root_cache", None)
        if cached is not None and np.uint64(cached.native.hash) == np.uint64(rhash):
            return cached.native
        meta = self.chan.view(0, 0, "root_meta").copy()
        rec = self.chan.view(0, 0, "root_moves")
        nm, nh, size, superko, komi2, h, ptm = (int(x) for x in meta[:7])
        st = go.GameState(size=size, komi=komi2 / 2.0, enforce_superko=bool(superko))
        if nh:
            st.place_handicaps([divmod(int(a), size) for a in rec[:nh]])
        for a in rec[nh:nh + nm]:
            st.do_move(PASS_MOVE if a < 0 else divmod(int(a), size))
        if np.uint64(st.native.hash) != np.uint64(rhash) or st.current_player != ptm:
            raise RuntimeError("rank %d: the root replayed from the game record does not match "
                               "the master's (hash %x vs %x)" % (self.rank, st.native.hash,
                                                                 np.uint64(rhash)))
        self._root_cache = st
        return st.native

    def _slot_views(self, r):
        if self._views is None or self._views[0] != r:
            ch = self.chan
            self._views = (r, [{w: ch.view(r, k, w) for w in ("paths", "priors", "values",
                                                               "sens", "z")}
                               for k in range(ch.nslots)])
        return self._views[1]

    def serve(self, rank=None):
        """Evaluate this rank's waves until the master decides a move (returned) or stops
        (None). Waves are accepted in slot order; up to ``depth`` are on the GPU at once, and a
        wave's slot is answered twice: values when its network pass is done, rollout results
        when its rollouts are."""
        r = self.rank if rank is None else rank
        ch = self.chan
        K = ch.nslots
        views = self._slot_views(r)
        evq = collections.deque()  # [slot, wave, n, value handle, rollout handle]
        zq = collections.deque()   # [slot, wave, rollout handle, index of the wave]
        recv = 0
        ws = None
        last_req = None
        while True:
            busy = bool(evq or zq)
            got = 0
            if len(evq) < self.depth:
                k = self._wk
                got = ch.wait_request(r, k, self._wseq[k], self._wcmd,
                                      self.idle_us if busy else 500)
                if got == 1:
                    seq, n, wave, seed, rhash = ch.slot_info(r, k)
                    self._wseq[k] = seq
                    root = self._root_for(rhash)
                    ws = self._worker_search(root)
                    wid = ws.load_paths(views[k]["paths"][:n])
                    evq.append(self._start(ws, wid, n, k, seed))
                    self._wk = (k + 1) % K
                    self.rank_leaves += n
                    recv += 1
                    continue  # take every waiting request before retiring anything
                if got == 2 and not busy:
                    seq, cmd, arg = ch.cmd()
                    self._wcmd = seq
                    if cmd == _rg.CHAN_CMD_MOVE:
                        return PASS_MOVE if arg < 0 else divmod(int(arg), self.S)
                    if cmd == _rg.CHAN_CMD_STOP:
                        return None
            # values: the oldest wave once its pass is done (blocking only with `depth` waves
            # on the GPU); emulating the GPU's latency (the CPU study), only with `depth` waves
            # received or nothing more coming for idle_us
            now = time.perf_counter()
            if got == 1 or last_req is None:
                last_req = now
            quiet = got == 0 and now - last_req > self.flush_s
            idle = self.emulate_latency and got == 0 and len(evq) < self.depth
            while evq and (len(evq) >= self.depth or idle or
                           (not self.emulate_latency and _done(evq[0][3]))):
                k, wid, n, h, roll = evq.popleft()
                self._post_values(views[k], r, k, n, h, ws)
                if roll is None:
                    ws.drop_wave(wid)
                else:
                    zq.append([k, wid, roll, recv])
            # rollout results, in slot order. A partial rollout group is launched when the master
            # cannot send more (every slot of this rank holds a wave) or has sent nothing for
            # flush_s (the end of a search); emulating, results are held back `rollout_delay`
            # waves unless nothing more comes
            idle = got == 0 and not evq
            if zq and self._batcher is not None and self._batcher.cur is not None and \
                    (len(evq) + len(zq) >= self.nslots or (quiet and not evq)):
                self._batcher.flush()
            hold = self.rollout_delay if self.emulate_latency else 0
            while zq and zq[0][2].done() and (recv - zq[0][3] >= hold or idle):
                k, wid, roll, _ = zq.popleft()
                z = roll.result()
                views[k]["z"][:len(z)] = z
                ch.post_z(r, k)
                ws.drop_wave(wid)

    def _start(self, ws, wid, n, k, seed):
        """Start a loaded wave: its network pass (GPU: packed pinned slot, async) and its
        rollouts. Returns the evq entry."""
        ev = self.evaluator
        h = None
        if self.gpu is not None and getattr(ev, "wave_capable", None) is not None and \
                ev.wave_capable(self.S):
            if self._wslots is None:
                self._wslots = _Slots(ev.gpu["p"].device, self.depth)
            h = ev.submit_wave(ws, wid, n, self._wslots, int(max(self.batches)))
        roll = None
        if self.lmbda > 0:
            mode = self.worker_rollouts
            if mode == "null":
                roll = _ZNow(n)
            elif mode == "gpu":
                if self._batcher is None:
                    from .gpu_rollout import GpuRollouts, RolloutBatcher
                    self._batcher = RolloutBatcher(
                        GpuRollouts(self.rollout, self.gpu, slice_moves=self.ROLLOUT_SLICE),
                        self.rollout_group)
                roll = self._batcher.add(ws, wid, self.rollouts_per_leaf, self.rollout_limit,
                                         seed=int(seed) & 0x7FFFFFFF)
            else:
                ws.start_rollouts(wid)
                roll = _ZCpu(ws, wid)
        if h is None:
            h = _Sync(ev, ws.leaf_boards(wid), self.worker_threads)
        return [k, wid, n, h, roll]

    def _post_values(self, v, r, k, n, h, ws):
        pri, val, sens = h.result()
        if pri is not None:
            v["priors"][:n, :pri.shape[1]] = pri[:n]
        else:
            v["priors"][:n] = 1.0
        v["values"][:n] = 0.0 if val is None else np.asarray(val, np.float32).reshape(-1)[:n]
        v["sens"][:n] = sens[:n]
        self.chan.post_values(r, k)


class _Sync(object):
    """A wave evaluated on the host at once (CPU networks, the null evaluator): (priors,
    values, sensible) with the sensible mask made natively when the features lack it."""

    def __init__(self, ev, boards, nthreads):
        res = ev(boards)
        pri, val = res[0], res[1]
        sens = res[2] if len(res) > 2 else None
        if sens is None:
            from ..features.preprocessing import _FID
            sens = _rg.batch_features(boards, [_FID["sensibleness"]], nthreads)
        self.res = (None if pri is None else np.ascontiguousarray(pri, np.float32), val,
                    np.ascontiguousarray(np.asarray(sens).reshape(len(boards), -1), np.uint8))

    def result(self):
        return self.res


class RootExchange(object):
    """Asynchronous all-reduce (sum) of a small float32 vector, one in flight: exchange(v) posts
    v and returns the (sum, own contribution) of the previous exchange (None the first time).
    On GPUs the collective runs on its own stream (RCCL), staged through pinned memory, so it
    never waits for the search's network work queued on the other streams."""

    def __init__(self, n, device):
        self.n = int(n)
        self.gpu = device.type == "cuda"
        self.device = device
        self.pending = None
        self.k = 0
        if self.gpu:
            self.stream = torch.cuda.Stream(device)
            self.dev = [torch.empty(self.n, dtype=torch.float32, device=device) for _ in range(2)]
            self.hin = [torch.empty(self.n, dtype=torch.float32, pin_memory=True)
                        for _ in range(2)]
            self.hout = [torch.empty(self.n, dtype=torch.float32, pin_memory=True)
                         for _ in range(2)]
            self.events = [torch.cuda.Event() for _ in range(2)]

    def exchange(self, vec):
        prev = self.wait()
        self._post(np.asarray(vec, np.float32))
        return prev

    def wait(self):
        """Result of the exchange in flight (None if none)."""
        p, self.pending = self.pending, None
        if p is None:
            return None
        if self.gpu:
            ev, hout, own = p
            ev.synchronize()
            return hout.numpy().copy(), own
        work, t, own = p
        work.wait()
        return t.numpy(), own

    def _post(self, vec):
        if vec.size != self.n:
            raise ValueError("exchange vector of %d, expected %d" % (vec.size, self.n))
        if not self.gpu:
            t = torch.from_numpy(vec.copy())
            self.pending = (dist.all_reduce(t, async_op=True), t, vec.copy())
            return
        k = self.k = (self.k + 1) % 2
        hin, buf, hout, ev = self.hin[k], self.dev[k], self.hout[k], self.events[k]
        hin.numpy()[:] = vec  # the previous use of this buffer completed (waited above)
        with torch.cuda.stream(self.stream):
            buf.copy_(hin, non_blocking=True)
            work = dist.all_reduce(buf, async_op=True)
            work.wait()  # the exchange stream waits for the collective (no host block)
            hout.copy_(buf, non_blocking=True)
            ev.record(self.stream)
        self.pending = (ev, hout, vec.copy())


class SharedRootMCTS(ParallelMCTS):
    """APV-MCTS over all ranks of ``dp`` with shared root statistics (see the module doc).

    Call ``get_move(state)`` on every rank with the same state (all ranks return the same move)
    and ``update_with_move(move)`` on every rank. ``n_playout`` is the whole job's budget per
    move; each rank runs its share."""

    def __init__(self, policy=None, value=None, rollout=None, dp=None, **kw):
        super(SharedRootMCTS, self).__init__(policy, value, rollout, dp=dp, **kw)
        self.world = self.dp.world if self.dp is not None else 1
        self.exchanges = 0

    def search(self, state, n_playout=None, tick=None):
        total = int(n_playout or self.n_playout)
        if self.world == 1:
            return super(SharedRootMCTS, self).search(state, total, tick)
        M = state.size * state.size + 1
        dev = self.dp.device
        if self.dp.backend == "gloo":
            dev = torch.device("cpu")
        xch = RootExchange(4 * M + 2, dev)
        ext = np.zeros((4, M), np.float32)
        state_box = {"all_done": False}

        def step(s, done):
            d = s.root_deltas()
            vec = np.concatenate([d.reshape(-1), np.array([1.0 if done else 0.0,
                                                           float(d[0].sum())], np.float32)])
            prev = xch.exchange(vec)
            self.exchanges += 1
            if prev is None:
                return
            tot, own = prev
            ext[:] += (tot[:4 * M] - own[:4 * M]).reshape(4, M)
            s.set_root_external(ext)
            state_box["all_done"] = tot[4 * M] >= self.world - 0.5

        def on_wave(s):
            step(s, False)
            if tick is not None:
                tick(s)

        share = int(math.ceil(total / float(self.world)))
        s = super(SharedRootMCTS, self).search(state, share, on_wave)
        # this rank is done: keep exchanging (zero deltas, done flag) until every rank is, so
        # that all ranks issue the same sequence of collectives
        while not state_box["all_done"]:
            step(s, True)
        xch.wait()
        return s
