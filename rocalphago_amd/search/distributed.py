"""APV-MCTS on several GPUs (the reference's ParallelMCTS is an empty stub,
AlphaGo/mcts.py:219-220). One process per GPU, torch.distributed "nccl" = RCCL between them
(gloo in the CPU tests). Two designs, compared by search/efficiency.py (one tree with the same
total budget as the yardstick; profiles/search_efficiency_r4.json):

DistributedMCTS (default since round 4: ``bench.py --gpus N``, ``benchmarks/mcts_bench.py
--distributed``) is ONE search: one tree on rank 0, each round's leaves evaluated on all GPUs
(below). With the one-GPU search's leaves in flight per round (N waves of 512 / N, at least 128)
its budget efficiency is 1.0 at N = 2, 4, 8 and no node is expanded twice; its rate is bounded by
rank 0's host tree work (select + pack + backup, ~2.2 us per simulation:
benchmarks/mcts_null_bench.py), not by N.

SharedRootMCTS (``mode="shared"``) — every rank runs the full single-GPU pipelined search on the
same position and the ranks all-reduce the statistics their trees added at the root's children
after every wave (4 x 362 floats, one wave of lag), mixed into each rank's root selection
(Search.set_root_external). Measured: the N trees expand the same nodes (duplication N with a
deterministic evaluator) and the job searches like ONE rank (efficiency 1/N), so its N-fold
simulations/s over-credit the search; the bench reports its live duplication. Kept for
comparison.

DistributedMCTS (``mode="master"``) — one tree on rank 0, leaf evaluation spread over all ranks:

  * rank 0 owns the only tree (the native ``_rocgo.Search``). Every *round* it selects one wave of
    ``batch`` leaves per rank (virtual loss keeps the waves apart), packs each wave's leaves as
    flat per-point records (LeafCodec: colours, stone ages, player / ko / last moves / passes, and
    — only for boards that enforce positional superko — the superko-illegal mask and the ladder
    planes the master computed) and broadcasts them;
  * every rank, rank 0 included, rebuilds its wave's leaf boards from the records
    (``Board.from_arrays``), reads the ladders on its own host thread pool, builds the feature
    planes with the HIP feature kernel, runs the policy and value networks and starts the wave's
    fast rollouts on its rollout streams (WaveEvaluator). It returns the priors, values and
    sensible-move masks of this round's wave and the rollout results of the wave it started
    ``rollout_delay`` rounds earlier at the latest -- as soon as they are done, usually the next
    round or two (rollouts take longer than a network pass; the native tree keeps such a wave's
    virtual loss until its rollout backup, as in the single-GPU pipeline);
  * results come back to rank 0 with one gather; it backs them up and selects the next round.

So the tree, the selection and the backups stay on one host (no tree synchronisation), and all
the per-leaf work that scales — ladder reading, features, both networks, rollouts — is split
over the GPUs and their host threads. Plain root parallelism (independent trees, visit counts
all-reduced only at the end) remains available as ``ParallelMCTS(dp=...)``.
"""
import math
import collections
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from .._native import engine as _engine
from ..engine import gamestate as go
from ..engine.gamestate import PASS_MOVE
from .apv import ParallelMCTS

_rg = _engine()

CMD_ROUND, CMD_MOVE, CMD_STOP, CMD_FLUSH = 0, 1, 2, 3
HDR = 8  # header words before the per-rank leaf counts


class LeafCodec(object):
    """Per-leaf byte records: colours [P] int8 | ages [P] int16 | meta8 [8] int32 |
    superko-illegal [P] uint8 | ladder planes [2, P] uint8 (the last two only meaningful when the
    wave's boards enforce superko)."""

    def __init__(self, S, superko=True):
        self.S = S
        P = self.P = S * S
        self.o_age = P
        self.o_meta = 3 * P
        self.o_ill = 3 * P + 32
        self.o_lad = 4 * P + 32
        # without positional superko the leaves' ladder planes are read by the evaluating rank
        # and there is no illegal mask: the record stops after the meta words (half the bytes)
        self.superko = bool(superko)
        self.L = (6 * P + 32 + 7) // 8 * 8 if superko else (3 * P + 32 + 7) // 8 * 8

    def pack(self, search, wid, nthreads, out=None):
        """The wave's records, written by the native search straight into the record columns
        (one parallel pass over the leaves; ``out``: a [>= n, L] uint8 buffer to fill, e.g. a
        row of the round's scatter buffer). Returns (records [n, L], superko)."""
        superko = self.superko
        n, P = search.num_leaves(wid), self.P
        rec = out[:n] if out is not None else np.empty((n, self.L), np.uint8)
        search.pack_inputs(wid, colors=rec[:, :P].view(np.int8),
                           ages=rec[:, self.o_age:self.o_meta].view(np.int16),
                           meta8=rec[:, self.o_meta:self.o_ill].view(np.int32),
                           illegal=rec[:, self.o_ill:self.o_lad] if superko else None,
                           ladders=rec[:, self.o_lad:self.o_lad + 2 * P] if superko else None)
        return rec, superko

    def unpack(self, rec):
        P = self.P
        colors = np.ascontiguousarray(rec[:, :P]).view(np.int8)
        ages = np.ascontiguousarray(rec[:, self.o_age:self.o_meta]).view(np.int16)
        meta8 = np.ascontiguousarray(rec[:, self.o_meta:self.o_ill]).view(np.int32)
        if not self.superko:
            return colors, ages, meta8, None, None
        illegal = np.ascontiguousarray(rec[:, self.o_ill:self.o_lad])
        lad = np.ascontiguousarray(rec[:, self.o_lad:self.o_lad + 2 * P]).reshape(-1, 2, P)
        return colors, ages, meta8, illegal, lad


class WaveEvaluator(object):
    """Evaluates one shipped wave on this rank: (priors [n, P], values [n], sensible [n, P]) and
    a rollout handle whose ``result()`` is the mean outcome per leaf for BLACK."""

    def __init__(self, net, rollout, lmbda, rollouts_per_leaf=1, rollout_limit=500, nthreads=8):
        self.net = net  # a NetworkEvaluator
        self.rollout = rollout
        self.lmbda = lmbda
        self.R = int(rollouts_per_leaf)
        self.limit = int(rollout_limit)
        self.nthreads = nthreads
        self.keyed = False  # CPU rollouts seeded by the leaf position (search/efficiency.py)
        model = net.policy if net.policy is not None else net.value
        inner = getattr(getattr(model, "model", None), "net", None)  # (None: a host evaluator)
        self.device = inner.device if inner is not None else torch.device("cpu")
        self.gpu = self.device.type == "cuda"
        self._gro = None
        # the networks run on their own stream: the collectives queued on the default stream
        # (and the host syncs on their results) must not wait for a wave still being evaluated
        self.stream = torch.cuda.Stream(self.device) if self.gpu else None

    def _boards(self, colors, ages, meta8, S, komi):
        zw, zb, _ = go._zobrist(S)
        return _rg.boards_from_arrays(colors, ages, meta8, S, komi, zw.ravel(), zb.ravel())

    def __call__(self, codec, rec, superko, komi, seed):
        ev, pend = self.submit(codec, rec, superko, komi, seed)
        pr, v, sens = ev.result()
        return pr, v, sens, pend

    def submit(self, codec, rec, superko, komi, seed, boards=None):
        """Start the wave's evaluation: (handle whose result() is (priors, values, sensible) as
        numpy, rollout handle or None). On the GPU the networks run asynchronously into pinned
        host buffers, so the caller can take part in collectives meanwhile. ``boards``: the
        leaves' native boards when this rank has them (rank 0's own wave: the tree's leaf
        boards), instead of rebuilding them from the records."""
        colors, ages, meta8, illegal, lad = codec.unpack(rec)
        if boards is None:
            boards = self._boards(colors, ages, meta8, codec.S, komi)
        pend = self._rollouts(boards, colors, meta8, codec.S, komi, seed) \
            if self.lmbda > 0 else None
        if self.gpu:
            with torch.cuda.stream(self.stream):
                return self._gpu_eval(boards, colors, ages, meta8, illegal, lad, superko), pend
        res = self.net(boards)
        return _Done(tuple(res[:3]) if len(res) > 2 else (res[0], res[1], None)), pend

    def planes(self, boards, colors, ages, meta8, illegal, lad, superko):
        """(policy planes, value planes, the planes holding the sensibleness plane) of a
        shipped wave on the device: from the master's superko-aware ladder planes and illegal
        mask when the boards enforce superko, else the evaluator's HIP feature path on the
        rebuilt boards (the single-GPU search's own path)."""
        ev = self.net
        ev._plans()
        n = len(boards)

        def one(key):
            if superko:
                meta4 = np.zeros((n, 4), np.int32)
                meta4[:, :2] = meta8[:, :2]
                meta4[:, 2] = 1
                return ev.gpu[key].from_arrays(colors, ages, meta4, illegal, lad)
            return ev.gpu[key](boards)

        if ev.shared or ev.value is None:
            x = one("p")
            return (x[:, :ev.npol].contiguous() if ev.shared else x), x, x
        xp = one("p") if ev.policy is not None else None
        xv = one("v")
        return xp, xv, (xp if xp is not None else xv)

    def _gpu_eval(self, boards, colors, ages, meta8, illegal, lad, superko):
        ev = self.net
        plans = ev._plans()
        n = len(boards)
        xp, xv, x = self.planes(boards, colors, ages, meta8, illegal, lad, superko)
        ppol, pval = plans
        with torch.no_grad():
            sens = x[:, ev._sens_off].reshape(n, -1) if ev._sens_off is not None else None
            pr = ppol.forward(xp) if ppol is not None else None
            v = pval.forward(xv).reshape(-1) if pval is not None else None
        host = []
        for t in (pr, v, sens):
            if t is None:
                host.append(None)
                continue
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            host.append(h)
        done = torch.cuda.Event()
        done.record()
        return _Copied(done, host)

    def _rollouts(self, boards, colors, meta8, S, komi, seed):
        if self.gpu:
            if self._gro is None:
                from .gpu_rollout import GpuRollouts
                self._gro = GpuRollouts(self.rollout, self.device)
            from .gpu_rollout import _Pending
            ev, _, _, _, host = self._gro._launch(colors, meta8, S, komi, self.R, self.limit,
                                                  seed)
            return _Pending(ev, host, colors.shape[0], self.R)
        win = self.rollout.rollouts(boards, seed=seed, limit=self.limit, nthreads=self.nthreads,
                                    keyed=self.keyed)
        z = np.where(win == go.BLACK, 1.0, np.where(win == go.WHITE, -1.0, 0.0))
        return _Done(z.astype(np.float32))


class _Done(object):
    def __init__(self, value):
        self.value = value

    def result(self):
        return self.value


class _Copied(object):
    """Device results copied into pinned host tensors; valid once ``event`` completed."""

    def __init__(self, event, host):
        self.event, self.host = event, host

    def result(self):
        self.event.synchronize()
        return tuple(None if h is None else h.float().numpy() if h.dtype != torch.uint8
                     else h.numpy() for h in self.host)


class DistributedMCTS(ParallelMCTS):
    """One search tree on rank 0, leaf evaluation spread over all ranks (see module doc).

    Call ``get_move(state)`` on EVERY rank (all ranks return the same move; only rank 0's
    ``state`` is read) and ``update_with_move(move)`` on every rank after playing it."""

    def __init__(self, policy=None, value=None, rollout=None, dp=None, rollout_delay=6,
                 force_master=None, **kw):
        """``force_master`` (default: RAG_FORCE_PG=1): run the round loop — record packing,
        WaveEvaluator on shipped records, the round pipeline — even with one rank, instead of
        the single-GPU ParallelMCTS search (the GPU tests of the multi-GPU leaf path)."""
        kw.setdefault("pipeline", 1)
        super(DistributedMCTS, self).__init__(policy, value, rollout, dp=None, **kw)
        if force_master is None:
            force_master = os.environ.get("RAG_FORCE_PG") == "1"
        self.force_master = bool(force_master)
        self.ddp = dp
        self.world = dp.world if dp is not None and dp.enabled else 1
        self.rank = dp.rank if dp is not None and dp.enabled else 0
        self.device = dp.device if dp is not None else torch.device("cpu")
        if self.world > 1 and dist.get_backend() == "gloo":
            self.device = torch.device("cpu")  # gloo collectives on host tensors
        self.delay = max(0, int(rollout_delay)) if self.lmbda > 0 else 0
        self.leaf_eval = WaveEvaluator(self.evaluator, self.rollout, self.lmbda,
                                       self.rollouts_per_leaf, self.rollout_limit,
                                       self.nthreads)
        self._pending = collections.deque()  # (round, rollout handle) of this rank's waves
        self.rank_leaves = 0
        self._round = 0

    # ------------------------------------------------------------------ collectives
    def _bcast(self, t):
        if self.world > 1:
            dist.broadcast(t, 0)
        return t

    def _header(self, cmd, counts, extra=0, superko=0, komi=7.5, S=19, gather=0):
        h = torch.zeros(HDR + self.world, dtype=torch.int64, device=self.device)
        if self.rank == 0:
            h[:HDR] = torch.tensor([cmd, self._round, extra, superko, int(komi * 2), S,
                                    int(gather), 0])
            if counts is not None:
                h[HDR:] = torch.tensor(counts, dtype=torch.int64)
        return self._bcast(h).cpu().numpy()

    def _round_records(self, codec):
        """Rank 0's [world, batch, L] record buffer of a round (reused; a wave's rows past its
        leaf count are stale and never read)."""
        buf = getattr(self, "_recbuf", None)
        if buf is None or buf.shape[2] != codec.L:
            buf = self._recbuf = np.zeros((self.world, self.batch, codec.L), np.uint8)
        return buf

    def _ship(self, codec, recs, counts, superko, komi):
        """Phase 1 of a round on every rank: receive the waves, start evaluating this rank's."""
        B = self.batch
        rnd = self._round
        n = int(counts[self.rank])
        if int(np.sum(counts)) == 0:  # an empty round only carries rollout results back
            return (rnd, 0, None, codec)
        mine = None
        if self.world > 1:
            # each rank receives only its own wave's records (scatter, not a broadcast of all);
            # rank 0's round buffer goes to the device in one copy
            buf = torch.empty((B, codec.L), dtype=torch.uint8, device=self.device)
            if self.rank == 0:
                allr = torch.from_numpy(self._round_records(codec)).to(self.device)
                dist.scatter(buf, scatter_list=list(allr.unbind(0)), src=0)
            else:
                dist.scatter(buf, src=0)
            if n:
                mine = recs[0] if self.rank == 0 else buf[:n].cpu().numpy()
        handle = None
        if n:
            mine = mine if mine is not None else recs[0]
            seed = (self.seed * 7919 + rnd * 131 + self.rank) & 0x7FFFFFFF
            own = getattr(self, "_own_boards", None) if self.rank == 0 else None
            handle, pend = self.leaf_eval.submit(codec, mine, superko, komi, seed, boards=own)
            if pend is not None:
                self._pending.append((rnd, pend))
            self.rank_leaves += n
        return (rnd, n, handle, codec)

    def _collect(self, shipped):
        """Phase 2: this rank's results of a shipped round (and the rollout results of the wave
        it started ``rollout_delay`` rounds earlier) all-gathered to rank 0. Returns (on rank 0)
        per rank (priors, values, sens, (round, z) or None)."""
        rnd, n, handle, codec = shipped
        P = codec.P
        PW = self._prior_width(P)  # P, or P + 1 with the network's pass probability
        B = self.batch
        W = PW + P + 3  # priors | sensible | value | rollout z | pad
        out = np.zeros((B, W), np.float32)
        meta = np.zeros(4, np.float32)  # [n, z round, z count, 0]
        if n:
            pr, v, sens = handle.result()
            if pr is not None:
                out[:n, :PW] = pr[:, :PW]
            if sens is not None:
                out[:n, PW:PW + P] = sens
            if v is not None:
                out[:n, PW + P] = v
        meta[0] = n
        # the oldest pending rollout wave comes back as soon as it is done (its leaves keep
        # their virtual loss until then), and at the latest `rollout_delay` rounds after it was
        # shipped (then this collect waits for it)
        # (never a wave shipped after the collected round: rank 0 backs its values up first)
        if self._pending and self._pending[0][0] <= rnd and (
                self._pending[0][0] <= rnd - self.delay or n == 0 or
                getattr(self._pending[0][1], "done", lambda: True)()):
            zr, pend = self._pending.popleft()
            z = pend.result()
            out[:len(z), PW + P + 1] = z
            meta[1], meta[2] = zr, len(z)
        flat = np.concatenate([out.reshape(-1), meta])
        if self.world > 1:
            # to rank 0 only (gather, not all_gather: the other ranks never read the results)
            flat = torch.from_numpy(flat).to(self.device)
            if self.rank == 0:
                gathered = [torch.empty_like(flat) for _ in range(self.world)]
                dist.gather(flat, gather_list=gathered, dst=0)
                gathered = torch.stack(gathered).cpu().numpy()
            else:
                dist.gather(flat, dst=0)
                gathered = None
        else:
            gathered = [flat]
        if self.rank != 0:
            return None
        res = []
        for g in gathered:
            o, m = g[:-4].reshape(B, W), g[-4:]
            k = int(m[0])
            zr = (int(m[1]), o[:int(m[2]), PW + P + 1].copy()) if m[2] > 0 else None
            res.append((np.ascontiguousarray(o[:k, :PW]), o[:k, PW + P], o[:k, PW:PW + P] > 0.5,
                        zr))
        return res

    def _prior_width(self, P):
        from ..models.policy import has_pass_logit
        return P + (1 if has_pass_logit(self.evaluator.policy) else 0)

    def _round_trip(self, codec, recs, counts, superko, komi):
        """Ship and collect one round (unpipelined)."""
        return self._collect(self._ship(codec, recs, counts, superko, komi))

    # ------------------------------------------------------------------ rank 0: the search
    def search(self, state, n_playout=None):
        """Two rounds in flight: rank 0 selects and ships round k+1 while every GPU still
        evaluates round k, then collects and backs up round k (virtual loss keeps the two rounds'
        leaves apart, as in the single-GPU pipeline)."""
        s = self._sync_root(state)
        codec = LeafCodec(state.size, bool(s.root_board.enforce_superko))
        target = s.root_visits + (n_playout or self.n_playout)
        # round -> [wave id, leaf counts per rank, {rank: rollout z}] until its rollouts are in
        waves = {}
        inflight = None  # (shipped, counts, wid) of the round not collected yet
        stall = 0
        # rank 0's round split: tree selection, record packing, header + scatter + starting its
        # own wave, collecting (its own results + the gather), backups
        tm = dict.fromkeys(("t_select", "t_pack", "t_ship", "t_gather", "t_backup"), 0.0)
        rounds = 0
        superko = int(s.root_board.enforce_superko)
        B, W = self.batch, self.world
        while True:
            # ONE native wave per round (one parallel descent + board build, one record pack,
            # one value backup, one rollout backup), dealt to the ranks in contiguous chunks of
            # at most `batch` leaves: leaf i goes to rank i // batch
            t0 = time.perf_counter()
            room = target - s.root_visits - (sum(inflight[1]) if inflight else 0)
            want = min(B * W, max(room, 0))
            wid, n = s.select(want) if want > 0 else (-1, 0)
            counts = [max(0, min(B, n - r * B)) for r in range(W)]
            recs = [None] * W
            ta = time.perf_counter()
            if n > 0:
                flat = self._round_records(codec).reshape(W * B, codec.L)
                codec.pack(s, wid, self.nthreads, out=flat)
                recs = [flat[r * B:r * B + c] if c else None for r, c in enumerate(counts)]
            t1 = time.perf_counter()
            if n == 0 and inflight is None and not waves:
                stall += 1
                if stall > 3 or s.root_visits >= target:
                    break
                continue
            stall = 0
            shipped = None
            if n or not inflight:
                # a new round (possibly empty: it only brings rollout results back)
                self._header(CMD_ROUND, counts, superko=superko, komi=state.komi, S=state.size,
                             gather=inflight is not None)
                self._own_boards = s.leaf_boards(wid)[:counts[0]] if counts[0] else None
                shipped = self._ship(codec, recs, counts, superko, state.komi)
                self._own_boards = None
                self._round += 1
            else:
                self._header(CMD_FLUSH, [0] * W, gather=1)
            ts = time.perf_counter()
            res = self._collect(inflight[0]) if inflight is not None else None
            t2 = time.perf_counter()
            if res is not None:
                self._backup(s, res, inflight, waves)
            inflight = (shipped, counts, wid) if shipped is not None else None
            rounds += 1
            tm["t_select"] += ta - t0
            tm["t_pack"] += t1 - ta
            tm["t_ship"] += ts - t1
            tm["t_gather"] += t2 - ts
            tm["t_backup"] += time.perf_counter() - t2
            if s.root_visits >= target and not waves and inflight is None:
                break
            if s.root_visits >= target and not waves and inflight is not None and \
                    sum(inflight[1]) == 0:
                self._header(CMD_FLUSH, [0] * W, gather=1)
                self._backup(s, self._collect(inflight[0]), inflight, waves)
                break
        for k, v in tm.items():
            self._acc(k, v)
        # (t_eval: everything between selection and backup, the pre-round-5 split)
        self._acc("t_eval", tm["t_ship"] + tm["t_gather"])
        self._acc("rounds", rounds)
        return s

    def _backup(self, s, res, inflight, waves):
        """Back up a collected round: the value backup of its wave (the ranks' results joined
        in leaf order), and every rollout result that came back with it — a round's rollouts
        are backed up once all the ranks that evaluated leaves of it have returned theirs."""
        shipped, counts, wid = inflight
        rnd = shipped[0]
        live = [r for r in range(len(counts)) if counts[r]]
        if live:
            cat = (lambda i: res[live[0]][i]) if len(live) == 1 else \
                (lambda i: np.concatenate([res[r][i] for r in live]))
            s.backup_value(wid, cat(0) if self.evaluator.policy is not None else None,
                           cat(1) if self.evaluator.value is not None else None,
                           cat(2).astype(np.uint8) if self._has_sens() else None)
            if self.lmbda > 0:
                waves[rnd] = [wid, list(counts), {}]
        for r, (_, _, _, zr) in enumerate(res):
            if zr is None:
                continue
            ent = waves[zr[0]]
            ent[2][r] = zr[1]
            if len(ent[2]) == sum(1 for c in ent[1] if c):
                z = np.concatenate([ent[2][q] for q in range(len(ent[1])) if ent[1][q]])
                s.backup_rollout(ent[0], z)
                del waves[zr[0]]
        self.stats["waves"] += len(live)
        self.stats["sims"] += sum(counts)

    def _has_sens(self):
        self.evaluator._plans()
        return self.evaluator._sens_off is not None

    def get_move(self, state):
        if self.world == 1 and not self.force_master:
            return super(DistributedMCTS, self).get_move(state)
        if self.rank != 0:
            return self.serve()
        try:
            s = self.search(state)
        except BaseException:
            self.stop()  # release the serving ranks before failing
            raise
        a = s.best_move()
        self._header(CMD_MOVE, [0] * self.world, extra=int(a))
        return PASS_MOVE if a < 0 else divmod(int(a), state.size)

    def update_with_move(self, last_move):
        if self.rank == 0:
            super(DistributedMCTS, self).update_with_move(last_move)

    # ------------------------------------------------------------------ ranks > 0
    def serve(self):
        """Evaluate rounds until rank 0 decides a move (returned) or stops (None)."""
        inflight = None
        while True:
            h = self._header(None, None)
            cmd, self._round = int(h[0]), int(h[1])
            if cmd == CMD_MOVE:
                a = int(h[2])
                S = int(h[5]) or 19
                return PASS_MOVE if a < 0 else divmod(a, S)
            if cmd == CMD_STOP:
                return None
            if cmd == CMD_FLUSH:
                self._collect(inflight)
                inflight = None
                continue
            shipped = self._ship(LeafCodec(int(h[5]), bool(h[3])), None, h[HDR:], int(h[3]),
                                 h[4] / 2.0)
            if int(h[6]):
                self._collect(inflight)
            inflight = shipped

    def stop(self):
        """Rank 0: release the serving ranks (their serve() returns None)."""
        if self.world > 1 and self.rank == 0:
            self._header(CMD_STOP, [0] * self.world)

    def leaf_counts(self):
        """Leaves evaluated by each rank (collective: call on every rank)."""
        t = torch.zeros(self.world, dtype=torch.float64, device=self.device)
        t[self.rank] = self.rank_leaves
        if self.world > 1:
            dist.all_reduce(t)
        return t.cpu().numpy()


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
