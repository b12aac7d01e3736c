"""Native lock-step self-play on the GPU (RL policy training, value-dataset generation).

The reference advances its self-play games in a Python loop: per ply every unfinished game's
features are extracted, the batch is evaluated, and ``do_move`` is called game by game
(/root/reference/AlphaGo/training/reinforcement_policy_trainer.py:51-75,
/root/reference/AlphaGo/ai.py:107-133). ``NativeSelfPlay`` keeps the games in a native
``_rocgo.GameBatch``; one ply of all games that are to move is

  1. ``GameBatch.pack``: colours / stone ages / player+ko (and host-read ladder planes) of those
     games written in parallel into pinned buffers;
  2. one GPU pass: copies in, the HIP feature kernel (planes + sensible-move mask), the fused
     policy plan, the Gumbel-max sampling kernel over p^beta restricted to the sensible moves
     (the players' rule: ProbabilisticPolicyPlayer / GreedyPolicyPlayer, ai.py); only the chosen
     points come back;
  3. ``GameBatch.play``: the whole ply applied natively in parallel (move limit -> pass, as
     ai.py's ``len(history) > move_limit``).

The games are split into ``pipeline`` independent groups whose plies alternate: the chosen
points come back through pinned memory behind an event, so while the GPU runs one group's ply
the host applies and packs the other's (the host work of a ply is hidden behind GPU work).

The learner's planes stay on the device for the REINFORCE update (rows of the positions where
it did not pass, the reference's ``_make_training_pair`` rows), one [n, F, S, S] block per game.
"""
import numpy as np
import torch

from .._native import engine as _engine
from ..engine import gamestate as go

_rg = _engine()


def _player_kind(player):
    from ..players.ai import GreedyPolicyPlayer, ProbabilisticPolicyPlayer
    if isinstance(player, ProbabilisticPolicyPlayer):
        return "prob"
    if isinstance(player, GreedyPolicyPlayer):
        return "greedy"
    return None


class NativeSelfPlay(object):
    """Lock-step games of ``learner`` vs ``opponent`` (policy players on HIP models)."""

    def __init__(self, learner, opponent, nthreads=16, pipeline=2, graphs=True):
        self.learner, self.opponent = learner, opponent
        self.nthreads = nthreads
        self.pipeline = max(1, int(pipeline))
        # graphs=False: eager launches of the active games only (the graph-replay A/B)
        self.graphs = bool(graphs)
        self.device = learner.policy.model.device
        self._gf = {}
        self._pinned = {}
        self.stats = {"plies": 0, "positions": 0, "host_s": 0.0, "gpu_wait_s": 0.0}

    @staticmethod
    def supported(learner, opponent):
        """Both players are policy players over fused-HIP CUDA models of one board size, with
        no per-move host rules the batch cannot apply (pass_when_offered)."""
        for p in (learner, opponent):
            kind = _player_kind(p)
            if kind is None or getattr(p, "pass_when_offered", False):
                return False
            if not getattr(p, "device_select", True):
                return False
            model = getattr(p.policy, "model", None)
            if model is None or getattr(model, "device", None) is None or \
                    model.device.type != "cuda" or model._plan_for() is None:
                return False
        from ..ops.features import GpuFeatures
        S = learner.policy.model.input_shape[-1]
        return S == opponent.policy.model.input_shape[-1] and GpuFeatures.supports(S)

    # ------------------------------------------------------------------ buffers
    def _features(self, policy):
        key = id(policy)
        gf = self._gf.get(key)
        if gf is None:
            from ..ops.features import GpuFeatures
            # host ladder reads (the pack): RAG_LADDERS=gpu faulted the GPU once in 19x19
            # self-play (256 games to the 500-move limit; open item in docs/KERNELS.md), so the
            # self-play engine does not take the GPU ladder kernel
            gf = self._gf[key] = GpuFeatures(policy.preprocessor.feature_list, self.device,
                                             self.nthreads, ladders="host")
        return gf

    # ------------------------------------------------------------------ one ply
    def _launch(self, batch, player, idx, S, slot=0, limit=None, group=None):
        """Queue one ply of games ``idx`` (pack -> copies in -> features -> policy -> sampling
        -> chosen points copied back into pinned memory) without waiting for the GPU.

        ``group`` (the fixed game list of a pipeline group, idx a subset of it): every game of
        the group is packed and evaluated, so the GPU pass has one shape per (group, player) and
        replays as a captured HIP graph after its first eager run -- one host call instead of ~25
        Python kernel launches (the launch sequence was the self-play's host bound,
        profiles/selfplay_host_r3.txt). Finished games ride along; their moves are ignored.
        graphs=False: eager launches of the active games only."""
        import time
        t0 = time.perf_counter()
        if group is None or not self.graphs:
            group = None
            packed = idx
            pos = np.arange(len(idx))
        else:
            packed = group
            pos = np.searchsorted(group, idx)
        n = len(packed)
        P = S * S
        policy = player.policy
        gf = self._features(policy)
        host_lad = gf.ladders and gf.ladder_device == "host"
        b = self._slot(slot, n, S, gf, host_lad, persistent=group is not None)
        t1 = time.perf_counter()
        batch.pack(packed, b["hv"]["colors"], b["hv"]["ages"], b["hv"]["meta4"],
                   b["hv"].get("ladders"))
        t2 = time.perf_counter()
        self.stats["pack_s"] = self.stats.get("pack_s", 0.0) + t2 - t1
        kind = _player_kind(player)
        beta = float(getattr(player, "beta", 1.0))
        gs = getattr(player, "greedy_start", None)
        g = b["hv"]["greedy"]
        if kind == "greedy":
            g[:] = 1
        elif gs is not None:
            g[:] = [batch.board(int(i)).move_count >= gs for i in packed]
        else:
            g[:] = 0
        rng = getattr(player, "rng", np.random)
        seed = (int(rng.randint(0, 2 ** 31 - 1)) << 31) | int(rng.randint(0, 2 ** 31 - 1))
        b["hv"]["seed"][0] = seed
        t3 = time.perf_counter()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        if group is None:
            self._gpu_pass(b, policy, gf, n, S, P, beta)
        else:
            self._replay(b, policy, gf, n, S, P, beta, slot)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.stats["launch_s"] = self.stats.get("launch_s", 0.0) + time.perf_counter() - t3
        if limit is None:
            limit = player.move_limit if player.move_limit is not None else -1
        self.stats["host_s"] += time.perf_counter() - t0
        return {"idx": idx, "pos": pos, "planes": b["planes"][:n], "moves": b["h"]["moves"][:n],
                "event": ev, "event0": ev0, "limit": limit, "player": player}

    def _slot(self, slot, n, S, gf, host_lad, persistent):
        """Pinned host staging and device buffers of one pipeline slot, for n games: fixed
        addresses (a captured graph reads and writes them)."""
        P = S * S
        key = (slot, n, S, host_lad, gf.F) if persistent else ("eager", slot)
        b = self._pinned.get(key)
        if b is not None and (persistent or b["n"] >= n):
            return b
        specs = {"colors": ((n, P), torch.int8), "ages": ((n, P), torch.int16),
                 "meta4": ((n, 4), torch.int32), "greedy": ((n,), torch.uint8),
                 "seed": ((1,), torch.int64)}
        if host_lad:
            specs["ladders"] = ((n, 2, P), torch.uint8)
        # every input field lives in ONE pinned buffer (16-byte aligned views) mirrored by one
        # device buffer: a ply's inputs go up in one copy instead of one per field (each small
        # copy held the stream ~5 us; 7.5 copies per ply were 4 % of the RL trace)
        offs, total = {}, 0
        for k, (shp, dt) in specs.items():
            offs[k] = total
            nbytes = int(np.prod(shp)) * torch.empty((), dtype=dt).element_size()
            total += (nbytes + 15) // 16 * 16
        hraw = torch.zeros((total,), dtype=torch.uint8, pin_memory=True)
        draw = torch.zeros((total,), dtype=torch.uint8, device=self.device)

        def view(raw, k):
            shp, dt = specs[k]
            nb = int(np.prod(shp)) * torch.empty((), dtype=dt).element_size()
            return raw[offs[k]:offs[k] + nb].view(dt).view(shp)

        h = {k: view(hraw, k) for k in specs}
        h["moves"] = torch.zeros((n,), dtype=torch.int32, pin_memory=True)
        d = {k: view(draw, k) for k in specs}
        b = {"n": n, "h": h, "d": d, "hv": {k: v.numpy() for k, v in h.items()},
             "hraw": hraw, "draw": draw,
             "planes": torch.empty((n, gf.F, S, S), dtype=torch.uint8, device=self.device),
             "sens": torch.empty((n, P), dtype=torch.uint8, device=self.device),
             "mv": torch.empty((n,), dtype=torch.int32, device=self.device), "graphs": {}}
        self._pinned[key] = b
        return b

    def _gpu_pass(self, b, policy, gf, n, S, P, beta):
        from ..ops import hipops as ops
        h, d = b["h"], b["d"]
        b["draw"].copy_(b["hraw"], non_blocking=True)
        planes = gf.run(d["colors"][:n], d["ages"][:n], d["meta4"][:n], None,
                        d["ladders"][:n] if "ladders" in d else None, n, S,
                        out=b["planes"][:n], sens_out=b["sens"][:n])
        plan = policy.model._plan_for()
        with torch.no_grad():
            probs = plan.forward(planes, clone=False) if plan is not None else \
                policy.forward_device(planes)
        sens = b["sens"][:n]
        if probs.shape[1] == P + 1:  # pass-logit network: pass is always a candidate
            sens = torch.cat([sens, torch.ones((n, 1), dtype=torch.uint8, device=self.device)],
                             1)
        mv = ops.sample_moves(probs, sens, beta, d["greedy"][:n], 0, out=b["mv"][:n],
                              seed_dev=d["seed"])
        h["moves"][:n].copy_(mv, non_blocking=True)

    def _replay(self, b, policy, gf, n, S, P, beta, slot):
        """The slot's GPU pass as a captured HIP graph (captured after one eager run of this
        shape; recaptured when the plan's buffers moved)."""
        plan = policy.model._plan_for()
        if plan is None:
            return self._gpu_pass(b, policy, gf, n, S, P, beta)
        gens = tuple(getattr(o, "gen", 0) for o in (plan.trunk, plan.head))
        key = (id(policy), beta)
        ent = b["graphs"].get(key)
        if ent is None or ent[1] != gens:
            if ent is None and key not in b.setdefault("seen", set()):
                b["seen"].add(key)
                return self._gpu_pass(b, policy, gf, n, S, P, beta)  # warm-up, eager
            graph = torch.cuda.CUDAGraph()
            side = self.__dict__.get("_cap_stream")
            if side is None:
                side = self._cap_stream = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
                    self._gpu_pass(b, policy, gf, n, S, P, beta)
            torch.cuda.current_stream().wait_stream(side)
            ent = b["graphs"][key] = (graph, gens)
        plan.sync_weights()  # the graph reads the packed bf16 weights at fixed addresses
        ent[0].replay()

    def _finish(self, batch, job, S):
        """Wait for a queued ply and apply it natively; returns (planes, played, pos): the
        planes rows of the ply's games are ``planes[pos]`` (valid until the slot's next
        launch)."""
        import time
        t0 = time.perf_counter()
        job["event"].synchronize()
        t1 = time.perf_counter()
        # GPU time of the pass (ev0 fires once the stream reaches it, i.e. after the other
        # group's pass): summed against the self-play wall time it says whether the pipelined
        # loop keeps the GPU busy, which the host share alone cannot
        self.stats["gpu_pass_s"] = self.stats.get("gpu_pass_s", 0.0) + \
            job["event0"].elapsed_time(job["event"]) * 1e-3
        mv = job["moves"].numpy()[job["pos"]].astype(np.int32)
        mv[(mv < 0) | (mv >= S * S)] = -1
        t2 = time.perf_counter()
        _, played = batch.play(job["idx"], mv, job["limit"])
        self.stats["play_s"] = self.stats.get("play_s", 0.0) + time.perf_counter() - t2
        self.stats["plies"] += 1
        self.stats["positions"] += len(job["idx"])
        self.stats["gpu_wait_s"] += t1 - t0
        self.stats["host_s"] += time.perf_counter() - t1
        return job["planes"], played, job["pos"]

    def _ply(self, batch, player, idx, S, limit=None):
        return self._finish(batch, self._launch(batch, player, idx, S, limit=limit), S)[:2]

    def _groups(self, num_games):
        """Games split into independent groups whose plies alternate on the GPU: while one
        group's ply runs, the host applies the previous ply of the other and packs its next."""
        # small batches (the 7x7 reference shape) are bound by per-ply overhead: one group
        k = self.pipeline if num_games >= 64 * self.pipeline else 1
        grp = np.zeros(num_games, np.int64)
        for g, part in enumerate(np.array_split(np.arange(num_games), k)):
            grp[part] = g
        return k, grp

    @staticmethod
    def _active(batch, grp, k):
        a = batch.active()
        return a[grp[a] == k]

    # ------------------------------------------------------------------ games
    def play(self, num_games, size, komi=7.5):
        """Play ``num_games`` games (learner is BLACK in even games, WHITE in odd ones, as the
        reference). Returns (per game: the learner's device plane rows [n_g, F, S, S] in move
        order, or [] if it never moved; per game: its flat moves; learner colours; winners int8
        [num_games]). The rows are gathered once at the end (one index per ply, one sort by
        game), not as per-position tensor views."""
        import time
        t_start = time.perf_counter()
        zw, zb, _ = go._zobrist(size)
        batch = _rg.GameBatch(num_games, size, komi, False, zw.ravel().copy(),
                              zb.ravel().copy(), self.nthreads)
        colors = [go.BLACK if i % 2 == 0 else go.WHITE for i in range(num_games)]
        odd = np.arange(1, num_games, 2, dtype=np.int32)
        if len(odd):
            self._ply(batch, self.opponent, odd, size)
        K, grp = self._groups(num_games)
        groups = [np.nonzero(grp == k)[0].astype(np.int32) for k in range(K)]
        current = [self.learner] * K
        jobs = [None] * K
        recs = []  # (a learner ply's slot planes, played rows in them, their games, moves)

        def start(k):
            idx = self._active(batch, grp, k)
            return self._launch(batch, current[k], idx, size, slot=k,
                                group=groups[k]) if len(idx) else None
        for k in range(K):
            jobs[k] = start(k)
        while any(j is not None for j in jobs):
            for k in range(K):
                if jobs[k] is None:
                    continue
                idx = jobs[k]["idx"]
                planes, played, pos = self._finish(batch, jobs[k], size)
                if current[k] is self.learner:
                    t_r = time.perf_counter()
                    r = np.nonzero(played >= 0)[0]
                    if len(r):
                        # the slot's planes buffer is refilled by its next ply: copy it out now,
                        # whole (a device-side clone queued behind the pass; selecting the played
                        # rows here needed a host->device index copy, which synchronised the
                        # stream -- i.e. waited for the OTHER group's just-launched pass every
                        # learner ply); the rows are selected once, in _per_game
                        recs.append((planes.clone(), pos[r], idx[r], played[r]))
                    self.stats["rec_s"] = self.stats.get("rec_s", 0.0) + time.perf_counter() - t_r
                current[k] = self.opponent if current[k] is self.learner else self.learner
                jobs[k] = start(k)
        self.illegal = batch.illegal
        t_g = time.perf_counter()
        feats, moves = self._per_game(recs, num_games)
        self.stats["gather_s"] = self.stats.get("gather_s", 0.0) + time.perf_counter() - t_g
        self.stats["wall_s"] = self.stats.get("wall_s", 0.0) + time.perf_counter() - t_start
        return feats, moves, colors, batch.winners()

    def _per_game(self, recs, num_games):
        if not recs:
            return [[] for _ in range(num_games)], [[] for _ in range(num_games)]
        dev = self.device
        # recs: (a ply's whole slot planes [n, F, S, S], the played games' rows in it, their
        # game ids, their moves); one concatenation, one host->device row index, one gather
        base = np.cumsum([0] + [pl.shape[0] for pl, _, _, _ in recs])[:-1]
        sel = np.concatenate([b + p for b, (_, p, _, _) in zip(base, recs)]).astype(np.int64)
        gid = np.concatenate([g for _, _, g, _ in recs]).astype(np.int64)
        mv = np.concatenate([m for _, _, _, m in recs]).astype(np.int64)
        order = np.argsort(gid, kind="stable")  # plies were recorded in move order
        counts = np.bincount(gid, minlength=num_games)
        allrows = torch.cat([pl for pl, _, _, _ in recs])
        rows = allrows.index_select(0, torch.from_numpy(sel[order]).to(dev))
        del allrows
        parts = torch.split(rows, counts.tolist())
        mparts = np.split(mv[order], np.cumsum(counts)[:-1])
        feats = [p if c else [] for p, c in zip(parts, counts)]
        return feats, [m.tolist() for m in mparts]

    def sample_positions(self, num_games, size, targets, move_limit, komi=7.5):
        """Value-dataset self-play (``learner`` plays both colours): returns each game's native
        board copied when it reached ``targets[g]`` moves (or its final board if it ended
        earlier) and the winners int8 [num_games]. A game that reaches ``move_limit`` moves
        passes out (the winner is that of the limit position, as the Python loop that stops
        there)."""
        import time
        t_start = time.perf_counter()
        zw, zb, _ = go._zobrist(size)
        batch = _rg.GameBatch(num_games, size, komi, False, zw.ravel().copy(),
                              zb.ravel().copy(), self.nthreads)
        targets = np.asarray(targets, np.int64)
        counts = np.zeros(num_games, np.int64)
        snaps = [None] * num_games
        pending = np.ones(num_games, bool)
        own = self.learner.move_limit
        # play() passes once move_count > limit: no real move at move_limit moves or later
        limit = move_limit - 1 if own is None else min(move_limit - 1, own)
        K, grp = self._groups(num_games)
        groups = [np.nonzero(grp == k)[0].astype(np.int32) for k in range(K)]
        jobs = [None] * K

        def start(k):
            idx = self._active(batch, grp, k)
            if not len(idx):
                return None
            due = idx[pending[idx] & (counts[idx] >= targets[idx])]
            for g in due:
                snaps[int(g)] = batch.board(int(g)).copy()
            pending[due] = False
            return self._launch(batch, self.learner, idx, size, slot=k, limit=limit,
                                group=groups[k])
        for k in range(K):
            jobs[k] = start(k)
        while any(j is not None for j in jobs):
            for k in range(K):
                if jobs[k] is None:
                    continue
                idx = jobs[k]["idx"]
                self._finish(batch, jobs[k], size)
                counts[idx] += 1
                jobs[k] = start(k)
        for g in np.nonzero(pending)[0]:
            snaps[int(g)] = batch.board(int(g)).copy()
        self.illegal = batch.illegal
        self.stats["wall_s"] = self.stats.get("wall_s", 0.0) + time.perf_counter() - t_start
        return snaps, batch.winners()
