"""APV-MCTS: asynchronous policy-and-value Monte Carlo tree search.

The reference declares ``ParallelMCTS`` as an empty stub (AlphaGo/mcts.py:219-220); this is the
full search, built for a GPU evaluator:

  * the tree, PUCT selection with virtual loss, expansion, negamax backup and tree reuse are
    native C++ (csrc/mcts/search.cpp, ``_rocgo.Search``);
  * every *wave* selects ``batch`` leaves (virtual loss spreads them), extracts their input
    planes natively on a thread pool, and evaluates the policy and value networks for all of
    them in one batched pass on the GPU (hand-written HIP kernels via the fused plans);
  * while the GPU runs, the fast-rollout playouts of the same leaves run either on the native
    thread pool or — ``rollout_device="gpu"`` — as the gfx950 rollout kernel
    (csrc/hip/rollout.hip, one wavefront per game, ``rollouts_per_leaf`` games per leaf);
  * leaf value V = (1 - lmbda) * v_theta + lmbda * z (the AlphaGo mixing).

``ParallelMCTS(policy, value=None, ...)`` mirrors the reference MCTS interface
(``get_move(state)``, ``update_with_move(move)``); ``ParallelMCTSPlayer`` mirrors MCTSPlayer.
"""
import collections
import time

import numpy as np
import torch

from .._native import engine as _engine
from ..engine.gamestate import PASS_MOVE
from ..features.preprocessing import _FID

_rg = _engine()


class _nullctx(object):
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


class _Slots(object):
    """Round-robin pool of _Slot buffers for the pipelined search (at most ``depth`` waves in
    flight; a slot is handed out again only after its previous wave was backed up)."""

    def __init__(self, device, depth):
        self.device = device
        self.depth = max(1, int(depth))
        self.pool = []
        self.next = 0

    def take(self, n, S, F, PW, host_ladders, cap=0):
        if self.pool and (self.pool[0].B < n or self.pool[0].S != S or
                          self.pool[0].planes.shape[1] != F or
                          self.pool[0].o_pri.shape[1] != PW or
                          ("ladders" in self.pool[0].h) != host_ladders):
            # restart the rotation with the pool: once it refills, the slot handed out next is
            # pool[0], the oldest wave's (a stale odd ``next`` would return a slot still in flight)
            self.pool = []
            self.next = 0
        if len(self.pool) < self.depth:
            self.pool.append(_Slot(max(n, cap, 64), S, F, PW, self.device, host_ladders))
            return self.pool[-1]
        s = self.pool[self.next % len(self.pool)]
        self.next += 1
        return s


class _Ready(object):
    """An evaluation that finished synchronously."""

    def __init__(self, res):
        self.res = res

    def result(self):
        r = self.res
        return (r[0], r[1], r[2] if len(r) > 2 else None)


class _Pending(object):
    """A queued GPU evaluation: pinned host copies that are valid once ``event`` completes."""

    def __init__(self, event, priors, values, sens):
        self.event = event
        self.host = (priors, values, sens)

    def result(self):
        self.event.synchronize()
        return tuple(None if h is None else h.numpy() for h in self.host)


class _Slot(object):
    """Pinned host staging and device buffers of one in-flight wave (up to ``B`` leaves):
    the native search packs the leaves straight into the pinned inputs (Search.pack_inputs),
    the GPU pass copies them in, builds the planes, runs both networks and copies priors,
    values and sensible masks back into the pinned outputs. Reused round-robin: a slot is
    recycled only after its wave's backup read the outputs."""

    def __init__(self, B, S, F, PW, device, host_ladders):
        P = S * S

        def pin(shape, dt):
            return torch.empty(shape, dtype=dt, pin_memory=True)

        self.B, self.S, self.P = B, S, P
        # every input field is a view of ONE pinned buffer mirrored by one device buffer: a wave's
        # inputs go up in one copy instead of one per field (each copy is a blit launch of
        # ~5-9 us on the GPU; the self-play plies do the same, training/selfplay.py)
        specs = {"colors": ((B, P), torch.int8), "ages": ((B, P), torch.int16),
                 "meta4": ((B, 4), torch.int32)}
        if host_ladders:
            specs["ladders"] = ((B, 2, P), torch.uint8)
        offs, total = {}, 0
        for k, (shp, dt) in specs.items():
            offs[k] = total
            nbytes = int(np.prod(shp)) * torch.empty((), dtype=dt).element_size()
            total += (nbytes + 15) // 16 * 16
        self.hraw = pin((total,), torch.uint8)
        self.draw = torch.empty((total,), dtype=torch.uint8, device=device)

        def view(raw, k):
            shp, dt = specs[k]
            nb = int(np.prod(shp)) * torch.empty((), dtype=dt).element_size()
            return raw[offs[k]:offs[k] + nb].view(dt).view(shp)

        self.h = {k: view(self.hraw, k) for k in specs}
        self.d = {k: view(self.draw, k) for k in specs}
        self.n = {k: v.numpy() for k, v in self.h.items()}
        self.h_ill = self.d_ill = None
        self.planes = torch.empty((B, F, S, S), dtype=torch.uint8, device=device)
        self.o_pri = pin((B, PW), torch.float32)
        self.o_val = pin((B,), torch.float32)
        self.o_sens = pin((B, P), torch.uint8)
        self.event = torch.cuda.Event()

    def illegal(self, device):
        if self.h_ill is None:
            self.h_ill = torch.empty((self.B, self.P), dtype=torch.uint8, pin_memory=True)
            self.d_ill = torch.empty((self.B, self.P), dtype=torch.uint8, device=device)
        return self.h_ill.numpy()


class _SlotResult(object):
    """Handle of a wave evaluated into a slot: result() waits for the slot's event and returns
    numpy views of its pinned outputs (priors, values, sensible)."""

    def __init__(self, slot, n, has_pri, has_val, has_sens):
        self.slot, self.n = slot, n
        self.flags = (has_pri, has_val, has_sens)

    def result(self):
        s, n = self.slot, self.n
        s.event.synchronize()
        return (s.o_pri[:n].numpy() if self.flags[0] else None,
                s.o_val[:n].numpy() if self.flags[1] else None,
                s.o_sens[:n].numpy() if self.flags[2] else None)


class NetworkEvaluator(object):
    """Batched leaf evaluation: native boards -> (move priors [n, S*S], values [n])."""

    def __init__(self, policy=None, value=None, nthreads=8, two_streams=True, graph=False):
        self.policy = policy
        self.value = value
        # policy and value trunks of a wave on two streams (two_streams=False: one): 95.4k vs
        # 92.8k sims/s, profiles/mcts_eval_streams_r2.txt
        self.two_streams = bool(two_streams)
        # stream priority of the wave passes (torch: lower = higher priority; the search runs
        # them on a stream of this priority, above its GPU rollouts' streams)
        self.priority = 0
        # graph=True: a wave size seen before replays a captured HIP graph of its whole pass
        # (measured slower inside the search, 66.4k vs 70k sims/s: the search is GPU-bound and
        # the replay costs GPU time; kept for host-bound callers)
        self.graph = bool(graph)

        self.nthreads = nthreads
        self.pfids = policy.preprocessor.feature_ids if policy is not None else None
        self.vfids = value.preprocessor.feature_ids if value is not None else None

        # the value planes usually extend the policy planes (DEFAULT_FEATURES + color): then
        # one native extraction feeds both networks
        self.shared = (self.pfids is not None and self.vfids is not None and
                       list(self.vfids[:len(self.pfids)]) == list(self.pfids))
        if self.shared:
            self.npol = sum(_rg.feature_planes(f) for f in self.pfids)
        # on a GPU the planes are built by the HIP feature kernel (ops/features.py) and never
        # leave the device
        net = policy if policy is not None else value
        self.gpu = None
        if net is not None and net.model.net.device.type == "cuda":
            from ..ops.features import GpuFeatures
            dev = net.model.net.device
            if self.shared or value is None:
                self.gpu = {"p": GpuFeatures(value.preprocessor.feature_list if self.shared else
                                             policy.preprocessor.feature_list, dev, nthreads)}
            else:
                self.gpu = {"p": GpuFeatures(policy.preprocessor.feature_list, dev, nthreads)
                            if policy is not None else None,
                            "v": GpuFeatures(value.preprocessor.feature_list, dev, nthreads)}

    def _extract(self, fids, key, boards):
        if self.gpu is not None and self.gpu.get(key) is not None and \
                self.gpu[key].supports(boards[0].size):
            return self.gpu[key](boards)
        return _rg.batch_features(boards, fids, self.nthreads)

    def submit(self, boards):
        """Start the evaluation of a wave and return a handle whose ``result()`` gives
        ``(priors, values, sensible)`` as numpy arrays. On the GPU path everything after the
        native feature inputs is queued on the current stream and copied back into pinned host
        buffers asynchronously, so the caller can select the next wave while this one runs."""
        plans = self._plans()
        gf = None if self.gpu is None else (self.gpu.get("p") or self.gpu.get("v"))
        if plans is None or gf is None or not gf.supports(boards[0].size):
            return _Ready(self(boards))
        ppol, pval = plans
        n, S = len(boards), boards[0].size
        if self.shared or self.value is None:
            x = self.gpu["p"](boards, out=self._xbuf("p", n, S))
            xs = (x, None)
            planes = x
        else:
            xp = self.gpu["p"](boards, out=self._xbuf("p", n, S)) \
                if self.policy is not None else None
            xv = self.gpu["v"](boards, out=self._xbuf("v", n, S))
            xs = (xp, xv)
            planes = xp if xp is not None else xv
        with torch.no_grad():
            sens = planes[:, self._sens_off].reshape(n, -1) if self._sens_off is not None \
                else None
            pr, v = self._nets(n, xs, ppol, pval)
        host = []
        for t in (pr, v, sens):
            if t is None:
                host.append(None)
                continue
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            host.append(h)
        ev = torch.cuda.Event()
        ev.record()
        return _Pending(ev, *host)

    # ------------------------------------------------------------------ packed wave path
    def wave_capable(self, S):
        """True when submit_wave() can evaluate waves of board size S: fused HIP plans for every
        network, one shared GPU feature extractor (the value planes extend the policy planes, or
        a single network) and the sensibleness plane among the features."""
        plans = self._plans()
        return (plans is not None and self.gpu is not None and "v" not in self.gpu and
                self.gpu["p"].supports(S) and self._sens_off is not None)

    def submit_wave(self, search, wid, n, slots, cap=0):
        """Evaluate wave ``wid`` of the native search through a pinned slot (see _Slot): the
        leaves are packed natively into pinned memory (host ladder reads on the search pool),
        then copies in, feature kernel, both networks and copies out are queued on the current
        stream (a captured HIP graph for full waves with graph=True). Returns a handle whose
        result() gives numpy (priors, values, sensible)."""
        S = search.root_board.size
        gf = self.gpu["p"]
        superko = bool(search.root_board.enforce_superko)
        host_lad = gf.ladders and (gf.ladder_device == "host" or superko)
        slot = slots.take(n, S, gf.F, self._pw(S), host_lad, cap)
        nv = slot.n
        search.pack_inputs(wid, colors=nv["colors"], ages=nv["ages"], meta4=nv["meta4"],
                           ladders=nv.get("ladders") if host_lad else None,
                           illegal=slot.illegal(gf.device) if superko else None)
        if superko and not slot.n["meta4"][:n, 2].any():
            superko = False
        ppol, pval = self._plans()
        key = (n, S, superko, host_lad)
        if self.graph and n == slot.B and self._graph_ok(slot, key):
            for plan in (ppol, pval):
                if plan is not None:
                    plan.sync_weights()
            slot.graphs[key][0].replay()
        else:
            self._slot_pass(slot, n, S, superko, host_lad, ppol, pval)
        slot.event.record()
        return _SlotResult(slot, n, self.policy is not None, self.value is not None, True)

    def _pw(self, S):
        from ..models.policy import has_pass_logit
        return S * S + (1 if has_pass_logit(self.policy) else 0)

    def _slot_pass(self, slot, n, S, superko, host_lad, ppol, pval):
        gf = self.gpu["p"]
        d = slot.d
        with torch.no_grad():
            slot.draw.copy_(slot.hraw, non_blocking=True)  # all input fields, one copy
            il = None
            if superko:
                slot.d_ill[:n].copy_(slot.h_ill[:n], non_blocking=True)
                il = slot.d_ill[:n]
            x = slot.planes[:n]
            gf.run(d["colors"][:n], d["ages"][:n], d["meta4"][:n], il,
                   d["ladders"][:n] if host_lad else None, n, S, out=x)
            slot.o_sens[:n].copy_(x[:, self._sens_off].reshape(n, -1), non_blocking=True)
            # the policy packer reads its first planes of the shared input in place
            side = None
            if ppol is not None and pval is not None and self.two_streams:
                # the value trunk on its own stream fills the partial last block wave of each
                # policy conv and vice versa (separate plans, separate buffers)
                side = self.__dict__.get("_vstream")
                if side is None:
                    side = self._vstream = torch.cuda.Stream(x.device, priority=self.priority)
                side.wait_stream(torch.cuda.current_stream())
            if ppol is not None:
                pr = ppol.forward(x, clone=False)
                slot.o_pri[:n].copy_(pr, non_blocking=True)
            if pval is not None:
                with torch.cuda.stream(side) if side is not None else _nullctx():
                    v = pval.forward(x).reshape(-1)
                    slot.o_val[:n].copy_(v, non_blocking=True)
                if side is not None:
                    torch.cuda.current_stream().wait_stream(side)

    def _graph_ok(self, slot, key):
        """Capture the slot pass of this shape once (after one eager run warmed it up)."""
        graphs = slot.__dict__.setdefault("graphs", {})
        ppol, pval = self._plans()

        def gens():
            return tuple(getattr(o, "gen", 0) for p in (ppol, pval) if p is not None
                         for o in (p.trunk, p.head))

        ent = graphs.get(key)
        if ent is not None and ent[1] == gens():
            return True
        seen = slot.__dict__.setdefault("seen", set())
        if key not in seen:
            seen.add(key)
            return False  # eager first: allocations and weight packing happen outside capture
        n, S, superko, host_lad = key
        g = torch.cuda.CUDAGraph()
        side = self.__dict__.get("_cap_stream")
        if side is None:
            side = self._cap_stream = torch.cuda.Stream(slot.planes.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                self._slot_pass(slot, n, S, superko, host_lad, ppol, pval)
        torch.cuda.current_stream().wait_stream(side)
        graphs[key] = (g, gens())
        return True

    def _xbuf(self, key, n, S):
        """Persistent device input planes per (network, wave size, board size): a captured
        graph reads them at a fixed address."""
        bufs = self.__dict__.setdefault("_xbufs", {})
        t = bufs.get((key, n, S))
        if t is None:
            gf = self.gpu[key]
            t = torch.empty((n, gf.F, S, S), dtype=torch.uint8, device=gf.device)
            bufs[(key, n, S)] = t
        return t

    def _run_nets(self, xs, ppol, pval):
        if self.shared or self.value is None:
            x = xs[0]
            xp, xv = (x[:, :self.npol].contiguous() if self.shared else x), x
        else:
            xp, xv = xs
        if ppol is not None and pval is not None and self.two_streams:
            # the value trunk on its own stream: its blocks fill the partial last block wave of
            # each policy conv (a B = 512 trunk conv is 964 blocks on 512 slots) and vice versa.
            # The two plans own separate activations/workspaces, so they may run concurrently.
            main = torch.cuda.current_stream()
            side = self.__dict__.get("_vstream")
            if side is None:
                side = self._vstream = torch.cuda.Stream(xp.device, priority=self.priority)
            side.wait_stream(main)
            pr = ppol.forward(xp)
            with torch.cuda.stream(side):
                v = pval.forward(xv).reshape(-1)
            main.wait_stream(side)
            v.record_stream(main)
            return pr, v
        pr = ppol.forward(xp) if ppol is not None else None
        v = pval.forward(xv).reshape(-1) if pval is not None else None
        return pr, v

    def _nets(self, n, xs, ppol, pval):
        """Policy + value forward of one wave. A wave size seen before replays a captured HIP
        graph of the whole pass (input packing, both trunks, both heads): one host call instead
        of ~30 kernel launches through Python (0.37 -> 0.02 ms of host time per wave, measured).
        The packed bf16 weights are refreshed outside the graph when the fp32 masters changed.
        Measured slower inside the search (66.4k vs 70k sims/s: the search is GPU-bound there and
        the replay costs GPU time), so it is opt-in: graph=True."""
        if not self.graph:
            return self._run_nets(xs, ppol, pval)
        graphs = self.__dict__.setdefault("_graphs", {})
        key = (n, xs[0].shape[-1], id(ppol), id(pval))

        def gens():  # activation/workspace generations: a graph is valid only for its own
            return tuple(getattr(o, "gen", 0) for p in (ppol, pval) if p is not None
                         for o in (p.trunk, p.head))

        ent = graphs.get(key)
        if ent is not None and ent[2] != gens():
            # a larger eager wave reallocated the buffers this graph reads and writes
            del graphs[key]
            ent = None
        if ent is None:
            if len(graphs) >= 4 or n not in self.__dict__.setdefault("_seen_n", set()):
                self._seen_n.add(n)
                return self._run_nets(xs, ppol, pval)  # first sighting: eager (also warms up)
            g = torch.cuda.CUDAGraph()
            side = self.__dict__.get("_side")
            if side is None:
                side = self._side = torch.cuda.Stream(xs[0].device)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                self._run_nets(xs, ppol, pval)  # buffers sized before capture
                # thread-local capture: rollout launches of other threads (the multi-GPU search's
                # serving thread beside rank 0's master) may run while this thread captures
                with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                    out = self._run_nets(xs, ppol, pval)
            torch.cuda.current_stream().wait_stream(side)
            ent = graphs[key] = (g, out, gens())
        g, out, _ = ent
        for plan in (ppol, pval):
            if plan is not None:
                plan.sync_weights()
        g.replay()
        return out

    def _plans(self):
        """(policy plan, value plan) when every network present runs a fused HIP plan, else
        None (then submit() evaluates synchronously)."""
        if not hasattr(self, "_plan_cache"):
            pp = self.policy.model._plan_for() if self.policy is not None else None
            pv = self.value.model._plan_for() if self.value is not None else None
            ok = (self.policy is None or pp is not None) and (self.value is None or pv is not None)
            self._plan_cache = (pp, pv) if ok else None
            net = self.value if self.shared or self.policy is None else self.policy
            fl = net.preprocessor.feature_list if net is not None else []
            self._sens_off = None
            if "sensibleness" in fl:
                self._sens_off = sum(_rg.feature_planes(_FID[f])
                                     for f in fl[:fl.index("sensibleness")])
        return self._plan_cache

    def __call__(self, boards):
        n = len(boards)
        priors = values = None
        if n == 0:
            return priors, values
        if self.shared:
            x = self._extract(self.vfids, "p", boards)
            xp = x[:, :self.npol]
            xv = x
        else:
            xp = self._extract(self.pfids, "p", boards) if self.policy is not None else None
            xv = self._extract(self.vfids, "v", boards) if self.value is not None else None
        # the sensibleness plane doubles as the expansion move list (saves native move
        # generation in backup_value)
        sens = None
        planes = x if self.shared else (xp if xp is not None else xv)
        fl = (self.value if self.shared or self.policy is None else self.policy) \
            .preprocessor.feature_list
        if "sensibleness" in fl:
            off = 0
            for f in fl[:fl.index("sensibleness")]:
                off += _rg.feature_planes(_FID[f])
            sens = planes[:, off]
            sens = sens.reshape(n, -1).cpu().numpy() if not isinstance(sens, np.ndarray) \
                else np.ascontiguousarray(sens.reshape(n, -1))
        if self.policy is not None:
            if isinstance(xp, np.ndarray):
                xp = np.ascontiguousarray(xp)
            else:
                xp = xp.contiguous()
            priors = np.ascontiguousarray(self.policy.model.predict(xp), dtype=np.float32)
        if self.value is not None:
            values = np.ascontiguousarray(self.value.model.predict(xv),
                                          dtype=np.float32).reshape(-1)
        return priors, values, sens


class ParallelMCTS(object):
    """Wave-batched APV-MCTS over the native tree.

    policy: a CNNPolicy (priors); value: a CNNValue or None (then lmbda is forced to 1, i.e.
    rollouts only); rollout: a ``_rocgo.RolloutPolicy`` (default weights if None).
    """

    def __init__(self, policy=None, value=None, rollout=None, lmbda=0.5, c_puct=5.0,
                 n_playout=1600, batch=512, virtual_loss=3, rollout_limit=500,
                 playout_depth=722, nthreads=8, rollout_device="cpu", rollouts_per_leaf=1,
                 seed=1, evaluator=None, max_inflight=8, pipeline=3, dp=None,
                 rollout_group=8):
        # dp (parallel/dp.DPContext, world > 1): root parallelism over ranks — every rank
        # searches the same position with its own seed on its own GPU, and get_move() sums the
        # root visit counts over ranks (one all-reduce of S*S+1 counts), so all
        # ranks play the same move
        self.dp = dp if dp is not None and dp.enabled else None
        if self.dp is not None:
            seed = int(seed) + 7919 * self.dp.rank
        if value is None and lmbda < 1:
            lmbda = 1.0
        self.evaluator = evaluator or NetworkEvaluator(policy, value, nthreads)
        self.rollout = rollout or _rg.RolloutPolicy()
        self.lmbda = float(lmbda)
        self.c_puct = float(c_puct)
        self.n_playout = int(n_playout)
        self.batch = int(batch)
        self.virtual_loss = int(virtual_loss)
        self.rollout_limit = int(rollout_limit)
        self.playout_depth = int(playout_depth)
        self.nthreads = int(nthreads)
        self.rollout_device = rollout_device
        self.rollouts_per_leaf = int(rollouts_per_leaf)
        self.seed = int(seed)
        self._search = None
        self._history = None
        self._gpu_rollout = None
        self._inflight = []
        self.max_inflight = max_inflight
        # GPU rollouts of `rollout_group` consecutive waves go out as one launch
        # (gpu_rollout.RolloutBatcher); up to `max_inflight` waves' rollouts are in flight.
        # 8 / 8: a group's results come back when the next group's first wave is selected (at
        # most 8 waves, 4.5 on average, later); 6 / 8 returned them 3-8 waves later and left the
        # host waiting on a group launched 3 waves earlier: 128.5-130.3k against 137.1-138.9k
        # sims/s on one box (profiles/mcts_rollout_group_r6.txt)
        self.rollout_group = int(rollout_group)
        # leaves packed natively into pinned slots and evaluated in one GPU pass per wave when
        # the evaluator supports it (NetworkEvaluator.wave_capable); False: board objects
        self.packed_waves = True
        self.pipeline = int(pipeline)
        self.stats = {"waves": 0, "sims": 0}

    # ------------------------------------------------------------------ tree management
    def _configure(self, s):
        from ..models.policy import has_pass_logit
        s.pass_prior = has_pass_logit(getattr(self.evaluator, "policy", None))
        s.c_puct = self.c_puct
        s.lmbda = self.lmbda
        # CPU rollouts seeded by the leaf position instead of (seed, wave, index): every search
        # that reaches a position plays the same rollout from it (search/efficiency.py)
        s.keyed_rollouts = bool(getattr(self, "keyed_rollouts", False))
        s.n_vl = self.virtual_loss
        s.rollout_limit = self.rollout_limit
        s.max_depth = self.playout_depth
        s.seed = self.seed
        s.set_rollout_policy(self.rollout)

    def _sync_root(self, state):
        """Point the tree at ``state``: reuse the subtree when state extends the tree's root
        by at most a few moves, otherwise start a fresh tree."""
        hist = list(state.history)
        s = self._search
        if s is not None and self._history is not None and \
                hist[:len(self._history)] == self._history and \
                len(hist) - len(self._history) <= 4:
            ok = True
            for mv in hist[len(self._history):]:
                flat = -1 if mv is PASS_MOVE else mv[0] * state.size + mv[1]
                try:
                    s.advance(flat)
                except Exception:
                    ok = False
                    break
            if ok and s.root_board.hash == state.native.hash and \
                    s.root_board.current_player == state.current_player:
                self._history = hist
                return s
        s = _rg.Search(state.native, self.nthreads)
        self._configure(s)
        self._search = s
        self._history = hist
        return s

    # ------------------------------------------------------------------ search
    def _acc(self, key, dt):
        self.stats[key] = self.stats.get(key, 0.0) + dt

    def _wave(self, s, want):
        """One wave: select, (launch rollouts), evaluate, value backup. GPU rollouts stay in
        flight (up to ``max_inflight`` waves) and are backed up as they finish."""
        t0 = time.perf_counter()
        wid, n = s.select(want)
        if n == 0:
            return 0
        boards = s.leaf_boards(wid)
        t1 = time.perf_counter()
        pending = None
        if self.lmbda > 0:
            if self.rollout_device == "gpu":
                pending = self._gpu_rollouts(s, wid)
            else:
                s.start_rollouts(wid)  # native pool, overlapped with the network pass
        res = self.evaluator(boards)
        priors, values = res[0], res[1]
        sens = res[2] if len(res) > 2 else None
        t2 = time.perf_counter()
        s.backup_value(wid, priors, values, sens)
        t3 = time.perf_counter()
        if self.lmbda > 0:
            if pending is None:
                s.finish_rollouts(wid)
            else:
                self._inflight.append((wid, pending))
                self._harvest(s, self.max_inflight)
        t4 = time.perf_counter()
        self.stats["waves"] += 1
        self.stats["sims"] += n
        self._acc("t_select", t1 - t0)
        self._acc("t_eval", t2 - t1)
        self._acc("t_backup", t3 - t2)
        self._acc("t_rollout_wait", t4 - t3)
        return n

    def _harvest(self, s, keep):
        """Back up finished GPU rollout waves; block on the oldest while more than ``keep``
        are in flight."""
        while self._inflight:
            wid, pend = self._inflight[0]
            if len(self._inflight) <= keep and not pend.done():
                break
            s.backup_rollout(wid, pend.result())
            self._inflight.pop(0)

    def _gpu_rollouts(self, s, wid):
        if self._gpu_rollout is None:
            from .gpu_rollout import GpuRollouts, RolloutBatcher
            self._gpu_rollout = RolloutBatcher(GpuRollouts(self.rollout, torch.device("cuda")),
                                               self.rollout_group)
        return self._gpu_rollout.add(s, wid, self.rollouts_per_leaf, self.rollout_limit,
                                     seed=self.seed * 7919 + self.stats["waves"])

    def search(self, state, n_playout=None, tick=None):
        """Run ``n_playout`` simulations from ``state`` (tree reused when possible). ``tick(s)``,
        if given, runs after every wave's value backup."""
        s = self._sync_root(state)
        target = s.root_visits + (n_playout or self.n_playout)
        submit = getattr(self.evaluator, "submit", None)
        if self.pipeline > 1 and submit is not None:
            self._search_pipelined(s, target, submit, tick)
        else:
            stall = 0
            while s.root_visits < target:
                want = min(self.batch, target - s.root_visits)
                before = s.root_visits
                self._wave(s, want)
                if tick is not None:
                    tick(s)
                stall = stall + 1 if s.root_visits == before else 0
                if stall > 3:
                    break
        t = time.perf_counter()
        if self._gpu_rollout is not None:
            self._gpu_rollout.flush()
        self._harvest(s, 0)  # every rollout of this move backed up before choosing
        self._acc("t_rollout_wait", time.perf_counter() - t)
        return s

    def _search_pipelined(self, s, target, submit, tick=None):
        """Up to ``pipeline`` waves in flight: while the GPU evaluates wave k (features, policy
        and value nets, copies back to pinned memory) the host selects wave k+1 — virtual loss
        keeps the two apart — builds its feature inputs and launches its rollouts; then it
        backs up wave k. Host tree work and GPU network work overlap instead of alternating."""
        queue = collections.deque()
        queued = 0
        stall = 0
        # packed path: leaves go from the native tree straight into pinned slot buffers (no
        # Python board objects), one graph-capturable GPU pass per wave
        slots = None
        cap = getattr(self.evaluator, "wave_capable", None)
        if cap is not None and self.packed_waves and cap(s.root_board.size):
            slots = self.__dict__.get("_slots")
            if slots is None or slots.depth != self.pipeline:
                slots = self._slots = _Slots(self.evaluator.gpu["p"].device, self.pipeline)
        while True:
            t0 = time.perf_counter()
            if len(queue) < self.pipeline and s.root_visits + queued < target:
                want = min(self.batch, target - s.root_visits - queued)
                wid, n = s.select(want)
                if n > 0:
                    boards = None if slots is not None else s.leaf_boards(wid)
                    pending = None
                    if self.lmbda > 0:
                        if self.rollout_device == "gpu":
                            pending = self._gpu_rollouts(s, wid)
                        else:
                            s.start_rollouts(wid)
                    t1 = time.perf_counter()
                    if slots is not None:
                        with self._eval_stream():
                            handle = self.evaluator.submit_wave(s, wid, n, slots, self.batch)
                    else:
                        handle = submit(boards)
                    queue.append((wid, n, handle, pending))
                    queued += n
                    self._acc("t_select", t1 - t0)
                    self._acc("t_submit", time.perf_counter() - t1)
                    stall = 0
                    continue
                if not queue:
                    stall += 1
                    if stall > 3 or s.root_visits >= target:
                        break
                    continue
            if not queue:
                break
            wid, n, handle, pending = queue.popleft()
            queued -= n
            t1 = time.perf_counter()
            priors, values, sens = handle.result()
            t2 = time.perf_counter()
            s.backup_value(wid, priors, values, sens)
            t3 = time.perf_counter()
            if self.lmbda > 0:
                if pending is None:
                    s.finish_rollouts(wid)
                else:
                    self._inflight.append((wid, pending))
                    self._harvest(s, self.max_inflight)
            t4 = time.perf_counter()
            self.stats["waves"] += 1
            self.stats["sims"] += n
            self._acc("t_eval", t2 - t1)
            self._acc("t_backup", t3 - t2)
            self._acc("t_rollout_wait", t4 - t3)
            if tick is not None:
                tick(s)  # e.g. the distributed search's root-statistics exchange

    def _eval_stream(self):
        """Context of the wave passes: a high-priority stream when ``eval_priority`` is set (the
        hardware queue scheduler then prefers the networks' blocks over the rollouts')."""
        pr = getattr(self, "eval_priority", None)
        if pr is None or not torch.cuda.is_available():
            return _nullctx()
        st = self.__dict__.get("_hp_stream")
        if st is None:
            st = self._hp_stream = torch.cuda.Stream(priority=pr)
            st.wait_stream(torch.cuda.current_stream())
            self.evaluator.priority = pr
        return torch.cuda.stream(st)

    def get_move(self, state):
        s = self.search(state)
        a = s.best_move() if self.dp is None else self._merged_best(s, state.size)
        return PASS_MOVE if a < 0 else divmod(int(a), state.size)

    def _merged_best(self, s, size):
        """Most visited root move over all ranks (visit counts summed by all-reduce; ties go to
        the lowest point, pass last, identically on every rank)."""
        P = size * size
        mvs, vis, _, _ = s.root_stats()
        counts = np.zeros(P + 1, np.float64)  # slot P: pass
        for m, v in zip(mvs, vis):
            counts[P if m < 0 else m] += v
        t = torch.from_numpy(counts).to(self.dp.device)
        self.dp.allreduce_sum_(t)
        self.merged_visits = t.cpu().numpy()
        if self.merged_visits.max() <= 0:
            return s.best_move()
        best = int(np.argmax(self.merged_visits))
        return -1 if best == P else best

    def root_statistics(self):
        """(moves, visits, Q, prior) of the root children."""
        return self._search.root_stats()

    def update_with_move(self, last_move):
        s = self._search
        if s is None:
            return
        flat = -1 if last_move is PASS_MOVE else last_move[0] * s.root_board.size + last_move[1]
        try:
            s.advance(flat)
            self._history = (self._history or []) + [last_move]
        except Exception:
            self._search = None
            self._history = None


class ParallelMCTSPlayer(object):
    """Player wrapper (reference ai.py:136-149 MCTSPlayer shape) around ParallelMCTS."""

    def __init__(self, policy=None, value=None, rollout=None, lmbda=0.5, c_puct=5,
                 rollout_limit=500, playout_depth=722, n_playout=1600, **kw):
        self.mcts = ParallelMCTS(policy, value, rollout, lmbda, c_puct, n_playout,
                                 rollout_limit=rollout_limit, playout_depth=playout_depth, **kw)

    def get_move(self, state):
        sensible = state.get_legal_moves(include_eyes=False)
        if len(sensible) == 0:
            return PASS_MOVE
        move = self.mcts.get_move(state)
        self.mcts.update_with_move(move)
        return move
