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

The learner's planes stay on the device for the REINFORCE update (rows of the positions where
it did not pass, the reference's ``_make_training_pair`` rows).
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

    def __init__(self, learner, opponent, nthreads=16):
        self.learner, self.opponent = learner, opponent
        self.nthreads = nthreads
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
            gf = self._gf[key] = GpuFeatures(policy.preprocessor.feature_list, self.device,
                                             self.nthreads)
        return gf

    def _buf(self, name, shape, dtype):
        t = self._pinned.get(name)
        if t is None or t.shape[0] < shape[0] or tuple(t.shape[1:]) != tuple(shape[1:]):
            t = torch.empty(shape, dtype=dtype, pin_memory=True)
            self._pinned[name] = t
        return t

    # ------------------------------------------------------------------ one ply
    def _ply(self, batch, player, idx, S):
        import time
        from ..ops import hipops as ops
        t0 = time.perf_counter()
        n = len(idx)
        P = S * S
        policy = player.policy
        gf = self._features(policy)
        host_lad = gf.ladders and gf.ladder_device == "host"
        h = {"colors": self._buf("colors", (n, P), torch.int8),
             "ages": self._buf("ages", (n, P), torch.int16),
             "meta4": self._buf("meta4", (n, 4), torch.int32)}
        if host_lad:
            h["ladders"] = self._buf("ladders", (n, 2, P), torch.uint8)
        hv = {k: v[:n].numpy() for k, v in h.items()}
        batch.pack(idx, hv["colors"], hv["ages"], hv["meta4"], hv.get("ladders"))
        d = {k: v[:n].to(self.device, non_blocking=True) for k, v in h.items()}
        sens = torch.empty((n, P), dtype=torch.uint8, device=self.device)
        planes = gf.run(d["colors"], d["ages"], d["meta4"], None, d.get("ladders"), n, S,
                        sens_out=sens)
        probs = policy.forward_device(planes)
        if probs.shape[1] == P + 1:  # pass-logit network: pass is always a candidate
            sens = torch.cat([sens, torch.ones((n, 1), dtype=torch.uint8, device=self.device)],
                             1)
        greedy = None
        kind = _player_kind(player)
        beta = getattr(player, "beta", 1.0)
        gs = getattr(player, "greedy_start", None)
        if kind == "greedy":
            greedy = torch.ones(n, dtype=torch.uint8, device=self.device)
        elif gs is not None:
            g = np.array([batch.board(int(i)).move_count >= gs for i in idx], np.uint8)
            if g.any():
                greedy = torch.from_numpy(g).to(self.device)
        rng = getattr(player, "rng", np.random)
        seed = (int(rng.randint(0, 2 ** 31 - 1)) << 31) | int(rng.randint(0, 2 ** 31 - 1))
        mv = ops.sample_moves(probs, sens, beta, greedy, seed)
        t1 = time.perf_counter()
        mv = mv.cpu().numpy().astype(np.int32)  # the only sync of the ply
        t2 = time.perf_counter()
        mv[(mv < 0) | (mv >= P)] = -1
        limit = player.move_limit if player.move_limit is not None else -1
        _, played = batch.play(idx, mv, limit)
        self.stats["plies"] += 1
        self.stats["positions"] += n
        self.stats["gpu_wait_s"] += t2 - t1
        self.stats["host_s"] += (t1 - t0) + (time.perf_counter() - t2)
        return planes, played

    # ------------------------------------------------------------------ games
    def play(self, num_games, size, komi=7.5):
        """Play ``num_games`` games (learner is BLACK in even games, WHITE in odd ones, as the
        reference). Returns (per-game list of device plane rows, per-game list of flat learner
        moves, learner colours, winners int8 [num_games])."""
        zw, zb, _ = go._zobrist(size)
        batch = _rg.GameBatch(num_games, size, komi, False, zw.ravel().copy(),
                              zb.ravel().copy(), self.nthreads)
        feats = [[] for _ in range(num_games)]
        moves = [[] for _ in range(num_games)]
        colors = [go.BLACK if i % 2 == 0 else go.WHITE for i in range(num_games)]
        odd = np.arange(1, num_games, 2, dtype=np.int32)
        if len(odd):
            self._ply(batch, self.opponent, odd, size)
        current = self.learner
        while True:
            idx = batch.active()
            if len(idx) == 0:
                break
            planes, played = self._ply(batch, current, idx, size)
            if current is self.learner:
                for r in np.nonzero(played >= 0)[0]:
                    g = int(idx[r])
                    feats[g].append(planes[int(r)])
                    moves[g].append(int(played[r]))
            current = self.opponent if current is self.learner else self.learner
        self.illegal = batch.illegal
        return feats, moves, colors, batch.winners()
