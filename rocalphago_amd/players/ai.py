"""Policy players — reference AlphaGo/ai.py:1-149.

GreedyPolicyPlayer / ProbabilisticPolicyPlayer keep the reference behaviour (sensible moves only,
pass when none remain, when the move limit is exceeded, or when a pass is offered after move 100;
temperature applied in log space with beta = 1/T). ``get_moves`` evaluates all states in one
batched network call (features by native threads, forward on the HIP engine).

On a GPU, ``get_moves`` keeps the whole selection on the device (K12): feature planes and the
sensibleness mask from the feature kernel (features.hip), the forward on the fused HIP plan, and
one Gumbel-max sampling kernel over the masked, temperature-adjusted distribution (sample.hip) —
only the chosen points come back to the host. Same distribution as the host path (p^beta over the
sensible moves); the random stream differs, seeded from the player's ``rng``.

Fixed quirk Q6: ``move_limit=None`` means "no limit" in the batched path too.
"""
from operator import itemgetter

import numpy as np

from ..engine import gamestate as go
from ..search import mcts


def _over_limit(state, move_limit):
    return move_limit is not None and len(state.history) > move_limit


def _device_moves(policy, states, beta, greedy_rows, rng, player=None):
    """Batched move choice on the GPU, or None when the policy is not a HIP model (CPU model,
    duck-typed test policy, unsupported board size). The feature planes the choice was made on
    stay on the device as ``player.last_planes`` ([n, F, S, S] uint8; RL self-play learns from
    them instead of re-extracting the positions on the host)."""
    model = getattr(policy, "model", None)
    if model is None or not hasattr(policy, "forward_device") or \
            getattr(model, "device", None) is None or model.device.type != "cuda":
        return None
    import torch
    from ..ops import hipops as ops
    from ..ops.features import GpuFeatures
    S = states[0].size
    if any(st.size != S for st in states) or not GpuFeatures.supports(S):
        return None
    gf = getattr(policy, "_rag_gpu_features", None)
    if gf is None or gf.device != model.device:
        gf = GpuFeatures(policy.preprocessor.feature_list, model.device)
        policy._rag_gpu_features = gf
    n = len(states)
    sens = torch.empty((n, S * S), dtype=torch.uint8, device=model.device)
    x = gf([st.native for st in states], sens_out=sens)
    if player is not None:
        player.last_planes = x
    probs = policy.forward_device(x)
    if probs.shape[1] == S * S + 1:  # pass-logit network: pass is always a candidate
        sens = torch.cat([sens, torch.ones((n, 1), dtype=torch.uint8, device=model.device)], 1)
    greedy = None
    if any(greedy_rows):
        greedy = torch.tensor([1 if g else 0 for g in greedy_rows],
                              dtype=torch.uint8).to(model.device)
    seed = (int(rng.randint(0, 2 ** 31 - 1)) << 31) | int(rng.randint(0, 2 ** 31 - 1))
    mv = ops.sample_moves(probs, sens, beta, greedy, seed).cpu().numpy()
    return [go.PASS_MOVE if m < 0 or m >= S * S else (int(m) // S, int(m) % S) for m in mv]


class GreedyPolicyPlayer(object):
    """Plays the highest-probability sensible move."""

    device_select = True  # get_moves on the GPU when the policy is a HIP model

    def __init__(self, policy_function, pass_when_offered=False, move_limit=None):
        self.policy = policy_function
        self.pass_when_offered = pass_when_offered
        self.move_limit = move_limit

    def get_move(self, state):
        if _over_limit(state, self.move_limit):
            return go.PASS_MOVE
        if self.pass_when_offered:
            if len(state.history) > 100 and state.history[-1] == go.PASS_MOVE:
                return go.PASS_MOVE
        sensible_moves = state.get_legal_moves(include_eyes=False)
        if len(sensible_moves) > 0:
            move_probs = self.policy.eval_state(state, sensible_moves)
            return max(move_probs, key=itemgetter(1))[0]
        return go.PASS_MOVE

    def get_moves(self, states):
        if len(states) == 0:
            return []
        self.last_planes = None
        dev = _device_moves(self.policy, states, 1.0, [True] * len(states), np.random,
                            self) if self.device_select else None
        if dev is not None:
            return [go.PASS_MOVE if _over_limit(st, self.move_limit) else m
                    for st, m in zip(states, dev)]
        sensible = [st.get_legal_moves(include_eyes=False) for st in states]
        dists = self.policy.batch_eval_state(states, sensible)
        out = []
        for st, mp in zip(states, dists):
            if len(mp) == 0 or _over_limit(st, self.move_limit):
                out.append(go.PASS_MOVE)
            else:
                out.append(max(mp, key=itemgetter(1))[0])
        return out


class ProbabilisticPolicyPlayer(object):
    """Samples a sensible move from the (temperature-adjusted) policy distribution."""

    device_select = True

    def __init__(self, policy_function, temperature=1.0, pass_when_offered=False,
                 move_limit=None, greedy_start=None, rng=None):
        assert(temperature > 0.0)
        self.policy = policy_function
        self.move_limit = move_limit
        self.beta = 1.0 / temperature
        self.pass_when_offered = pass_when_offered
        self.greedy_start = greedy_start
        self.rng = rng or np.random

    def apply_temperature(self, distribution):
        log_probabilities = np.log(distribution)
        log_probabilities = log_probabilities * self.beta
        log_probabilities = log_probabilities - log_probabilities.max()
        probabilities = np.exp(log_probabilities)
        return probabilities / probabilities.sum()

    def _choose(self, state, move_probs):
        if self.greedy_start is not None and len(state.history) >= self.greedy_start:
            return max(move_probs, key=itemgetter(1))[0]
        moves, probabilities = zip(*move_probs)
        probabilities = self.apply_temperature(np.asarray(probabilities, dtype=np.float64))
        choice_idx = self.rng.choice(len(moves), p=probabilities)
        return moves[choice_idx]

    def get_move(self, state):
        if _over_limit(state, self.move_limit):
            return go.PASS_MOVE
        if self.pass_when_offered:
            if len(state.history) > 100 and state.history[-1] == go.PASS_MOVE:
                return go.PASS_MOVE
        sensible_moves = state.get_legal_moves(include_eyes=False)
        if len(sensible_moves) > 0:
            move_probs = self.policy.eval_state(state, sensible_moves)
            return self._choose(state, move_probs)
        return go.PASS_MOVE

    def get_moves(self, states):
        """Batched get_move: one network evaluation for all states."""
        if len(states) == 0:
            return []
        greedy = [self.greedy_start is not None and len(st.history) >= self.greedy_start
                  for st in states]
        self.last_planes = None
        dev = _device_moves(self.policy, states, self.beta, greedy, self.rng, self) \
            if self.device_select else None
        if dev is not None:
            return [go.PASS_MOVE if _over_limit(st, self.move_limit) else m
                    for st, m in zip(states, dev)]
        sensible_move_lists = [st.get_legal_moves(include_eyes=False) for st in states]
        all_moves_distributions = self.policy.batch_eval_state(states, sensible_move_lists)
        move_list = [None] * len(states)
        for i, move_probs in enumerate(all_moves_distributions):
            if len(move_probs) == 0 or _over_limit(states[i], self.move_limit):
                move_list[i] = go.PASS_MOVE
            else:
                move_list[i] = self._choose(states[i], move_probs)
        return move_list


class MCTSPlayer(object):
    """Search player (reference ai.py:136-149) over the reference-semantics MCTS."""

    def __init__(self, value_function, policy_function, rollout_function, lmbda=.5, c_puct=5,
                 rollout_limit=500, playout_depth=40, n_playout=100):
        self.mcts = mcts.MCTS(value_function, policy_function, rollout_function, lmbda, c_puct,
                              rollout_limit, playout_depth, n_playout)

    def get_move(self, state):
        sensible_moves = state.get_legal_moves(include_eyes=False)
        if len(sensible_moves) > 0:
            move = self.mcts.get_move(state)
            self.mcts.update_with_move(move)
            return move
        return go.PASS_MOVE
