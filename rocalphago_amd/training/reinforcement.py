"""RL policy training (REINFORCE vs an opponent pool) — reference
AlphaGo/training/reinforcement_policy_trainer.py.

Same CLI and output contract (``weights.00000.hdf5`` copy of the initial weights, one
``weights.%05d.hdf5`` per iteration, ``metadata.json`` with opponents / win_ratio / cmd_line_args
written with sort_keys + indent 2; ``--resume``).

Self-play: all unfinished games advance in lock-step; each ply is ONE batched policy evaluation
for every game in which that player is to move. On a GPU the games live in a native
``GameBatch`` and a ply is one native pack + one GPU pass (features, policy, sampling) + one
native move application for all games (training/selfplay.py); otherwise GameState objects and
the players' ``get_moves``.

Update semantics (quirk Q7, the reference's *intended* behaviour): every game contributes the
gradient of its mean REINFORCE log-loss over the learner's positions with learning-rate sign +1
for a win, -1 for a loss. ``per_game`` mode (default, single process) applies one SGD step per
game exactly like the reference loop; ``batched`` mode (default under data parallelism) sums the
signed per-game gradients of all games on all ranks (one fwd/bwd with per-sample weights
sign/len(game), RCCL all-reduce) and applies one step — identical to first order.
"""
import json
import os
from shutil import copyfile

import numpy as np
import torch

from ..engine import gamestate as go
from ..models import kerasish as K
from ..models.policy import CNNPolicy
from ..parallel.dp import DPContext
from ..players.ai import ProbabilisticPolicyPlayer
from ..utils.go_util import flatten_idx


# games kept native (training/selfplay.py) whenever both players support it; False: the
# Python lock-step loop (benchmarks/rl_bench.py --selfplay python)
NATIVE_SELFPLAY = True
# pipelined game groups of the native self-play (training/selfplay.py NativeSelfPlay)
SELFPLAY_PIPELINE = 2

def _make_training_pair(st, mv, preprocessor):
    st_tensor = preprocessor.state_to_tensor(st)
    mv_tensor = np.zeros((1, st.size * st.size))
    mv_tensor[(0, flatten_idx(mv, st.size))] = 1
    return (st_tensor, mv_tensor)


def log_loss(y_true, y_pred):
    """REINFORCE objective: -y * log(clip(p)) (Keras then averages over classes and batch)."""
    return -y_true * torch.log(torch.clamp(y_pred, K.EPSILON, 1.0 - K.EPSILON))


log_loss._rag_head_mode = 2  # fused HIP head: REINFORCE mode


def _play_games(learner, opponent, states, num_games):
    """Lock-step self-play; returns per-game (features list, labels list), learner colors."""
    preprocessor = learner.policy.preprocessor
    state_feats = [[] for _ in range(num_games)]
    state_moves = [[] for _ in range(num_games)]
    learner_color = [go.BLACK if i % 2 == 0 else go.WHITE for i in range(num_games)]
    odd_states = states[1::2]
    if odd_states:
        moves = opponent.get_moves(odd_states)
        for st, mv in zip(odd_states, moves):
            st.do_move(mv)
    current, other = learner, opponent
    unfinished = {i: states[i] for i in range(num_games)}
    while len(unfinished) > 0:
        idxs = list(unfinished.keys())
        sts = [unfinished[i] for i in idxs]
        moves = current.get_moves(sts)
        learnable = [k for k, mv in enumerate(moves)
                     if current is learner and mv is not go.PASS_MOVE]
        if learnable:
            planes = getattr(current, "last_planes", None)
            if planes is not None and planes.shape[0] == len(sts):
                # the GPU player's own feature planes, gathered on the device (no second,
                # host-side extraction of the same positions)
                feats = planes[torch.tensor(learnable, device=planes.device)]
            else:
                feats = preprocessor.states_to_tensor_u8([sts[k] for k in learnable])
            for j, k in enumerate(learnable):
                state_feats[idxs[k]].append(feats[j])
                state_moves[idxs[k]].append(flatten_idx(moves[k], sts[k].size))
        just_finished = []
        for idx, state, mv in zip(idxs, sts, moves):
            state.do_move(mv)
            if state.is_end_of_game:
                just_finished.append(idx)
        for idx in just_finished:
            del unfinished[idx]
        current, other = other, current
    return state_feats, state_moves, learner_color


def _stack(rows):
    """Position rows -> one batch: device rows (the GPU player's planes) stay on the device.
    A game's rows may already be one [n, F, S, S] block (native self-play)."""
    if isinstance(rows, torch.Tensor):
        return rows
    if isinstance(rows[0], torch.Tensor):
        return torch.stack(rows)
    return torch.from_numpy(np.stack(rows))


def run_n_games(optimizer, learner, opponent, num_games, mock_states=[], mode="per_game",
                dp=None):
    """Play ``num_games`` learner-vs-opponent games, learn from the learner's moves, return the
    learner's win ratio (reference reinforcement_policy_trainer.py:21-86)."""
    if mode == "per_game" and dp is not None and dp.enabled:
        # per-game updates would need one all-reduce per non-empty game, and ranks have
        # different numbers of them: the collectives cannot pair up
        raise ValueError("mode='per_game' cannot run data-parallel (WORLD_SIZE > 1); use "
                         "mode='batched' (one all-reduced REINFORCE update per game batch)")
    board_size = learner.policy.model.input_shape[-1]
    model = learner.policy.model
    from .selfplay import NativeSelfPlay
    if not mock_states and NATIVE_SELFPLAY and NativeSelfPlay.supported(learner, opponent):
        # games kept native, one GPU pass + one native call per ply (training/selfplay.py)
        sp = NativeSelfPlay(learner, opponent, pipeline=SELFPLAY_PIPELINE)
        feats, moves, learner_color, winners = sp.play(num_games, board_size)
        won = [int(w) == c for w, c in zip(winners, learner_color)]
        run_n_games.last_stats = sp.stats
    else:
        states = [go.GameState(size=board_size) for _ in range(num_games)]
        if mock_states:
            states = mock_states
        feats, moves, learner_color = _play_games(learner, opponent, states, num_games)
        won = [st.get_winner() == c for st, c in zip(states, learner_color)]
    S2 = board_size * board_size
    if mode == "per_game":
        for f, m, w in zip(feats, moves, won):
            if len(f) == 0:
                continue
            optimizer.lr = abs(optimizer.lr) * (+1 if w else -1)
            X = _stack(f)
            Y = np.zeros((len(m), S2), np.float32)
            Y[np.arange(len(m)), m] = 1
            model.train_on_batch(X, Y)
    else:
        _batched_update(model, optimizer, feats, moves, won, S2, dp)
    wins = sum(won)
    return float(wins) / num_games


_UPDATE_CHUNK = 8192  # positions per fused fwd/bwd of the batched REINFORCE update


def _batched_update(model, optimizer, feats, moves, won, S2, dp):
    """One SGD step on sum_g sign_g * grad(mean log-loss of game g), summed across ranks."""
    X, lab, sw = [], [], []
    for f, m, w in zip(feats, moves, won):
        if len(f) == 0:
            continue
        X.append(_stack(f))
        lab.extend(m)
        sw.extend([(1.0 if w else -1.0) / len(f)] * len(f))
    dev = model.device
    net = model.net
    if X:
        x = torch.cat([t.to(dev) for t in X])
        labels = torch.tensor(lab, dtype=torch.int64, device=dev)
        w = torch.tensor(sw, dtype=torch.float32, device=dev)
        plan = model._plan_for()
        if plan is not None:
            # the summed signed loss splits over micro-batches: a large game batch (hundreds
            # of games x hundreds of moves) runs as chunks whose gradients are added up, which
            # bounds the activation memory and keeps the kernels' 32-bit offsets in range
            n = x.shape[0]
            acc = None
            for s in range(0, n, _UPDATE_CHUNK):
                B = plan.prepare(x[s:s + _UPDATE_CHUNK])
                plan.fwd_bwd(B, labels[s:s + _UPDATE_CHUNK], w[s:s + _UPDATE_CHUNK], 2, 1.0)
                if n > _UPDATE_CHUNK:
                    acc = net.flat_grad.clone() if acc is None else acc.add_(net.flat_grad)
            if acc is not None:
                net.flat_grad.copy_(acc)
        else:
            y = torch.zeros((len(lab), S2), device=dev)
            y[torch.arange(len(lab)), labels] = 1
            params = [v.detach().requires_grad_() for v in net._views]
            out = net.forward(x.float(), training=True, params=params)
            loss = (log_loss(y, out).mean(-1) * w).sum()
            grads = torch.autograd.grad(loss, params, allow_unused=True)
            with torch.no_grad():
                for gv, g in zip(net._gviews, grads):
                    gv.copy_(g if g is not None else torch.zeros_like(gv))
    else:
        net.flat_grad.zero_()
    if dp is not None and dp.enabled:
        dp.allreduce_sum_(net.flat_grad)
    optimizer.lr = abs(optimizer.lr)
    optimizer.apply(net)


def run_training(cmd_line_args=None):
    import argparse
    parser = argparse.ArgumentParser(description='Perform reinforcement learning to improve given policy network. Second phase of pipeline.')  # noqa: E501
    parser.add_argument("model_json", help="Path to policy model JSON.")
    parser.add_argument("initial_weights", help="Path to HDF5 file with inital weights (i.e. result of supervised training).")  # noqa: E501
    parser.add_argument("out_directory", help="Path to folder where the model params and metadata will be saved after each epoch.")  # noqa: E501
    parser.add_argument("--learning-rate", help="Keras learning rate (Default: 0.001)", type=float, default=0.001)  # noqa: E501
    parser.add_argument("--policy-temp", help="Distribution temperature of players using policies (Default: 0.67)", type=float, default=0.67)  # noqa: E501
    parser.add_argument("--save-every", help="Save policy as a new opponent every n batches (Default: 500)", type=int, default=500)  # noqa: E501
    parser.add_argument("--game-batch", help="Number of games per mini-batch (per rank) (Default: 20)", type=int, default=20)  # noqa: E501
    parser.add_argument("--move-limit", help="Maximum number of moves per game", type=int, default=500)  # noqa: E501
    parser.add_argument("--iterations", help="Number of training batches/iterations (Default: 10000)", type=int, default=10000)  # noqa: E501
    parser.add_argument("--resume", help="Load latest weights in out_directory and resume", default=False, action="store_true")  # noqa: E501
    parser.add_argument("--update", help="per_game (reference) or batched (default with >1 rank)", choices=["per_game", "batched"], default=None)  # noqa: E501
    parser.add_argument("--verbose", "-v", help="Turn on verbose mode", default=False, action="store_true")  # noqa: E501
    parser.add_argument("--dtype", help="GPU compute precision: bf16 (fused HIP kernels) or fp32 (reference precision, generic executor). Default: bf16", choices=["bf16", "fp32"], default="bf16")  # noqa: E501
    if cmd_line_args is None:
        args = parser.parse_args()
    else:
        args = parser.parse_args(cmd_line_args)

    dp = DPContext()
    mode = args.update or ("batched" if dp.enabled else "per_game")
    if mode == "per_game" and dp.enabled:
        raise SystemExit("--update per_game is single-process only (replicas would diverge "
                         "without a gradient all-reduce); use --update batched with WORLD_SIZE > 1")
    ZEROTH_FILE = "weights.00000.hdf5"

    if args.resume:
        if not os.path.exists(os.path.join(args.out_directory, "metadata.json")):
            raise ValueError("Cannot resume without existing output directory")
    if dp.is_root and not os.path.exists(args.out_directory):
        if args.verbose:
            print("creating output directory {}".format(args.out_directory))
        os.makedirs(args.out_directory)
    dp.barrier()

    if not args.resume:
        if dp.is_root:
            copyfile(args.initial_weights, os.path.join(args.out_directory, ZEROTH_FILE))
        if args.verbose and dp.is_root:
            print("copied {} to {}".format(args.initial_weights,
                                           os.path.join(args.out_directory, ZEROTH_FILE)))
        player_weights = ZEROTH_FILE
    else:
        args.initial_weights = os.path.join(args.out_directory,
                                            os.path.basename(args.initial_weights))
        if not os.path.exists(args.initial_weights):
            raise ValueError("Cannot resume; weights {} do not exist".format(args.initial_weights))
        elif args.verbose and dp.is_root:
            print("Resuming with weights {}".format(args.initial_weights))
        player_weights = os.path.basename(args.initial_weights)
    dp.barrier()

    policy = CNNPolicy.load_model(args.model_json, device=dp.device).set_dtype(args.dtype)
    policy.model.load_weights(args.initial_weights)
    dp.broadcast_model(policy.model)
    player = ProbabilisticPolicyPlayer(policy, temperature=args.policy_temp,
                                       move_limit=args.move_limit)
    opp_policy = CNNPolicy.load_model(args.model_json, device=dp.device).set_dtype(args.dtype)
    opponent = ProbabilisticPolicyPlayer(opp_policy, temperature=args.policy_temp,
                                         move_limit=args.move_limit)
    if args.verbose and dp.is_root:
        print("created player and opponent with temperature {}".format(args.policy_temp))

    if not args.resume:
        metadata = {
            "model_file": args.model_json,
            "init_weights": args.initial_weights,
            "learning_rate": args.learning_rate,
            "temperature": args.policy_temp,
            "game_batch": args.game_batch,
            "opponents": [ZEROTH_FILE],
            "win_ratio": {}
        }
    else:
        with open(os.path.join(args.out_directory, "metadata.json"), "r") as f:
            metadata = json.load(f)
    metadata["cmd_line_args"] = metadata.get("cmd_line_args", [])
    metadata["cmd_line_args"].append(vars(args))

    def save_metadata():
        if dp.is_root:
            with open(os.path.join(args.out_directory, "metadata.json"), "w") as f:
                json.dump(metadata, f, sort_keys=True, indent=2)

    optimizer = K.SGD(lr=args.learning_rate)
    player.policy.model.compile(loss=log_loss, optimizer=optimizer)
    rng = np.random.RandomState(1234)  # identical opponent choice on every rank
    start = 1
    if args.resume:
        start = int(player_weights.split(".")[1]) + 1
    for i_iter in range(start, start + args.iterations):
        opp_weights = metadata["opponents"][rng.randint(len(metadata["opponents"]))]
        opp_path = os.path.join(args.out_directory, opp_weights)
        opponent.policy.model.load_weights(opp_path)
        if args.verbose and dp.is_root:
            print("Batch {}\tsampled opponent is {}".format(i_iter, opp_weights))
        win_ratio = run_n_games(optimizer, player, opponent, args.game_batch, mode=mode, dp=dp)
        if dp.enabled:
            win_ratio = dp.allreduce_mean_(torch.tensor([float(win_ratio)], dtype=torch.float32,
                                                        device=dp.device)).item()
        metadata["win_ratio"][player_weights] = (opp_weights, win_ratio)
        player_weights = "weights.%05d.hdf5" % i_iter
        if dp.is_root:
            player.policy.model.save_weights(os.path.join(args.out_directory, player_weights))
        if i_iter % args.save_every == 0:
            metadata["opponents"].append(player_weights)
        save_metadata()
        dp.barrier()
    return metadata


if __name__ == '__main__':
    run_training()
