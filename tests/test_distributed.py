"""Multi-process data parallelism on the CPU (gloo, world_size 2) — same code path as RCCL on GPU.

* SL training with DPContext: replicas stay identical and match single-process training on the
  concatenated global batch (mean of equal-sized local means == global mean).
* BucketedAllReduce: layer-triggered async bucket all-reduce == plain mean all-reduce.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

FEATS = ["board", "ones", "turns_since"]  # 12 planes


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)


def _make_model(lr=0.05):
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    policy = CNNPolicy(FEATS, board=9, filters_per_layer=8, layers=3, device="cpu", seed=7)
    policy.model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=lr),
                         metrics=["accuracy"])
    return policy.model


def _dataset():
    from rocalphago_amd.training.data import DeviceDataset
    return DeviceDataset.synthetic(64, 12, 9, torch.device("cpu"), seed=11)


def _sl_worker(rank, world, port, outdir, steps, local_b):
    _setup(rank, world, port)
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.training.supervised import SupervisedTrainer
    dp = DPContext(device="cpu")
    model = _make_model()
    if rank == 1:  # diverge on purpose: broadcast_model must restore rank 0's weights
        with torch.no_grad():
            model.net.flat.add_(1.0)
        model.net.bump()
    dp.broadcast_model(model)
    trainer = SupervisedTrainer(model, _dataset(), local_b, ["noop"], dp, seed=0)
    gb = local_b * world
    for s in range(steps):
        trainer.step(torch.arange(s * gb + rank * local_b, s * gb + (rank + 1) * local_b))
    loss, acc = trainer.pop_metrics()
    np.save(os.path.join(outdir, "flat%d.npy" % rank), model.net.flat.detach().numpy())
    np.save(os.path.join(outdir, "metrics%d.npy" % rank), np.array([loss, acc]))
    dp.shutdown()


def _bucket_worker(rank, world, port, outdir, comm_dtype="fp32"):
    _setup(rank, world, port)
    from rocalphago_amd.parallel.dp import BucketedAllReduce, DPContext
    dp = DPContext(device="cpu")
    n = 1000
    offsets = [0, 100, 250, 600, 900]
    g = torch.arange(n, dtype=torch.float32) * (rank + 1)
    br = BucketedAllReduce(dp, g, offsets, bucket_bytes=200 * 4, comm_dtype=comm_dtype)
    for layer in reversed(range(len(offsets))):
        br.layer_done(layer)
    br.finish()
    np.save(os.path.join(outdir, "bucket%d.npy" % rank), g.numpy())
    # second use of the same bucketer (reset state) with only finish()
    g.copy_(torch.ones(n) * (rank + 1))
    br.finish()
    np.save(os.path.join(outdir, "bucket_b%d.npy" % rank), g.numpy())
    dp.shutdown()


def _spawn(fn, args, world=2):
    mp.spawn(fn, args=(world, _port()) + args, nprocs=world, join=True)


@pytest.mark.timeout(300)
def test_dp_sl_training_matches_single_process(tmp_path):
    steps, local_b, world = 3, 8, 2
    _spawn(_sl_worker, (str(tmp_path), steps, local_b), world)
    f0 = np.load(tmp_path / "flat0.npy")
    f1 = np.load(tmp_path / "flat1.npy")
    assert np.array_equal(f0, f1), "replicas diverged"
    m0, m1 = np.load(tmp_path / "metrics0.npy"), np.load(tmp_path / "metrics1.npy")
    assert np.allclose(m0, m1)

    # single process on the global batch
    from rocalphago_amd.training.supervised import SupervisedTrainer
    torch.set_num_threads(1)
    model = _make_model()
    start = model.net.flat.detach().clone()
    trainer = SupervisedTrainer(model, _dataset(), local_b * world, ["noop"], None, seed=0)
    gb = local_b * world
    for s in range(steps):
        trainer.step(torch.arange(s * gb, (s + 1) * gb))
    ref = model.net.flat.detach().numpy()
    assert not np.allclose(ref, start.numpy()), "training did not move the weights"
    np.testing.assert_allclose(f0, ref, rtol=1e-4, atol=1e-6)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("comm_dtype", ["fp32", "bf16"])
def test_bucketed_allreduce_mean(tmp_path, comm_dtype):
    _spawn(_bucket_worker, (str(tmp_path), comm_dtype))
    n = 1000
    want = np.arange(n, dtype=np.float32) * 1.5  # mean of x1 and x2
    rtol = 1e-6 if comm_dtype == "fp32" else 2 ** -7  # bf16: 8-bit significand
    got = [np.load(tmp_path / ("bucket%d.npy" % r)) for r in range(2)]
    assert np.array_equal(got[0], got[1])  # replicas identical either way
    for r in range(2):
        np.testing.assert_allclose(got[r], want, rtol=rtol)
        np.testing.assert_allclose(np.load(tmp_path / ("bucket_b%d.npy" % r)),
                                   np.full(n, 1.5, np.float32))


class _UniformEval(object):
    """Evaluator stub for the search workers: uniform priors, no value."""

    def __call__(self, boards):
        n, P = len(boards), boards[0].size ** 2
        return np.full((n, P), 1.0 / P, np.float32), None


def _mcts_worker(rank, world, port, outdir):
    _setup(rank, world, port)
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.search.apv import ParallelMCTS
    dp = DPContext(device="cpu")
    mc = ParallelMCTS(evaluator=_UniformEval(), lmbda=1.0, n_playout=96, batch=16,
                      rollout_limit=60, nthreads=1, dp=dp)
    st = GameState(size=7)
    moves, local, merged = [], [], []
    for _ in range(3):
        mv = mc.get_move(st)
        mvs, vis, _, _ = mc.root_statistics()
        v = np.zeros(50)
        for m, n in zip(mvs, vis):
            v[49 if m < 0 else m] += n
        local.append(v)
        merged.append(mc.merged_visits.copy())
        moves.append(-1 if mv is None else mv[0] * 7 + mv[1])
        st.do_move(mv)
        mc.update_with_move(mv)
    np.save(os.path.join(outdir, "mv%d.npy" % rank), np.array(moves))
    np.save(os.path.join(outdir, "loc%d.npy" % rank), np.array(local))
    np.save(os.path.join(outdir, "mrg%d.npy" % rank), np.array(merged))
    dp.shutdown()


@pytest.mark.timeout(300)
def test_root_parallel_mcts(tmp_path):
    """Root parallelism: each rank searches its own tree (own rollout seeds), the root visit
    counts are all-reduced and every rank plays the same most-visited move."""
    _spawn(_mcts_worker, (str(tmp_path),))
    m0, m1 = np.load(tmp_path / "mv0.npy"), np.load(tmp_path / "mv1.npy")
    assert np.array_equal(m0, m1)
    l0, l1 = np.load(tmp_path / "loc0.npy"), np.load(tmp_path / "loc1.npy")
    g0, g1 = np.load(tmp_path / "mrg0.npy"), np.load(tmp_path / "mrg1.npy")
    np.testing.assert_allclose(g0, l0 + l1)
    np.testing.assert_allclose(g1, l0 + l1)
    assert not np.array_equal(l0, l1), "ranks ran identical searches (seeds not per rank)"
    for k in range(len(m0)):
        assert m0[k] == int(np.argmax(g0[k])) or (m0[k] == -1 and np.argmax(g0[k]) == 49)


def _rl_worker(rank, world, port, outdir):
    _setup(rank, world, port)
    import numpy as np_
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.players.ai import ProbabilisticPolicyPlayer
    from rocalphago_amd.training import reinforcement as rl
    dp = DPContext(device="cpu")
    np_.random.seed(100 + rank)  # different self-play games per rank
    learner = CNNPolicy(FEATS, board=7, filters_per_layer=8, layers=2, device="cpu", seed=3)
    opponent = CNNPolicy(FEATS, board=7, filters_per_layer=8, layers=2, device="cpu", seed=4)
    dp.broadcast_model(learner.model)
    opt = K.SGD(lr=0.01)
    learner.model.compile(loss=rl.log_loss, optimizer=opt)
    ratio = rl.run_n_games(opt, ProbabilisticPolicyPlayer(learner, move_limit=40),
                           ProbabilisticPolicyPlayer(opponent, move_limit=40), 4,
                           mode="batched", dp=dp)
    np_.save(os.path.join(outdir, "rl%d.npy" % rank), learner.model.net.flat.detach().numpy())
    np_.save(os.path.join(outdir, "ratio%d.npy" % rank), np_.array([ratio]))
    dp.shutdown()


@pytest.mark.timeout(300)
def test_dp_rl_selfplay_sharded(tmp_path):
    """RL self-play sharded over 2 ranks: different games, one all-reduced REINFORCE update,
    identical replicas afterwards."""
    _spawn(_rl_worker, (str(tmp_path),))
    a, b = np.load(tmp_path / "rl0.npy"), np.load(tmp_path / "rl1.npy")
    assert np.array_equal(a, b)
    from rocalphago_amd.models.policy import CNNPolicy
    fresh = CNNPolicy(FEATS, board=7, filters_per_layer=8, layers=2, device="cpu", seed=3)
    assert not np.allclose(a, fresh.model.net.flat.detach().numpy()), "no update happened"


def _write_value_fixture(tmp):
    """Tiny CNNValue (7x7, 3 planes of 'board' + color) and an HDF5 dataset of 40 positions."""
    from rocalphago_amd.io import h5lite
    from rocalphago_amd.models.value import CNNValue
    feats = ["board", "color"]
    net = CNNValue(feats, board=7, filters_per_layer=8, layers=2, dense=16, seed=5,
                   device="cpu")
    model_json = os.path.join(tmp, "value.json")
    net.save_model(model_json)
    rng = np.random.RandomState(0)
    X = (rng.rand(40, 4, 7, 7) < 0.3).astype(np.uint8)
    y = rng.choice([-1.0, 1.0], size=(40, 1)).astype(np.float32)
    data = os.path.join(tmp, "vdata.h5")
    with h5lite.File(data, "w") as f:
        f["states"] = X
        f["values"] = y
        f["features"] = np.bytes_(",".join(feats))
    return model_json, data


def _value_worker(rank, world, port, outdir, model_json, data):
    _setup(rank, world, port)
    from rocalphago_amd.training import value_trainer as vt
    captured = {}
    orig = vt.CNNValue.load_model

    def load(*a, **kw):
        captured["net"] = orig(*a, **kw)
        return captured["net"]

    vt.CNNValue.load_model = staticmethod(load)
    # 0.93 * 40 = 37 -> 36 training rows = 9 minibatches of 4: an odd number of batches, so
    # ranks would run 5 vs 4 all-reduces without the shared step count
    meta = vt.run_training([model_json, data, os.path.join(outdir, "out"), "-B", "4", "-E", "2",
                            "--symmetries", "noop,rot90"])
    np.save(os.path.join(outdir, "vflat%d.npy" % rank),
            captured["net"].model.net.flat.detach().numpy())
    np.save(os.path.join(outdir, "vloss%d.npy" % rank),
            np.array([e["val_loss"] for e in meta["epochs"]]))


@pytest.mark.timeout(300)
def test_dp_value_training_uneven_batches(tmp_path):
    """Value trainer under 2 gloo ranks with an odd number of minibatches per epoch: same step
    count on every rank (no collective mismatch), identical replicas, sharded validation whose
    all-reduced MSE every rank agrees on, per-rank metrics streams, resumable sidecar."""
    import json
    model_json, data = _write_value_fixture(str(tmp_path))
    _spawn(_value_worker, (str(tmp_path), model_json, data))
    a, b = np.load(tmp_path / "vflat0.npy"), np.load(tmp_path / "vflat1.npy")
    assert np.array_equal(a, b), "value replicas diverged"
    l0, l1 = np.load(tmp_path / "vloss0.npy"), np.load(tmp_path / "vloss1.npy")
    np.testing.assert_allclose(l0, l1)
    out = tmp_path / "out"
    assert (out / "weights.00001.hdf5").exists()
    side = json.load(open(out / "weights.00001.opt.json"))
    assert side["iterations"] == 2 * 5  # ceil(36 / (4 * 2)) = 5 steps per epoch
    for r in range(2):
        recs = [json.loads(line) for line in open(out / ("metrics.rank%d.jsonl" % r))]
        assert len(recs) == 2 and recs[-1]["rank"] == r and recs[-1]["steps"] == 5


def _resnet_worker(rank, world, port, outdir):
    _setup(rank, world, port)
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import ResnetPolicy
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.training.supervised import SupervisedTrainer
    dp = DPContext(device="cpu")
    pol = ResnetPolicy(FEATS, board=9, filters_per_layer=8, layers=3, device="cpu", seed=2)
    model = pol.model
    model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.05), metrics=["accuracy"])
    dp.broadcast_model(model)
    trainer = SupervisedTrainer(model, _dataset(), 8, ["noop"], dp, seed=0)
    for s in range(3):
        trainer.step(torch.arange(s * 16 + rank * 8, s * 16 + (rank + 1) * 8))
    vl, va = trainer.evaluate(torch.arange(48, 64))
    np.save(os.path.join(outdir, "rflat%d.npy" % rank), model.net.flat.detach().numpy())
    np.save(os.path.join(outdir, "rbuf%d.npy" % rank),
            torch.cat([v.reshape(-1) for v in model.net.buffer_views()]).numpy())
    np.save(os.path.join(outdir, "rval%d.npy" % rank), np.array([vl, va]))
    dp.shutdown()


@pytest.mark.timeout(300)
def test_dp_resnet_bn_buffers_synced(tmp_path):
    """ResnetPolicy under DP: the BatchNorm running averages are averaged over ranks each step,
    so replicas (weights AND BN buffers) stay identical; validation is sharded by rank and the
    all-reduced result equals a single-process evaluation of the same rows."""
    _spawn(_resnet_worker, (str(tmp_path),))
    b0, b1 = np.load(tmp_path / "rbuf0.npy"), np.load(tmp_path / "rbuf1.npy")
    assert b0.size > 0
    np.testing.assert_array_equal(b0, b1)
    f0, f1 = np.load(tmp_path / "rflat0.npy"), np.load(tmp_path / "rflat1.npy")
    np.testing.assert_array_equal(f0, f1)
    v0, v1 = np.load(tmp_path / "rval0.npy"), np.load(tmp_path / "rval1.npy")
    np.testing.assert_allclose(v0, v1)
    # single-process evaluation of the trained replica on the same 16 rows
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import ResnetPolicy
    from rocalphago_amd.training.supervised import SupervisedTrainer
    torch.set_num_threads(1)
    pol = ResnetPolicy(FEATS, board=9, filters_per_layer=8, layers=3, device="cpu", seed=2)
    pol.model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.05),
                      metrics=["accuracy"])
    with torch.no_grad():
        pol.model.net.flat.copy_(torch.from_numpy(f0))
    pol.model.net.bump()
    tr = SupervisedTrainer(pol.model, _dataset(), 8, ["noop"], None, seed=0)
    vl, va = tr.evaluate(torch.arange(48, 64))
    np.testing.assert_allclose(v0, [vl, va], rtol=1e-5)


def _rl_pergame_worker(rank, world, port, outdir):
    _setup(rank, world, port)
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.players.ai import ProbabilisticPolicyPlayer
    from rocalphago_amd.training import reinforcement as rl
    dp = DPContext(device="cpu")
    pol = CNNPolicy(FEATS, board=7, filters_per_layer=8, layers=2, device="cpu", seed=3)
    opt = K.SGD(lr=0.01)
    pol.model.compile(loss=rl.log_loss, optimizer=opt)
    p = ProbabilisticPolicyPlayer(pol, move_limit=10)
    try:
        rl.run_n_games(opt, p, p, 2, mode="per_game", dp=dp)
        ok = 0
    except ValueError:
        ok = 1
    np.save(os.path.join(outdir, "pg%d.npy" % rank), np.array([ok]))
    dp.shutdown()


@pytest.mark.timeout(300)
def test_dp_rl_per_game_rejected(tmp_path):
    _spawn(_rl_pergame_worker, (str(tmp_path),))
    assert np.load(tmp_path / "pg0.npy")[0] == 1 and np.load(tmp_path / "pg1.npy")[0] == 1


def test_forced_single_rank_group_cpu(monkeypatch):
    """RAG_FORCE_PG=1 at WORLD_SIZE=1 (gloo here, RCCL on a GPU box: tests/test_gpu_rccl.py):
    the DP code paths run real collectives of one rank, which leave values unchanged."""
    import torch.distributed as dist

    from rocalphago_amd.parallel.dp import BucketedAllReduce, DPContext
    from rocalphago_amd.parallel.watchdog import RankWatchdog
    from rocalphago_amd.search.distributed import RootExchange
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("RAG_FORCE_PG", "1")
    dp = DPContext(device="cpu")
    try:
        assert dp.enabled and dp.world == 1 and dp.backend == "gloo"
        g = torch.randn(1000)
        ref = g.clone()
        b = BucketedAllReduce(dp, g, [0, 300, 700], bucket_bytes=256)
        for layer in (2, 1, 0):
            b.layer_done(layer)
        b.finish()
        assert torch.equal(g, ref)
        dp.barrier()
        rx = RootExchange(8, torch.device("cpu"))
        v = np.arange(8, dtype=np.float32)
        assert rx.exchange(v) is None
        tot, own = rx.wait()
        assert np.array_equal(tot, v) and np.array_equal(own, v)
        wd = RankWatchdog(0, 1, 60.0, phase="forced", on_stall=lambda m: None)
        wd.beat(3)
        wd._publish(force=True)
        assert wd.heartbeats()[0][:2] == ("forced", 3)
        wd.stop()
    finally:
        dp.shutdown()
    assert not dist.is_initialized()


def _rl_games(n_games=6, board=7, planes=12, seed=0):
    """Fixed synthetic REINFORCE batch: per game a few positions, moves and an outcome."""
    rng = np.random.RandomState(seed)
    feats, moves, won = [], [], []
    for g in range(n_games):
        n = 3 + g % 4
        feats.append([(rng.rand(planes, board, board) < 0.3).astype(np.float32)
                      for _ in range(n)])
        moves.append([int(m) for m in rng.randint(0, board * board, n)])
        won.append(bool(g % 3 != 1))
    return feats, moves, won


def _rl_policy():
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.training import reinforcement as rl
    pol = CNNPolicy(FEATS, board=7, filters_per_layer=8, layers=3, device="cpu", seed=3)
    opt = K.SGD(lr=0.05)
    pol.model.compile(loss=rl.log_loss, optimizer=opt)
    return pol.model, opt


def _rl_sym_worker(rank, world, port, outdir):
    """Each rank updates on its shard (games rank::world) of the fixed batch, once with the
    outcomes as given and once with every outcome flipped, from the same initial weights."""
    _setup(rank, world, port)
    from rocalphago_amd.parallel.dp import DPContext
    from rocalphago_amd.training import reinforcement as rl
    dp = DPContext(device="cpu")
    feats, moves, won = _rl_games()
    mine = list(range(rank, len(won), world))
    for tag, flip in (("w", False), ("l", True)):
        model, opt = _rl_policy()
        init = model.net.flat.detach().clone()
        rl._batched_update(model, opt, [feats[i] for i in mine], [moves[i] for i in mine],
                           [won[i] != flip for i in mine], 49, dp)
        np.save(os.path.join(outdir, "d%s%d.npy" % (tag, rank)),
                (model.net.flat.detach() - init).numpy())
    dp.shutdown()


@pytest.mark.timeout(300)
def test_dp_rl_update_symmetry_and_union(tmp_path):
    """Cross-rank version of the reference's gradient-symmetry check
    (/root/reference/tests/test_reinforcement_policy_trainer.py:82-126):
    the all-reduced batched REINFORCE update over 2 ranks equals the single-process batched
    update on the union of the games, and flipping every win/loss gives the equal and opposite
    weight change."""
    from rocalphago_amd.training import reinforcement as rl
    _spawn(_rl_sym_worker, (str(tmp_path),))
    dw0, dw1 = np.load(tmp_path / "dw0.npy"), np.load(tmp_path / "dw1.npy")
    dl0, dl1 = np.load(tmp_path / "dl0.npy"), np.load(tmp_path / "dl1.npy")
    assert np.array_equal(dw0, dw1) and np.array_equal(dl0, dl1), "replicas diverged"
    feats, moves, won = _rl_games()
    model, opt = _rl_policy()
    init = model.net.flat.detach().clone()
    rl._batched_update(model, opt, feats, moves, won, 49, None)
    single = (model.net.flat.detach() - init).numpy()
    assert np.abs(single).max() > 0
    assert np.linalg.norm(dw0 - single) <= 1e-5 * np.linalg.norm(single)
    np.testing.assert_allclose(dl0, -dw0, rtol=1e-3, atol=1e-7 * np.abs(dw0).max())


def _adopt_worker(rank, world, port, outdir):
    import torch.distributed as dist
    _setup(rank, world, port)
    dist.init_process_group("gloo")
    from rocalphago_amd.parallel.dp import DPContext
    # a group exists but the environment claims a single process: not adopted by default
    os.environ["WORLD_SIZE"] = "1"
    os.environ.pop("RAG_FORCE_PG", None)
    plain = DPContext(device="cpu")
    adopted = DPContext(device="cpu", adopt=True)
    res = [int(plain.enabled), plain.world, int(adopted.enabled), adopted.world, adopted.rank,
           adopted.local_rank]
    with open(os.path.join(outdir, "r%d.txt" % rank), "w") as f:
        f.write(" ".join(map(str, res)))
    dist.barrier()
    dist.destroy_process_group()


def test_dpcontext_adopts_an_existing_group_only_on_request(tmp_path):
    """DPContext used to switch itself on whenever any process group existed, taking
    rank/world from the group but the device from the environment."""
    mp.spawn(_adopt_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    ndev = max(1, torch.cuda.device_count())
    for r in range(2):
        got = open(os.path.join(str(tmp_path), "r%d.txt" % r)).read().split()
        assert got == ["0", "1", "1", "2", str(r), str(r % ndev)], got
