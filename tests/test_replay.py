"""Bit-packed GPU-resident positions (training/replay.py) and the replay buffer."""
import numpy as np
import pytest
import torch

from rocalphago_amd.training.replay import (PackedDataset, ReplayBuffer, pack_bits,
                                            unpack_bits)


def test_pack_roundtrip():
    rs = np.random.RandomState(0)
    for F in (1, 12, 48, 49, 64):
        x = torch.from_numpy((rs.rand(5, F, 9, 9) > 0.5).astype(np.uint8))
        b = pack_bits(x)
        assert b.dtype == torch.int64 and b.shape == (5, 9, 9)
        assert torch.equal(unpack_bits(b, F), x)
    with pytest.raises(ValueError):
        pack_bits(torch.zeros(1, 65, 3, 3, dtype=torch.uint8))


def test_packed_dataset_host_batch_matches_plain():
    from rocalphago_amd.training.data import DeviceDataset
    rs = np.random.RandomState(1)
    st = (rs.rand(20, 12, 9, 9) > 0.6).astype(np.uint8)
    acts = rs.randint(0, 81, 20)
    plain = DeviceDataset(st, acts, "cpu")
    packed = PackedDataset(st, acts, "cpu")
    idx = torch.tensor([3, 0, 7, 19])
    tf = torch.tensor([0, 1, 5, 7], dtype=torch.int32)
    a, b = plain.host_batch(idx, tf), packed.host_batch(idx, tf)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_replay_ring_and_sizing():
    rb = ReplayBuffer(10, 49, 9, "cpu")
    x = (torch.rand(7, 49, 9, 9) > 0.5).to(torch.uint8)
    rb.add(x, torch.arange(7.0))
    assert len(rb) == 7 and rb.head == 7
    rb.add(x, torch.arange(7.0) + 100)  # wraps: 3 at the end, 4 at the front
    assert len(rb) == 10 and rb.head == 4 and rb.added == 14
    assert rb.targets[:4].tolist() == [103.0, 104.0, 105.0, 106.0]
    assert torch.equal(rb.planes_u8(torch.tensor([0])), x[3:4])
    idx = rb.sample(32, torch.Generator().manual_seed(0))
    assert idx.max() < 10
    big = ReplayBuffer.for_memory(48, 19, "cpu", budget_bytes=2 ** 20)
    assert big.capacity == 2 ** 20 // ReplayBuffer.bytes_per_position(19)
    # 288 GB of HBM at half occupancy holds tens of millions of packed 19x19 positions
    assert 144e9 / ReplayBuffer.bytes_per_position(19) > 4e7


def test_supervised_trainer_on_packed_cpu():
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.training.supervised import SupervisedTrainer
    rs = np.random.RandomState(2)
    st = (rs.rand(32, 12, 9, 9) > 0.6).astype(np.uint8)
    ds = PackedDataset(st, rs.randint(0, 81, 32), "cpu")
    pol = CNNPolicy(["board", "ones", "turns_since"], board=9, filters_per_layer=8, layers=2,
                    device="cpu")
    pol.model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.1))
    tr = SupervisedTrainer(pol.model, ds, 8, ["noop", "rot90"], None)
    tr.step(torch.arange(8))
    loss, _ = tr.pop_metrics()
    assert np.isfinite(loss)


def test_value_trainer_from_replay_cpu():
    from rocalphago_amd.features.preprocessing import VALUE_FEATURES
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.value import CNNValue
    from rocalphago_amd.training.value_trainer import ValueTrainer
    val = CNNValue(VALUE_FEATURES, board=7, filters_per_layer=8, layers=2, device="cpu")
    val.model.compile(loss="mse", optimizer=K.SGD(lr=0.01))
    rb = ReplayBuffer(64, 49, 7, "cpu")
    rb.add((torch.rand(40, 49, 7, 7) > 0.5).to(torch.uint8), torch.randint(0, 2, (40,)) * 2 - 1)
    tr = ValueTrainer.from_replay(val.model, rb, 8, ["noop", "fliplr"])
    tr.step(rb.sample(8, torch.Generator().manual_seed(1)))
    assert np.isfinite(tr.pop_loss())
