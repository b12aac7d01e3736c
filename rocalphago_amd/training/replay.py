"""GPU-resident position storage sized for MI355X HBM (288 GB per GPU).

A 19x19 position with F <= 64 binary feature planes is stored bit-packed: one 64-bit word per
point (bit f = plane f), 2.9 KB instead of 17.3 KB of uint8 planes — about 6x more positions in
the same HBM (tens of millions per GPU). The trunk input packer unpacks the bits on the fly
(``rag_pack_input_bits`` in csrc/hip/conv.hip, same index gather and dihedral transform as the
uint8 path), so training reads packed positions directly.

* ``pack_bits`` / ``unpack_bits``: uint8 planes [N, F, S, S] <-> int64 words [N, S, S]
  (plain tensor ops, any device).
* ``PackedDataset``: a ``DeviceDataset`` (SL positions + move labels) stored packed.
* ``ReplayBuffer``: a fixed-capacity ring of packed positions with targets (value-net outcomes or
  move labels) for self-play data; ``ReplayBuffer.for_memory`` sizes it from a byte budget or a
  fraction of the free device memory.
"""
import numpy as np
import torch

from .data import DeviceDataset, apply_transform_np, label_transform_table


def pack_bits(planes):
    """uint8/bool planes [N, F, S, S] (F <= 64) -> int64 words [N, S, S]."""
    planes = torch.as_tensor(planes)
    N, F = planes.shape[0], planes.shape[1]
    if F > 64:
        raise ValueError("at most 64 planes can be bit-packed")
    out = torch.zeros((N,) + tuple(planes.shape[2:]), dtype=torch.int64, device=planes.device)
    for f in range(F):
        out |= (planes[:, f].to(torch.int64) & 1) << f
    return out


def unpack_bits(bits, nplanes):
    """int64 words [N, S, S] -> uint8 planes [N, F, S, S]."""
    bits = torch.as_tensor(bits)
    shifts = torch.arange(nplanes, device=bits.device, dtype=torch.int64).view(1, -1, 1, 1)
    return ((bits.unsqueeze(1) >> shifts) & 1).to(torch.uint8)


class PackedDataset(DeviceDataset):
    """DeviceDataset whose ``states`` are bit-packed int64 words [N, S, S]."""

    def __init__(self, states, actions, device, board=None):
        states = np.asarray(states)
        self.N, self.F, self.S = states.shape[0], states.shape[1], states.shape[-1]
        acts = np.asarray(actions).astype(np.int64)
        labels = acts[:, 0] * self.S + acts[:, 1] if acts.ndim == 2 else acts
        self.device = torch.device(device)
        # pack in chunks on the target device (bounded host memory for large datasets)
        chunks = []
        for s in range(0, self.N, 65536):
            chunks.append(pack_bits(torch.from_numpy(
                np.ascontiguousarray(states[s:s + 65536], dtype=np.uint8)).to(self.device)))
        self.states = torch.cat(chunks) if chunks else torch.zeros(
            (0, self.S, self.S), dtype=torch.int64, device=self.device)
        self.labels = torch.from_numpy(labels).to(self.device)
        self.tf_table = torch.from_numpy(label_transform_table(self.S)).to(self.device)

    @classmethod
    def from_hdf5(cls, h5file, device):
        return cls(h5file["states"][()], h5file["actions"][()], device)

    @property
    def planes(self):
        return self.F

    def host_batch(self, index, tf):
        idx = index.to(self.device)
        st = unpack_bits(self.states[idx], self.F).cpu().numpy()
        tfs = tf.cpu().numpy()
        X = np.stack([apply_transform_np(s, t) for s, t in zip(st, tfs)]).astype(np.float32)
        lab = self.batch_labels(idx, tf.to(self.device)).cpu().numpy()
        Y = np.zeros((len(st), self.S * self.S), np.float32)
        Y[np.arange(len(st)), lab] = 1
        return X, Y


class ReplayBuffer(object):
    """Ring buffer of bit-packed positions + float targets on one device."""

    BYTES_PER_POINT = 8

    def __init__(self, capacity, planes, board, device, target_dtype=torch.float32):
        if planes > 64:
            raise ValueError("at most 64 planes can be bit-packed")
        self.capacity = int(capacity)
        self.F, self.S = planes, board
        self.device = torch.device(device)
        self.states = torch.zeros((self.capacity, board, board), dtype=torch.int64,
                                  device=self.device)
        self.targets = torch.zeros((self.capacity,), dtype=target_dtype, device=self.device)
        self.size = 0
        self.head = 0
        self.added = 0

    @classmethod
    def bytes_per_position(cls, board, target_dtype=torch.float32):
        return board * board * cls.BYTES_PER_POINT + torch.finfo(target_dtype).bits // 8 \
            if target_dtype.is_floating_point else board * board * cls.BYTES_PER_POINT + 8

    @classmethod
    def for_memory(cls, planes, board, device, budget_bytes=None, fraction=0.5,
                   target_dtype=torch.float32):
        """Capacity from an explicit byte budget or ``fraction`` of the device's free memory
        (on a 288 GB MI355X, half of HBM holds ~49 M packed 19x19 positions)."""
        device = torch.device(device)
        if budget_bytes is None:
            if device.type == "cuda":
                free, _ = torch.cuda.mem_get_info(device)
                budget_bytes = int(free * fraction)
            else:
                budget_bytes = 1 << 28
        per = cls.bytes_per_position(board, target_dtype)
        return cls(max(1, budget_bytes // per), planes, board, device, target_dtype)

    def __len__(self):
        return self.size

    def add(self, planes_or_bits, targets):
        """Append positions (uint8 planes [n, F, S, S] or packed words [n, S, S]) with their
        targets; the oldest entries are overwritten once full."""
        x = torch.as_tensor(planes_or_bits)
        bits = x if x.dtype == torch.int64 and x.dim() == 3 else pack_bits(x)
        bits = bits.to(self.device)
        t = torch.as_tensor(targets, dtype=self.targets.dtype).reshape(-1).to(self.device)
        n = bits.shape[0]
        if n > self.capacity:
            bits, t, n = bits[-self.capacity:], t[-self.capacity:], self.capacity
        end = self.head + n
        if end <= self.capacity:
            self.states[self.head:end] = bits
            self.targets[self.head:end] = t
        else:
            k = self.capacity - self.head
            self.states[self.head:] = bits[:k]
            self.targets[self.head:] = t[:k]
            self.states[:n - k] = bits[k:]
            self.targets[:n - k] = t[k:]
        self.head = end % self.capacity
        self.size = min(self.capacity, self.size + n)
        self.added += n

    def sample(self, n, generator=None):
        """n random indices (with replacement) into the filled part of the buffer."""
        if self.size == 0:
            raise ValueError("empty replay buffer")
        return torch.randint(0, self.size, (n,), generator=generator, device=self.device)

    def planes_u8(self, index):
        return unpack_bits(self.states[index], self.F)
