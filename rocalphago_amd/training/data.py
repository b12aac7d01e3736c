"""Training data: device-resident position datasets and the 8 board symmetries.

The reference streams every sample through a single-threaded python generator that reads HDF5,
transforms each plane with numpy and builds float64 batches (supervised_policy_trainer.py:19-45).
Here the whole uint8 dataset is loaded into HBM once (one 48-plane 19x19 position is 17.3 KB:
288 GB holds ~16 M of them), and a batch is (index tensor, transform-id tensor): the HIP
pack-input kernel gathers the rows, applies the dihedral transform and converts to the padded
bf16 layout in one pass (K08); labels are remapped through a precomputed [8, S*S] table.
"""
import numpy as np
import torch

# reference order/names (supervised_policy_trainer.py:76-85)
TRANSFORM_NAMES = ["noop", "rot90", "rot180", "rot270", "fliplr", "flipud", "diag1", "diag2"]

BOARD_TRANSFORMATIONS = {
    "noop": lambda feature: feature,
    "rot90": lambda feature: np.rot90(feature, 1),
    "rot180": lambda feature: np.rot90(feature, 2),
    "rot270": lambda feature: np.rot90(feature, 3),
    "fliplr": lambda feature: np.fliplr(feature),
    "flipud": lambda feature: np.flipud(feature),
    "diag1": lambda feature: np.transpose(feature),
    "diag2": lambda feature: np.fliplr(np.rot90(feature, 1))
}


def transform_ids(names):
    return [TRANSFORM_NAMES.index(n) for n in names]


def label_transform_table(S):
    """table[t, p] = index of the one-hot target after transform t (same map as the planes)."""
    table = np.zeros((8, S * S), dtype=np.int64)
    for t, name in enumerate(TRANSFORM_NAMES):
        for p in range(S * S):
            onehot = np.zeros((S, S))
            onehot[divmod(p, S)] = 1
            q = int(np.argmax(BOARD_TRANSFORMATIONS[name](onehot)))
            table[t, p] = q
    return table


def apply_transform_np(planes, t):
    """(F, S, S) planes -> transformed copy (CPU reference path)."""
    fn = BOARD_TRANSFORMATIONS[TRANSFORM_NAMES[t]]
    return np.stack([fn(p) for p in planes])


class DeviceDataset(object):
    """uint8 states [N, F, S, S] + flat action labels [N] resident on ``device``."""

    def __init__(self, states, actions, device, board=None):
        states = np.asarray(states)
        self.N, self.F, self.S = states.shape[0], states.shape[1], states.shape[-1]
        acts = np.asarray(actions).astype(np.int64)
        labels = acts[:, 0] * self.S + acts[:, 1] if acts.ndim == 2 else acts
        self.device = torch.device(device)
        self.states = torch.from_numpy(np.ascontiguousarray(states, dtype=np.uint8)).to(
            self.device)
        self.labels = torch.from_numpy(labels).to(self.device)
        self.tf_table = torch.from_numpy(label_transform_table(self.S)).to(self.device)

    @classmethod
    def from_hdf5(cls, h5file, device):
        return cls(h5file["states"][()], h5file["actions"][()], device)

    @classmethod
    def synthetic(cls, n, planes, board, device, seed=0, density=0.35):
        """Random binary planes / uniform labels generated on the device (benchmarks)."""
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        ds = cls.__new__(cls)
        ds.N, ds.F, ds.S = n, planes, board
        ds.device = torch.device(device)
        ds.states = (torch.rand((n, planes, board, board), generator=g, device=device) <
                     density).to(torch.uint8)
        ds.labels = torch.randint(0, board * board, (n,), generator=g, device=device)
        ds.tf_table = torch.from_numpy(label_transform_table(board)).to(ds.device)
        return ds

    def batch_labels(self, index, tf):
        return self.tf_table[tf, self.labels[index]]

    def host_batch(self, index, tf):
        """CPU path: (X float32 [B,F,S,S], Y one-hot [B,S*S]) materialised with numpy."""
        idx = index.cpu().numpy()
        tfs = tf.cpu().numpy()
        st = self.states.cpu().numpy()
        X = np.stack([apply_transform_np(st[i], t) for i, t in zip(idx, tfs)]).astype(
            np.float32)
        lab = self.batch_labels(index.to(self.device), tf.to(self.device)).cpu().numpy()
        Y = np.zeros((len(idx), self.S * self.S), np.float32)
        Y[np.arange(len(idx)), lab] = 1
        return X, Y
