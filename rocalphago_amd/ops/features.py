"""GPU feature planes (csrc/hip/features.hip, csrc/hip/ladder.hip) for batched search evaluation.

``GpuFeatures(feature_list)(boards)`` returns the same uint8 ``[n, F, S, S]`` planes as
``_rocgo.batch_features`` but built on the device: the native engine only exports colours,
stone ages and the player / ko. Everything else (groups, liberties, captures, simulated
liberties after each move, the recursive eye rule, legality) is computed by one wavefront per
position. The two ladder planes come either from the native search on the host thread pool
(``ladders="host"``) or from the GPU ladder kernels (``ladders="gpu"``: one wavefront per ladder
read, an explicit DFS with in-place moves and undo, csrc/hip/ladder.hip). Measured on one MI355X
(256 mid-game 19x19 positions): the GPU path builds all planes in 2.1 ms against 2.7-3.0 ms with
16 host threads, but inside the pipelined search the host ladders run while the GPU evaluates
the previous wave, whereas the GPU ladder reads (a few long sequential DFS per batch) sit on the
GPU's critical path: 97k vs 45k simulations/s (lambda = 0). So "host" is the default and "gpu"
is for callers with no concurrent GPU work (RAG_LADDERS=gpu switches the default). Boards that
enforce positional superko always use the native search (their legality depends on the game
history). The planes stay on the GPU and feed the fused network input packer directly
(models/fused.py prepare()).
"""
import os

import numpy as np
import torch

from .._native import engine as _engine
from ..features.preprocessing import Preprocess, _FID
from .hipops import _check, _lib, _ptr, _stream

_rg = _engine()
_LADDERS = (_FID["ladder_capture"], _FID["ladder_escape"])
_DEFAULT_LADDERS = os.environ.get("RAG_LADDERS", "host")


def _h2d(a, device):
    if a is None:
        return None
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(device, non_blocking=True)


def gpu_ladders(colors, meta, S, out=None, work=None):
    """Ladder planes [n, 2, S*S] uint8 (capture, escape) on the device from device colours
    [n, S*S] int8 and meta [n, 4] int32 (player to move, ko point) — the native
    is_ladder_capture / is_ladder_escape of every point, without positional superko."""
    n = colors.shape[0]
    dev = colors.device
    if out is None:
        out = torch.empty((n, 2, S * S), dtype=torch.uint8, device=dev)
    need = int(_lib().rag_ladder_workspace(n, S))
    if work is None or work.numel() < need:
        work = torch.empty(need, dtype=torch.uint8, device=dev)
    _check(_lib().rag_ladders(_ptr(colors), _ptr(meta), n, S, _ptr(work), _ptr(out), _stream()),
           "ladders")
    return out, work


class GpuFeatures(object):
    def __init__(self, feature_list, device=None, nthreads=8, ladders=None):
        self.pre = Preprocess(feature_list)
        self.fids = self.pre.feature_ids
        self.F = self.pre.output_dim
        self.device = torch.device(device or "cuda")
        self.fids_dev = torch.tensor(self.fids, dtype=torch.int32, device=self.device)
        self.ladders = any(f in _LADDERS for f in self.fids)
        self.nthreads = nthreads
        self._work = None
        self._retired = []
        self.ladder_device = ladders or _DEFAULT_LADDERS
        if self.ladder_device not in ("host", "gpu"):
            raise ValueError("ladders must be 'host' or 'gpu'")

    @staticmethod
    def supports(size):
        return size * size <= 384

    def __call__(self, boards, out=None, sens_out=None):
        """Planes [n, F, S, S] on the device; with ``sens_out`` (uint8 [n, S*S] or [n, 1, S, S])
        also the sensibleness mask (legal, not an own true eye) from the same native inputs."""
        host = self.ladders and (self.ladder_device == "host" or
                                 any(b.enforce_superko for b in boards))
        colors, ages, meta, illegal, lad = _rg.gpu_feature_inputs(boards, host, self.nthreads)
        return self.from_arrays(colors, ages, meta, illegal, lad, out, sens_out)

    def run(self, c, a, m, il, ld, n, S, out=None, sens_out=None):
        """Planes from device inputs (colours [n, S*S] int8, ages int16, meta [n, 4] int32,
        superko-illegal mask or None, ladder planes [n, 2, S*S] or None: read on the GPU);
        with ``sens_out`` (uint8, n*S*S elements) also the sensibleness mask."""
        if self.ladders and ld is None:
            old = self._work
            ld, self._work = gpu_ladders(c, m, S, work=self._work)
            if old is not None and self._work is not old:
                # a grown workspace never frees the old one: a captured HIP graph (self-play
                # plies replay as graphs) may still address it
                self._retired.append(old)
        if out is None:
            out = torch.empty((n, self.F, S, S), dtype=torch.uint8, device=self.device)
        if sens_out is not None and (sens_out.numel() != n * S * S or
                                     sens_out.dtype != torch.uint8 or
                                     not sens_out.is_contiguous()):
            raise ValueError("sens_out must be contiguous uint8 with n*S*S elements")
        # one pass: the planes and (optionally) the sensible-move mask
        _check(_lib().rag_features(_ptr(c), _ptr(a), _ptr(m), _ptr(il), _ptr(ld), n, S,
                                   _ptr(self.fids_dev), len(self.fids), self.F, _ptr(out),
                                   _ptr(sens_out), _stream()), "features")
        return out

    def from_arrays(self, colors, ages, meta, illegal, lad, out=None, sens_out=None):
        """Planes from the native inputs directly: colours [n, S*S] int8, stone ages int16,
        meta [n, 4] int32 (player, ko, superko flag, 0), the superko-illegal mask (or None) and
        the ladder planes [n, 2, S*S] (or None: read on the GPU) — e.g. leaves shipped to another
        rank (search/distributed.py)."""
        n = colors.shape[0]
        S = int(round(np.sqrt(colors.shape[1])))
        if illegal is not None and not np.any(illegal):
            illegal = None
        c, a, m, il, ld = (_h2d(x, self.device) for x in (colors, ages, meta, illegal, lad))
        return self.run(c, a, m, il, ld, n, S, out, sens_out)
