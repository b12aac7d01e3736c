"""GPU feature planes (csrc/hip/features.hip) for batched search evaluation.

``GpuFeatures(feature_list)(boards)`` returns the same uint8 ``[n, F, S, S]`` planes as
``_rocgo.batch_features`` but built on the device: the native engine only exports colours,
stone ages, the player / ko and — if the ladder planes are requested — the ladder reads (a deep
sequential search that stays native, run on a thread pool); everything else (groups, liberties,
captures, simulated liberties after each move, the recursive eye rule, legality) is computed by
one wavefront per position. The planes stay on the GPU and feed the fused network input packer
directly (models/fused.py prepare()).
"""
import numpy as np
import torch

from .._native import engine as _engine
from ..features.preprocessing import Preprocess, _FID
from .hipops import _check, _lib, _ptr, _stream

_rg = _engine()
_LADDERS = (_FID["ladder_capture"], _FID["ladder_escape"])


class GpuFeatures(object):
    def __init__(self, feature_list, device=None, nthreads=8):
        self.pre = Preprocess(feature_list)
        self.fids = self.pre.feature_ids
        self.F = self.pre.output_dim
        self.device = torch.device(device or "cuda")
        self.fids_dev = torch.tensor(self.fids, dtype=torch.int32, device=self.device)
        self.ladders = any(f in _LADDERS for f in self.fids)
        self.nthreads = nthreads
        self._sens_fid = None

    @staticmethod
    def supports(size):
        return size * size <= 384

    def _h2d(self, a):
        if a is None:
            return None
        return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(self.device,
                                                                          non_blocking=True)

    def __call__(self, boards, out=None, sens_out=None):
        """Planes [n, F, S, S] on the device; with ``sens_out`` (uint8 [n, S*S] or [n, 1, S, S])
        also the sensibleness mask (legal, not an own true eye) from the same native inputs."""
        n = len(boards)
        S = boards[0].size
        colors, ages, meta, illegal, lad = _rg.gpu_feature_inputs(boards, self.ladders,
                                                                  self.nthreads)
        c, a, m, il, ld = (self._h2d(x) for x in (colors, ages, meta, illegal, lad))
        if out is None:
            out = torch.empty((n, self.F, S, S), dtype=torch.uint8, device=self.device)
        _check(_lib().rag_features(_ptr(c), _ptr(a), _ptr(m), _ptr(il), _ptr(ld), n, S,
                                   _ptr(self.fids_dev), len(self.fids), self.F, _ptr(out),
                                   _stream()), "features")
        if sens_out is not None:
            if sens_out.numel() != n * S * S or sens_out.dtype != torch.uint8:
                raise ValueError("sens_out must be uint8 with n*S*S elements")
            if self._sens_fid is None:
                self._sens_fid = torch.tensor([_FID["sensibleness"]], dtype=torch.int32,
                                              device=self.device)
            _check(_lib().rag_features(_ptr(c), _ptr(a), _ptr(m), _ptr(il), None, n, S,
                                       _ptr(self._sens_fid), 1, 1, _ptr(sens_out), _stream()),
                   "features(sensibleness)")
        return out
