"""Loaders for the two native artefacts.

* ``engine()`` returns the C++ pybind11 module (rules engine, features, LZF, search). It is
  required everywhere (CPU and GPU); if the in-tree .so is missing or stale it is rebuilt.
* ``hip()`` returns the ctypes handle of the gfx950 HIP kernel library. On a machine with a GPU
  the HIP path is mandatory: a missing library raises instead of silently falling back to eager
  PyTorch (``RAG_ALLOW_TORCH_FALLBACK=1`` opts out, for debugging only).
"""
import ctypes
import importlib
import os
import threading

_lock = threading.Lock()
_engine = None
_hip = None


def engine():
    global _engine
    if _engine is not None:
        return _engine
    with _lock:
        if _engine is None:
            from . import _build
            try:
                _build.build_engine()
            except Exception:
                # a read-only checkout with a prebuilt module is fine
                if not os.path.exists(_build.ENGINE_SO):
                    raise
            _engine = importlib.import_module("rocalphago_amd._rocgo")
    return _engine


def hip_library_path():
    from . import _build
    return _build.HIP_SO


def hip(required=True):
    """ctypes handle to _hipkernels.so (built for gfx950)."""
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            from . import _build
            # RAG_HIP_SO: an alternative build of the kernel library (same-box A/B of two
            # source revisions, tools/ab_build.py)
            path = os.environ.get("RAG_HIP_SO") or _build.HIP_SO
            if not os.path.exists(path):
                try:
                    _build.build_hip()
                except Exception:
                    if required:
                        raise
                    return None
            _hip = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            from .ops import _abi
            _abi.declare(_hip)
    return _hip


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def torch_fallback_allowed():
    return os.environ.get("RAG_ALLOW_TORCH_FALLBACK", "0") == "1"
