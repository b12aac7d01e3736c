"""The in-tree HIP library resolves every one of its own symbols (a declared-but-undefined
launcher links fine into a shared object and only fails when ctypes loads it on the GPU box)."""
import os
import shutil
import subprocess

import pytest

SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rocalphago_amd",
                  "_hipkernels.so")


@pytest.mark.skipif(not os.path.exists(SO) or shutil.which("nm") is None,
                    reason="HIP library not built here")
def test_hip_library_has_no_undefined_own_symbols():
    out = subprocess.run(["nm", "-D", "--undefined-only", SO], stdout=subprocess.PIPE,
                         text=True, check=True).stdout
    # strong undefined symbols of our own code: launchers (rag_*) and anything in an anonymous
    # namespace (_GLOBAL__N_), e.g. an extern declared inside one
    own = [ln for ln in out.splitlines()
           if ("rag_" in ln or "_GLOBAL__N_" in ln) and not ln.strip().startswith("w ")]
    assert not own, own


@pytest.mark.skipif(not os.path.exists(SO), reason="HIP library not built here")
def test_hip_library_loads_with_every_symbol_bound():
    """dlopen with RTLD_NOW (what the GPU box's ctypes load does) binds every reference."""
    import ctypes
    ctypes.CDLL(SO, mode=os.RTLD_NOW | os.RTLD_LOCAL)
