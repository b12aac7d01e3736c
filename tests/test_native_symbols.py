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
    own = [ln for ln in out.splitlines() if "rag_" in ln]
    assert not own, own
