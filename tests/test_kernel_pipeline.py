"""Static check of the gfx950 code objects: no compiler-inserted `s_waitcnt vmcnt` in front of an
LDS read in the kernels that keep global_load_lds prefetches in flight across steps (such a
wait drains the staging ring every step; tools/check_drains.py). CPU only (hipcc cross-compile)."""
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.parametrize("src", ["conv_tap.hip", "wgrad_slab.hip", "wgrad.hip", "conv.hip"])
def test_no_staging_drains(src):
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc")
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from check_drains import drains
    bad = {k: v for k, v in drains(os.path.join(ROOT, "csrc", "hip", src)).items() if v}
    assert not bad, bad
