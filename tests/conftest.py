"""pytest configuration: repo root on sys.path, the `gpu` marker, shared fixtures."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The reference's own fixtures (SGF games, minimodel.json, Keras HDF5 files) are read in place,
# never copied: compatibility tests that need them skip when the reference is not mounted.
REFERENCE_DATA = os.environ.get("RAG_REFERENCE_DATA", "/root/reference/tests/test_data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels, RCCL)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def ref_data():
    if not os.path.isdir(REFERENCE_DATA):
        pytest.skip("reference test data not mounted")
    return REFERENCE_DATA


@pytest.fixture
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
