import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsme.so on the device)")


@pytest.fixture(scope="session")
def sme():
    import importlib
    return importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd")


@pytest.fixture(scope="session")
def synth():
    import importlib
    return importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd.synth")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first():
    """On a GPU box, torch's bundled HIP runtime opens the device before libsme's
    (measured: torch's lazy CUDA init fails with "No HIP GPUs are available" once
    libsme's runtime holds the device), so tests that mix torch tensors with
    libsme calls work in any order.  No-op without a GPU."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    yield
