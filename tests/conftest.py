import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rollout-bayesian-optimization_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmrbo.so on cuda:0)")


@pytest.fixture(scope="session")
def oracle():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    from oracle import oracle as O
    return O


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, f"golden_{name}.npz"))
    return {k: z[k] for k in z.files}


GOLDEN_CASES = ["c1", "c2", "c2cap", "c2near", "c3"]


@pytest.fixture(scope="session")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from mrbo import _lib
    _lib.load()
    return torch
