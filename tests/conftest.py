import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
_LIB = os.path.join(ROOT, "fakepta_amd", "lib", "libfakepta_amd.so")
if not os.path.exists(_LIB):  # the package refuses to import without its HIP library: build it (hipcc, no GPU)
    import subprocess
    subprocess.run(["make", "-C", os.path.join(ROOT, "fakepta_amd", "csrc")], check=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running statistical test")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        path = os.path.join(GOLDEN, name)
        if name.endswith(".npz"):
            return dict(np.load(path, allow_pickle=False))
        import json
        with open(path) as fh:
            return json.load(fh)
    return load


def rel_err(a, b):
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    den = np.linalg.norm(b.ravel())
    return np.linalg.norm((a - b).ravel()) / (den if den > 0 else 1.0)


def assert_parity(a, b, tol=1e-10):
    """SURVEY.md §8(c) tolerance: ||y - y_ref|| / ||y_ref|| <= tol and max-abs <= tol * max|y_ref|."""
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert rel_err(a, b) <= tol, rel_err(a, b)
    scale = np.max(np.abs(b)) if b.size else 0.0
    assert np.max(np.abs(a - b), initial=0.0) <= tol * max(scale, 1e-300)
