import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")

# Parity tolerance for floating-point quantities (BASELINE.json north_star:
# "loss parity to CPU ref within 1e-4"): |x - y| <= 1e-4 * max(1, |y|).
RTOL = 1e-4


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU cases")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def assert_close(x, y, tol=RTOL, what=""):
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    assert x.shape == y.shape, (what, x.shape, y.shape)
    err = np.abs(x - y) / np.maximum(1.0, np.abs(y))
    if err.size:
        i = int(np.argmax(err))
        assert err.flat[i] <= tol, (
            "%s: max scaled err %.3g at %d (x=%r y=%r)" % (what, err.flat[i], i,
                                                          x.flat[i], y.flat[i]))
    return float(err.max()) if err.size else 0.0
