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


# Row-summed gradients under cancellation.  A gradient entry is a sum over
# the batch rows (nn.h:94-98), and a policy-gradient entry cancels heavily
# (softmax Jacobian rows sum to zero), so |sum| can be ~1e-3 of the sum of
# |terms|.  Any fp32 evaluation order of n terms is within (n - 1) u
# sum|terms| of the exact sum (recursive-summation bound; + u per product for
# the terms' own rounding), u = 2^-24.  The oracle accumulates in double
# (sides = 1); the reference's own fp32 sums carry the same bound again
# (sides = 2).  Rule: |x - y| <= 1e-4 max(1, |y|) + sides (n + 8) u mag, with
# mag = sum|terms| per entry from or_model_grad_mag.
U32 = 2.0 ** -24


def assert_grad_close(x, y, mag, n_terms, sides=1, what=""):
    x = np.asarray(x, np.float64).ravel()
    y = np.asarray(y, np.float64).ravel()
    mag = np.asarray(mag, np.float64).ravel()
    assert x.shape == y.shape == mag.shape, (what, x.shape, y.shape, mag.shape)
    bound = RTOL * np.maximum(1.0, np.abs(y)) + sides * (n_terms + 8) * U32 * mag
    err = np.abs(x - y)
    if err.size:
        i = int(np.argmax(err / bound))
        assert err[i] <= bound[i], (
            "%s: err %.3g > bound %.3g at %d (x=%r y=%r mag=%.3g)" % (
                what, err[i], bound[i], i, x[i], y[i], mag[i]))
    return float((err / bound).max()) if err.size else 0.0


# adam_optimizer (nn.h:677-690) divides each gradient entry by its own running
# RMS, so an entry whose gradient is fp32 rounding noise (a sum that cancels to
# ~1e-7 of the gradient's largest entry) takes a step of up to lr with an
# arbitrary sign -- the reference's own builds disagree on such entries.  Rule:
# entries whose gradient was at noise level (|g| <= NOISE_REL * max|g|) in any
# adam step so far may differ by 2 * lr * steps; every other entry keeps the
# 1e-4 parity tolerance.
NOISE_REL = 1e-5


def noise_mask(grads, mask=None):
    """Update the cumulative noise mask with gradients [steps][n]."""
    g = np.abs(np.asarray(grads, np.float64)).reshape(-1, np.shape(grads)[-1])
    m = (g <= NOISE_REL * g.max(axis=1, keepdims=True)).any(axis=0)
    return m if mask is None else (mask | m)


def assert_params_close(x, y, mask=None, slack=0.0, what=""):
    """assert_close, except entries under `mask` may differ by `slack`."""
    if mask is None or not mask.any():
        return assert_close(x, y, what=what)
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    assert np.all(np.abs(x[mask] - y[mask]) <= slack + 1e-6), (
        what, "noise-level entries beyond 2*lr*steps",
        float(np.abs(x[mask] - y[mask]).max()), slack)
    return assert_close(x[~mask], y[~mask], what=what)


@pytest.fixture(scope="module")
def ctx():
    """One device context per test module.  No torch in the process: torch
    bundles its own libamdhip64 / librccl under the same sonames, and a
    process that loaded them first would make libxylo_hip bind those instead
    of /opt/rocm's (the runtime the bench measures on)."""
    from dependence_free_rl_amd import Context, runtime_info
    assert "torch" not in sys.modules, "GPU tests must not import torch"
    info = runtime_info()
    for key in ("libamdhip64", "librccl"):
        assert "/torch/" not in info[key], info
    c = Context(device=0)
    yield c
    c.close()
