"""The drop-in xylo/tensor.h on the device.

* tests/compat/tensor_ops.cc (the reference's tensor API only; its reference
  build is tests/golden/tensor_ops.npz): with the default thresholds the
  large GEMMs (>= 2^22 multiply-adds) and reductions (>= 2^20 floats) of its
  host tensors run on the device; with XYLO_HIP_DEVICE_MIN=0 every GEMM,
  transpose and reduction does.  Integers, shapes, flags and engine draws
  bit-exact against the reference, floats within 1e-4 max(1, |y|).
* tests/compat/tensor_device.cc: tensors created with on_device = true (HBM)
  -- elementwise maps, compound operators, reductions, GEMMs, transposes,
  fills, views, equality, the engine's draws -- against the same operations
  on host tensors of the same values."""
import os
import subprocess

import pytest

from compat_helpers import app, tensor_ops_mismatches

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("device_min", [None, "0"])
def test_tensor_ops_match_the_reference(device_min):
    env = dict(os.environ)
    env.pop("XYLO_HIP_DEVICE_MIN", None)
    if device_min is not None:
        env["XYLO_HIP_DEVICE_MIN"] = device_min
    out = subprocess.run([app("tensor_ops")], capture_output=True, text=True,
                         timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    bad, worst = tensor_ops_mismatches(out.stdout)
    print("device_min %s: worst float error %.3g x max(1, |y|)" % (device_min, worst))
    assert not bad, bad[:10]


def test_device_tensors_match_host_tensors():
    out = subprocess.run([app("tensor_device")], capture_output=True, text=True,
                         timeout=120)
    fails = [l for l in out.stdout.splitlines() if l.startswith("FAIL")]
    print("\n".join(out.stdout.splitlines()[-5:]))
    assert out.returncode == 0 and not fails, (fails[:10], out.stderr[-2000:])
    assert "tensor_device ok" in out.stdout


@pytest.mark.parametrize("case", ["all_neg_inf", "all_nan", "nan_first",
                                  "nan_mixed", "neg_inf_then_max"])
def test_device_max_argmax_follow_max_element(case):
    """xh_tensor_reduce's max / argmax above the device threshold (2^20
    floats) on the inputs where a parallel max differs from std::max_element
    (tensor.h's host path, the reference's tensor.cc:462-466): an all -inf
    vector (index 0), an all-NaN vector (index 0, value NaN), a NaN at index 0
    (max_element never leaves it), NaNs elsewhere (never chosen), the first
    of equal maxima."""
    import ctypes as C

    import numpy as np

    from dependence_free_rl_amd import _lib
    from dependence_free_rl_amd.trainer import Context

    n = (1 << 20) + 4099
    rng = np.random.default_rng(5)
    if case == "all_neg_inf":
        a = np.full(n, -np.inf, np.float32)
    elif case == "all_nan":
        a = np.full(n, np.nan, np.float32)
    elif case == "nan_first":
        a = rng.standard_normal(n).astype(np.float32)
        a[0] = np.nan
    elif case == "nan_mixed":
        a = rng.standard_normal(n).astype(np.float32)
        a[rng.integers(1, n, 5000)] = np.nan
    else:
        a = np.full(n, -np.inf, np.float32)
        a[[70000, 900001, 1000003]] = 3.5
    # std::max_element's scan, restated
    want = 0
    for i in np.flatnonzero(~np.isnan(a)) if not np.isnan(a[0]) else []:
        if a[want] < a[i]:
            want = int(i)
    ctx = Context(0)
    try:
        for op in (3, 4):  # XH_R_MAX, XH_R_ARGMAX
            v, idx = C.c_double(), C.c_int64(-1)
            _lib.check(_lib.lib.xh_tensor_reduce(
                ctx.h, op, a.ctypes.data, None, 0.0, n, 0, C.byref(v),
                C.byref(idx)))
            assert idx.value == want, (case, op, idx.value, want)
            if np.isnan(a[want]):
                assert np.isnan(v.value)
            else:
                assert v.value == float(a[want]), (case, v.value)
    finally:
        ctx.close()
