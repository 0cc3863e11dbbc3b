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
