"""The drop-in xylo/tensor.h against the reference's own (CPU).

tests/compat/tensor_ops.cc uses the reference's tensor API only and compiles
unchanged against both: tests/golden/tensor_ops.npz holds the reference
build's results (tests/golden/make_tensor_golden.py).  Here the drop-in
build runs with every operation on the host (XYLO_HIP_DEVICE_MIN above every
size: no device needed), once plainly and once under AddressSanitizer +
UndefinedBehaviorSanitizer; tests/test_gpu_tensor.py runs the
device paths."""
import os
import subprocess

import pytest

from compat_helpers import REPO, app, parse_tensor_ops, tensor_ops_mismatches

HOST_ONLY = {"XYLO_HIP_DEVICE_MIN": str(1 << 60)}


def _run(binary, extra_env=None):
    env = dict(os.environ, **HOST_ONLY, **(extra_env or {}))
    out = subprocess.run([binary], capture_output=True, text=True, timeout=300,
                         env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    return out


def test_tensor_ops_host_paths_match_the_reference():
    out = _run(app("tensor_ops"))
    bad, worst = tensor_ops_mismatches(out.stdout)
    assert not bad, bad[:10]
    print("worst float error %.3g x max(1, |y|)" % worst)


def test_tensor_ops_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", REPO, "build/compat/tensor_ops_asan"],
                   check=True, timeout=600, capture_output=True)
    out = _run(app("tensor_ops_asan"),
               {"ASAN_OPTIONS": "halt_on_error=1:detect_leaks=1:abort_on_error=1",
                "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert "runtime error" not in out.stderr and "Sanitizer" not in out.stderr
    bad, _ = tensor_ops_mismatches(out.stdout)
    assert not bad, bad[:10]


@pytest.mark.skipif(not os.path.exists(os.path.join(REPO, "oracle", "_ref",
                                                    "tensor_ops_ref")),
                    reason="the reference build exists only in the build "
                           "container (make -C oracle ref)")
def test_fixture_is_the_reference_builds_output():
    """tests/golden/tensor_ops.npz is what the reference's build prints now."""
    out = subprocess.run([os.path.join(REPO, "oracle", "_ref", "tensor_ops_ref")],
                         capture_output=True, text=True, timeout=300, check=True)
    bad, worst = tensor_ops_mismatches(out.stdout, tol=0.0)
    assert not bad and worst == 0.0, bad[:10]
    assert len(parse_tensor_ops(out.stdout)) > 150
