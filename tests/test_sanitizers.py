"""SURVEY §5 sanitizer runs (CPU): the C restatement under AddressSanitizer +
UndefinedBehaviorSanitizer (`make -C oracle asan`), driven through every
entry point by oracle/asan_driver.c; any report aborts the run."""
import os
import subprocess

from conftest import REPO

SAN_ENV = {"ASAN_OPTIONS": "halt_on_error=1:detect_leaks=1:abort_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"],
                   check=True, timeout=300)
    out = subprocess.run([os.path.join(REPO, "oracle", "_asan", "oracle_asan")],
                         capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, **SAN_ENV))
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "asan driver ok" in out.stdout
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr
