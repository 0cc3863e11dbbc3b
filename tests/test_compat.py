"""The drop-in C++20 layer (include/xylo_compat) on the CPU: the reference's
unmodified apps/bin_packing drivers compile against it; its model
initialisation, env construction and host-policy agents reproduce the real
reference bit for bit (golden fixtures from oracle/_ref/ref_harness)."""
import os
import subprocess

import numpy as np
import pytest

from compat_helpers import (CXX, FLAGS, REPO, app, compile_cc, fmt6,
                            read_rounds)
from conftest import golden

REF_APPS = ["ppo_training", "ac_training", "ppo2_training", "pg_training",
            "deep_agent", "random_agent", "firstfit_agent", "bestfit_agent",
            "minwaste_agent"]
REF = "/root/reference/apps/bin_packing"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent")
@pytest.mark.parametrize("name", REF_APPS)
def test_reference_app_compiles_unmodified(name):
    """same names, namespaces and signatures."""
    r = subprocess.run([CXX] + FLAGS + ["-fsyntax-only",
                                        "-Wno-logical-op-parentheses",
                                        os.path.join(REF, name + ".cc")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("algo", ["ppo", "ac"])
def test_driver_prologue_matches_reference(tmp_path, algo):
    """Seeded model init (he / normal draws from the global engine) and the
    workers' env construction equal the reference's (driver_*_s7 fixtures)."""
    exe = compile_cc(os.path.join(REPO, "tests", "compat", "driver_prologue.cc"),
                     str(tmp_path / "prologue"))
    out = tmp_path / "params.bin"
    env = dict(os.environ, XYLO_SEED="7")
    r = subprocess.run([exe, algo, str(out)], capture_output=True, text=True,
                       env=env, check=True)
    g = golden("driver_%s_s7" % algo)
    p = np.fromfile(out, np.float32)
    npol = g["policy_init"].size
    np.testing.assert_array_equal(p[:npol], g["policy_init"])
    np.testing.assert_array_equal(p[npol:], g["value_init"])
    f = [int(v) for v in r.stdout.split()]
    assert f[0] == int(g["x_models"][0]) and f[1] == int(g["x_envs"][0])
    np.testing.assert_array_equal(f[2:], g["items"])


@pytest.mark.skipif(not os.path.exists(app("random_agent")),
                    reason="build/compat/random_agent not built (make compat)")
def test_random_agent_matches_reference():
    """random_agent.cc unmodified, host policy + host env: per-round averages
    equal the reference's for the same seed (random_s5 fixture)."""
    env = dict(os.environ, XYLO_SEED="5")
    got, text = read_rounds([app("random_agent")], 3, env, timeout=60)
    want = golden("random_s5")["round_avg"]
    assert [k for k, _ in got] == [0, 1, 2], text[-500:]
    assert [x for _, x in got] == [fmt6(float(w)) for w in want]


def test_save_parameters_round_trip_cpu(tmp_path):
    """xylo::save_parameters -> raw float32 file -> mmap<float> +
    model::set_parameters (deep_agent.cc's loader) is the identity, bit for
    bit (no device involved)."""
    import subprocess
    from compat_helpers import app
    from conftest import golden
    if not os.path.exists(app("save_weights")):
        pytest.skip("build/compat/save_weights not built (make compat)")
    w = golden("deep_w20")["params"].astype("float32")
    src = tmp_path / "w.in"
    w.tofile(src)
    out = subprocess.run([app("save_weights"), "copy", str(src),
                          str(tmp_path / "w.out")], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.split() == ["equal", str(w.size)]
    assert (tmp_path / "w.out").read_bytes() == src.read_bytes()
