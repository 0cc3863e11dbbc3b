"""bench.py's contract pieces that need no GPU: the workload table follows
BASELINE.json's configs and SURVEY §8d's algorithmic FLOP / byte counts; a
GPU run of the JSON line itself is in test_gpu_scale.py."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


@pytest.fixture
def bench():
    import bench as b
    yield b
    b.select_config(3)  # module globals back to the headline config


def test_headline_is_config3(bench):
    k = bench.select_config(3)
    assert (bench.ALGO, bench.B, bench.D, bench.T, bench.H1, bench.H2) == (
        "ppo", 64, 2, 4, 128, 128)
    assert k["N"] == 32768 and bench.EPOCHS == 4


def test_flops_match_survey_8d(bench):
    bench.select_config(3)
    fp = bench.policy_fwd_flops_per_env_step()
    fv = bench.value_fwd_flops_per_row()
    assert fp == 2 * 64 * (4 * 128 + 128 * 128 + 128)
    # PPO = 13 Fp + 5 Fv = 28.51 MFLOP per env-step at C3
    assert abs((13 * fp + 5 * fv) / 1e6 - 28.51) < 0.01
    bench.select_config(5)
    fp5 = bench.policy_fwd_flops_per_env_step()
    fv5 = bench.value_fwd_flops_per_row()
    # AC: 4 Fp + 5 Fv = 18.21 MFLOP at C5
    assert abs((4 * fp5 + 5 * fv5) / 1e6 - 18.21) < 0.01
    bench.select_config(2)
    fp2 = bench.policy_fwd_flops_per_env_step()
    fv2 = bench.value_fwd_flops_per_row()
    assert abs((13 * fp2 + 5 * fv2) / 1e6 - 3.63) < 0.01


def test_pmc_traffic_only_for_the_same_shape(bench):
    bench.select_config(3)
    sha = bench.library_sha256()
    t, src, _ = bench.pmc_traffic(lib_sha=sha)
    if t is not None:  # a committed summary of this build at the 64-bin shape
        assert src.startswith("profiles/") and t > 0
    bench.select_config(5)
    t5, _, _ = bench.pmc_traffic(lib_sha=sha)
    # never the 64-bin kernel's counters for the 128-bin shape
    assert t5 is None or t5 != t


def test_pmc_traffic_only_for_this_library_build(bench, tmp_path, monkeypatch):
    """A PMC summary is cited only when its recorded library sha256 is the
    loaded library's: another build's summary (or one without the record)
    gives traffic None, whatever its file name."""
    import json
    bench.select_config(3)
    prof = tmp_path / "profiles"
    prof.mkdir()
    entry = {"kernel": "void xh::policy_train8_kernel<xh::PShape<64, 2, 128, 128>>()",
             "hbm_bytes": 123.0}
    for name, meta in (("r99z_c3", {"library_sha256": "0" * 64,
                                    "created": "2099-01-01T00:00:00+00:00"}),
                       ("r99y_c3", None)):
        summ = {"policy_train8_kernel": entry}
        if meta:
            summ["_meta"] = meta
        (prof / ("%s_pmc_summary.json" % name)).write_text(json.dumps(summ))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.pmc_traffic(lib_sha="f" * 64) == (None, None, None)
    summ = {"policy_train8_kernel": dict(entry, hbm_bytes=7.0),
            "_meta": {"library_sha256": "f" * 64,
                      "created": "2026-01-01T00:00:00+00:00"}}
    (prof / "r00a_c3_pmc_summary.json").write_text(json.dumps(summ))
    t, src, _ = bench.pmc_traffic(lib_sha="f" * 64)
    assert t == 7.0 and src == "profiles/r00a_c3_pmc_summary.json"


def test_roofline_math_comes_from_the_library(bench):
    """The train kernel's name, arithmetic and peak in the bench line are
    what xh_trainer_kernel_info reported; bench.py does not re-derive the
    kernel selection."""
    k = {"kernel": "policy_train_split_kernel", "math": "bf16_split",
         "bf16_products_per_f32_product": 4, "peak_tflops": 625.0}
    r = bench.kernel_roofline(k, 857e9, 2.0)
    assert r["kernel"] == k["kernel"] and r["math"] == "bf16_split"
    assert r["math_source"] == "xh_trainer_kernel_info" and r["peak"] == 625.0
    assert abs(r["achieved"] - 428.5) < 1e-6 and abs(r["frac"] - 0.6856) < 1e-4
    k2 = dict(k, math="f32_mfma", bf16_products_per_f32_product=None,
              peak_tflops=157.3)
    assert bench.kernel_roofline(k2, 857e9, 2.0)["peak"] == 157.3
    src = open(os.path.join(REPO, "bench.py")).read()
    assert "kernel_info()" in src and "train_split_active" not in src


@pytest.mark.parametrize("var", ["XH_TRAIN_KERNEL", "XH_ROLLOUT_KERNEL",
                                 "XH_VALUE_KERNEL"])
def test_bench_refuses_kernel_overrides(var):
    """A kernel-selection override in the environment stops the bench before
    it touches the device, unless --allow-kernel-override is given."""
    import subprocess
    env = dict(os.environ, **{var: "f32"})
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"),
                          "--steps", "1", "--warmup", "0"],
                         capture_output=True, text=True, env=env, timeout=60)
    assert out.returncode == 2 and var in out.stderr, (out.returncode, out.stderr)
    assert out.stdout.strip() == ""


def test_pmc_traffic_skips_another_env_count(bench, tmp_path, monkeypatch):
    """A summary that records its run's env count (the env-only and 1M-env
    trainer profiles) is cited only for that count: the 1M-env profile of
    the config-3 train kernel must not give the 32768-env line its bytes."""
    import json
    bench.select_config(3)
    prof = tmp_path / "profiles"
    prof.mkdir()
    k = "policy_train_spec8_kernel"
    for name, meta, b in (("r99a_c3", {}, 5.0),
                          ("r99b_c3_env1m", {"envs": 1048576,
                                             "workload": "config3_trainer"}, 9.0)):
        m = dict(meta, library_sha256="f" * 64, created="2026-01-0%dT00:00:00+00:00"
                 % (1 if b == 5.0 else 2))
        summ = {k: {"kernel": "xh::sp8::" + k + "(xh::PolicyTrainArgs)", "hbm_bytes": b},
                "_meta": m}
        (prof / ("%s_pmc_summary.json" % name)).write_text(json.dumps(summ))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    t, src, _ = bench.pmc_traffic(k, any_shape=True, lib_sha="f" * 64, envs=32768)
    assert t == 5.0 and src == "profiles/r99a_c3_pmc_summary.json"
    t, _, _ = bench.pmc_traffic(k, any_shape=True, lib_sha="f" * 64, envs=1048576)
    assert t == 9.0
