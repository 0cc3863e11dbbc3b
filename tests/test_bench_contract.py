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
    t, src, _ = bench.pmc_traffic()
    if t is not None:  # a committed summary of the 64-bin shape
        assert src.startswith("profiles/") and t > 0
    bench.select_config(5)
    t5, _, _ = bench.pmc_traffic()
    # never the 64-bin kernel's counters for the 128-bin shape
    assert t5 is None or t5 != t
