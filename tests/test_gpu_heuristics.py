"""The reference's heuristic agents as device policies:
against the reference's own agent programs (heur_* fixtures) and against the
oracle's restatement at other shapes.  Bit-exact: totals, episode counts,
engine states."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

KINDS = ["firstfit", "bestfit", "minwaste", "random"]



@pytest.mark.parametrize("kind", KINDS)
def test_heuristic_matches_reference_agent(ctx, kind):
    from dependence_free_rl_amd import heuristic_evaluate
    g = golden("heur_" + kind)
    for r in range(2):
        out = heuristic_evaluate(ctx, kind, 8, 2, 8, 1000, int(g["x_round"][r]),
                                 trace_cap=64)
        assert np.float32(out["totals"][0] / 1000.0) == g["round_avg"][r]
        if r == 0:
            assert out["steps"][0] == int(g["episode_len"].sum())
            assert (out["trace"] >= 0).all() and (out["trace"] < 8).all()


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("B,D", [(64, 2), (32, 1), (16, 3)])
def test_heuristic_vs_oracle(ctx, kind, B, D):
    from oracle import pyoracle as po
    from dependence_free_rl_amd import heuristic_evaluate
    n, ep, x0 = 2 * (64 // B), 40, 4242
    out = heuristic_evaluate(ctx, kind, B, D, n, ep, x0)
    for e in range(n):
        xe = po.minstd_jump(x0, e << 26)
        total, lens, x_end = po.heuristic_eval(B, D, kind, ep, xe)
        assert out["totals"][e] == total, (e, out["totals"][e], total)
        assert out["steps"][e] == lens.sum()
        assert out["rng"][e] == x_end


def test_heuristic_throughput_smoke(ctx):
    """Large batch: every env finishes its episodes; reports the rate."""
    from dependence_free_rl_amd import heuristic_evaluate
    n = 64 * 1024
    out = heuristic_evaluate(ctx, "firstfit", 8, 2, n, 20, 99)
    steps = out["steps"].sum()
    assert (out["steps"] >= 20).all()
    rate = steps / (out["elapsed_ms"] * 1e-3)
    print("firstfit 8x2: %d envs, %.3g env-steps/s" % (n, rate))
    assert np.all(np.abs(out["totals"] / 20 - 25.9) < 8)
