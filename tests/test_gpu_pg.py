"""REINFORCE (policy_gradient_learner, policy_gradient.h:88-147) on the GPU
through the C ABI, against the real reference's golden vectors (one env: the
reference's single engine stream) and against the CPU oracle with several envs
on independent streams (env g = the stream advanced by g * 2^26 draws).

Bit-exact: states, items, actions, dones, episode lengths, engine states.
Within 1e-4 * max(1, |y|): advantages, the policy gradient, parameters.
"""
import numpy as np
import pytest

from conftest import assert_close, golden
from gpu_helpers import meta

pytestmark = pytest.mark.gpu



def pg_trainer(ctx, B, D, N, E, widths, x0, params):
    from dependence_free_rl_amd import POLICY, Trainer
    w = tuple(widths) + (0,) * (2 - len(widths))
    tr = Trainer(ctx, algo="pg", bins=B, dims=D, num_envs=N, steps=E,
                 widths=w, rng_state=x0, gamma=0.99)
    tr.set_params(POLICY, params)
    return tr


def env_rows(tr, e):
    """Env e's transitions of the last rollout (step order)."""
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_BINS, BUF_DONE,
                                                BUF_ITEMS, BUF_LEN)
    L = int(tr.buffer(BUF_LEN)[e])
    return (L, tr.buffer(BUF_BINS)[:L, e], tr.buffer(BUF_ITEMS)[:L, e, :tr.D],
            tr.buffer(BUF_ACTION)[:L, e], tr.buffer(BUF_DONE)[:L, e])


@pytest.mark.parametrize("name", ["pg_b8d1", "pg_b8d2"])
def test_pg_matches_reference(ctx, name):
    """pg_learner with one worker: every episode step, the reversed
    rewards-to-go advantages, the gradient and the new parameters."""
    from dependence_free_rl_amd.trainer import (BUF_ADV, BUF_POLICY_GRADS,
                                                BUF_RNG, POLICY)
    g = golden(name)
    kv = meta(g)
    B, D, E = int(kv["B"]), int(kv["D"]), int(kv["episodes"])
    widths = [int(w) for w in kv["widths"].split(",")]
    tr = pg_trainer(ctx, B, D, 1, E, widths, int(g["x0"][0]), g["init_policy"])
    for it in range(int(kv["iters"])):
        p = "it%d_" % it
        tr.rollout()
        L, bins, items, act, done = env_rows(tr, 0)
        assert L == len(g[p + "step_choice"])
        np.testing.assert_array_equal(bins, g[p + "step_bins"])
        np.testing.assert_array_equal(items, g[p + "step_item"])
        np.testing.assert_array_equal(act, g[p + "step_choice"])
        np.testing.assert_array_equal(done, g[p + "step_done"])
        assert int(tr.buffer(BUF_RNG)[0]) == int(g[p + "x_end"][0])
        tr.learn()
        assert_close(tr.buffer(BUF_ADV)[:L, 0], g[p + "advantages"],
                     what=p + "advantages")
        assert_close(tr.buffer(BUF_POLICY_GRADS)[0], g[p + "policy_grads"][0],
                     what=p + "policy_grads")
        assert_close(tr.params(POLICY), g[p + "policy_params"],
                     what=p + "policy_params")


@pytest.mark.parametrize("B,D,N,E,widths", [(8, 2, 6, 2, (64, 32)),
                                            (16, 1, 5, 3, (48,))])
def test_pg_many_envs_vs_oracle(ctx, B, D, N, E, widths):
    """Several envs on independent streams, 3 iterations: per-env
    trajectories bit-exact, baseline over all trajectories, gradient and
    parameters within tolerance of the oracle."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd import init_full_policy
    from dependence_free_rl_amd.trainer import BUF_POLICY_GRADS, BUF_RNG, POLICY
    x0 = 987654
    p0 = init_full_policy(B, D, widths, seed=3)
    tr = pg_trainer(ctx, B, D, N, E, widths, x0, p0)
    orc = po.Trainer(po.OR_PG, B, D, N, 1,
                     po.full_model(B * 2 * D, list(widths), B, po.OR_SOFTMAX_XENT),
                     p0, x0=x0, episodes=E)
    orc.set_env_streams(1 << 26)
    for it in range(3):
        tr.rollout()
        orc.rollout()
        s_bins = orc.buf(po.BUF_STEP_BINS).reshape(-1, B, D)
        s_choice = orc.buf(po.BUF_STEP_CHOICE)
        s_done = orc.buf(po.BUF_STEP_DONE)
        k = 0
        for e in range(N):
            L, bins, items, act, done = env_rows(tr, e)
            np.testing.assert_array_equal(bins, s_bins[k:k + L])
            np.testing.assert_array_equal(act, s_choice[k:k + L])
            np.testing.assert_array_equal(done, s_done[k:k + L])
            assert done.sum() == E and done[-1] == 1
            k += L
        assert k == len(s_choice)
        np.testing.assert_array_equal(tr.buffer(BUF_RNG), orc.env_streams())
        tr.learn()
        orc.learn()
        assert_close(tr.buffer(BUF_POLICY_GRADS)[0],
                     orc.buf(po.BUF_POLICY_GRADS), what="policy_grads")
        assert_close(tr.params(POLICY), orc.params(0), what="policy_params")
