"""The wave-specialised config-2 train kernel (policy_train_spec4_kernel,
dependence_free_rl_amd/csrc/policy_spec4_kernels.hip; opt-in by
XH_TRAIN_KERNEL=spec4, read per launch) against the oracle and against the
default config-2 kernel (policy_train_split4h_kernel) on the same batch.

Reference: ppo_learner::optimize_action / actor_critic_learner's policy step
(policy_gradient.h:196-307) on the per-bin [64,64] policy, 32 bins, 1-D.
Group counts and grids chosen for the pipeline's edges: one group per
workgroup, a grid that is not a multiple of 8 (plain order, unequal J), odd
J, and one workgroup running every group (J = 96).  PPO and actor-critic.
"""
import os

import numpy as np
import pytest

from conftest import (GRAD_UNITS_P99_DRIFT, assert_close, assert_grad_close,
                      assert_grad_units, grad_units)

pytestmark = pytest.mark.gpu

N, T, B, D, WIDTHS = 48, 4, 32, 1, (64, 64)  # 96 two-env 64-row groups


def _oracle(algo, pp, vp, x0):
    from oracle import pyoracle as po
    head = po.OR_SOFTMAX_XENT if algo == "ac" else po.OR_SOFTMAX
    return po.Trainer({"ppo": po.OR_PPO, "ac": po.OR_AC}[algo], B, D, N, T,
                      po.perbin_model(2 * D, list(WIDTHS), head), pp,
                      po.full_model(B * 2 * D, [64, 32], 1), vp,
                      lr_pi=1e-5 if algo == "ac" else 1e-4,
                      lr_v=1e-4 if algo == "ac" else 1e-5, x0=x0)


def _run(ctx, algo, pp, vp, x0, cap, kernel_env):
    from dependence_free_rl_amd import POLICY, VALUE, Trainer
    from dependence_free_rl_amd.trainer import BUF_POLICY_GRADS, BUF_VALUE_GRAD
    old = os.environ.get("XH_TRAIN_KERNEL")
    if kernel_env:
        os.environ["XH_TRAIN_KERNEL"] = kernel_env
    try:
        tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                     widths=WIDTHS, rng_state=x0, train_grid_cap=cap)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        tr.rollout()
        tr.learn()
        info = tr.kernel_info()
        npi = tr.num_params(POLICY)
        g = tr.buffer(BUF_POLICY_GRADS).reshape(-1, npi).copy()
        v = tr.buffer(BUF_VALUE_GRAD).copy()
        tr.close()
    finally:
        if old is None:
            os.environ.pop("XH_TRAIN_KERNEL", None)
        else:
            os.environ["XH_TRAIN_KERNEL"] = old
    return info, g, v


@pytest.mark.parametrize("algo", ["ppo", "ac"])
@pytest.mark.parametrize("cap", [0, 5, 1])
def test_spec4_vs_oracle_and_split4h(ctx, algo, cap):
    from oracle import pyoracle as po
    from dependence_free_rl_amd import init_policy, init_value
    x0 = 4242 + cap
    pp = init_policy(D, *WIDTHS, seed=71)
    vp = init_value(B, D, seed=72)
    orc = _oracle(algo, pp, vp, x0)
    orc.rollout()
    orc.learn()
    ref = np.asarray(orc.buf(po.BUF_POLICY_GRADS))
    mag = np.asarray(orc.buf(po.BUF_POLICY_GRADS_MAG))
    rows = len(orc.buf(po.BUF_ROW_ENV))
    info, g, v = _run(ctx, algo, pp, vp, x0, cap, "spec4")
    assert info["policy_train"]["kernel"] == "policy_train_spec4_kernel", info
    grid = info["train_grid"]
    groups = N * T // 2
    assert grid == (min(cap, groups) if cap else min(groups, grid)), (cap, grid)
    J = -(-groups // grid)
    info_o, g_o, v_o = _run(ctx, algo, pp, vp, x0, cap, None)
    assert info_o["policy_train"]["kernel"] == "policy_train_split4h_kernel", info_o
    assert_close(v, orc.buf(po.BUF_VALUE_GRAD), what="value_grad")
    npi = g.shape[1]
    r, m = ref.reshape(-1, npi), mag.reshape(-1, npi)
    assert_grad_close(g.ravel(), ref, mag, n_terms=rows * B,
                      what="spec4 %s grid=%d" % (algo, grid))
    for ep in range(g.shape[0]):
        budget = {} if ep == 0 else {"p99_units": GRAD_UNITS_P99_DRIFT}
        assert_grad_units(g[ep], r[ep], m[ep],
                          what="spec4 %s B%d D%d N%d T%d grid=%d J=%d epoch%d"
                               % (algo, B, D, N, T, grid, J, ep), **budget)
    # epoch 0 against the default kernel on the same inputs: p99 within 2x + 2
    u_new, _, _ = grad_units(g[0], r[0], m[0])
    u_old, _, _ = grad_units(g_o[0], r[0], m[0])
    p_new, p_old = float(np.percentile(u_new, 99)), float(np.percentile(u_old, 99))
    print("spec4 vs split4h %s grid=%d J=%d: p99 units %.3g vs %.3g" % (
        algo, grid, J, p_new, p_old))
    assert p_new <= 2.0 * p_old + 2.0, (p_new, p_old)
