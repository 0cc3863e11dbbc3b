"""The opt-in learner options (xh_config.adv_normalize / lr_scale_rows), off
in the reference configuration, against the oracle with the same options on
(or_trainer_set_options).  The reference normalises no advantages
(policy_gradient.h:220-281) and applies the raw lr to row sums (nn.h:94-98,
624), so these checks are oracle-pinned only ("parity unpinned" against the
reference itself, which has no such option).  Tolerance: conftest.RTOL."""
import numpy as np
import pytest

from conftest import assert_close

pytestmark = pytest.mark.gpu


def _pair(ctx, algo, B, D, N, T, widths, adv_normalize, lr_scale_rows, x0):
    from oracle import pyoracle as po
    from dependence_free_rl_amd import (POLICY, VALUE, Trainer, init_policy,
                                        init_value)
    pp = init_policy(D, *widths, seed=3)
    vp = init_value(B, D, seed=4)
    tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                 widths=widths, rng_state=x0, adv_normalize=adv_normalize,
                 lr_scale_rows=lr_scale_rows, wd_policy=0.0)
    tr.set_params(POLICY, pp)
    tr.set_params(VALUE, vp)
    head = po.OR_SOFTMAX if algo == "ppo" else po.OR_SOFTMAX_XENT
    lr = (1e-4, 1e-5) if algo == "ppo" else (1e-5, 1e-4)
    orc = po.Trainer(po.OR_PPO if algo == "ppo" else po.OR_AC, B, D, N, T,
                     po.perbin_model(2 * D, list(widths), head), pp,
                     po.full_model(B * 2 * D, [64, 32], 1), vp,
                     lr_pi=lr[0], lr_v=lr[1], x0=x0)
    orc.set_options(adv_normalize, lr_scale_rows)
    return tr, orc


@pytest.mark.parametrize("algo,B,D,N,T,widths", [
    ("ppo", 8, 2, 16, 4, (128, 64)),
    ("ppo", 64, 2, 16, 4, (128, 128)),
    ("ac", 8, 2, 16, 8, (64, 32)),
])
@pytest.mark.parametrize("adv_norm,lr_rows", [(1, 0), (0, 1), (1, 1)])
def test_options_match_oracle(ctx, algo, B, D, N, T, widths, adv_norm, lr_rows):
    from oracle import pyoracle as po
    from dependence_free_rl_amd.trainer import BUF_ACTION, BUF_ADV, POLICY, VALUE
    tr, orc = _pair(ctx, algo, B, D, N, T, widths, adv_norm, lr_rows, 777)
    for it in range(2):
        tr.rollout()
        orc.rollout()
        np.testing.assert_array_equal(
            tr.buffer(BUF_ACTION), orc.buf(po.BUF_STEP_CHOICE).reshape(N, T).T)
        tr.learn()
        orc.learn()
        # advantages of the transition rows, mapped to the device's [T][N]
        adv = orc.buf(po.BUF_ADVANTAGES)
        env = orc.buf(po.BUF_ROW_ENV)
        step = orc.buf(po.BUF_ROW_STEP) - it * T
        end = orc.buf(po.BUF_ROW_IS_END)
        want = np.zeros((T, N), np.float32)
        for k in np.nonzero(end == 0)[0]:
            want[step[k], env[k]] = adv[k]
        got = tr.buffer(BUF_ADV)
        assert_close(got, want, what="advantages it%d" % it)
        if adv_norm:  # normalised over the T*N transitions
            assert abs(float(got.mean())) < 1e-3
            assert abs(float(got.std()) - 1.0) < 1e-3
        assert_close(tr.params(VALUE), orc.params(1), what="value params")
        assert_close(tr.params(POLICY), orc.params(0), what="policy params")


def test_options_off_is_reference(ctx):
    """Both options off (the default) is the reference learner: the same
    parameters as a trainer built without naming them."""
    from dependence_free_rl_amd import (POLICY, Trainer, init_policy,
                                        init_value)
    from dependence_free_rl_amd.trainer import VALUE
    outs = []
    for kw in ({}, {"adv_normalize": False, "lr_scale_rows": False}):
        tr = Trainer(ctx, bins=8, dims=2, num_envs=16, steps=4,
                     widths=(128, 64), rng_state=5, **kw)
        tr.set_params(POLICY, init_policy(2, 128, 64, seed=1))
        tr.set_params(VALUE, init_value(8, 2, seed=2))
        tr.iterate(2)
        outs.append(tr.params(POLICY))
        tr.close()
    np.testing.assert_array_equal(outs[0], outs[1])
