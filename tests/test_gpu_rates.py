"""optimizer::set_rate (nn.h:591) through xh_trainer_set_learning_rate: the
new rate applies from the next learn() and the optimizer state is kept.

sgd: changing the rate equals re-creating the (stateless) optimizer.
adam: the device parameters after two iterations (lr1 for the first 4
steps, lr2 for the next 4) equal the oracle's adam restatement
(oracle.c or_opt_step, pinned by the reference's own optimizers in
test_oracle_golden) replayed on the device's own per-step gradients."""
import numpy as np
import pytest

from conftest import assert_params_close, noise_mask

pytestmark = pytest.mark.gpu



def _trainer(ctx, pp, vp):
    from dependence_free_rl_amd import POLICY, VALUE, Trainer
    tr = Trainer(ctx, bins=8, dims=2, num_envs=64, steps=4, widths=(128, 64),
                 rng_state=4242)
    tr.set_params(POLICY, pp)
    tr.set_params(VALUE, vp)
    return tr


def test_sgd_rate_change_equals_new_optimizer(ctx):
    from dependence_free_rl_amd import POLICY, init_policy, init_value
    pp, vp = init_policy(2, 128, 64, seed=1), init_value(8, 2, seed=2)
    a, b = _trainer(ctx, pp, vp), _trainer(ctx, pp, vp)
    a.iterate(1)
    b.iterate(1)
    a.set_learning_rate(POLICY, 3e-4)
    b.set_optimizer(POLICY, "sgd", 3e-4)
    a.iterate(1)
    b.iterate(1)
    np.testing.assert_array_equal(a.params(POLICY), b.params(POLICY))


def test_adam_rate_change_keeps_state(ctx):
    from oracle import pyoracle as po
    from dependence_free_rl_amd import POLICY, init_policy, init_value
    from dependence_free_rl_amd.trainer import BUF_POLICY_GRADS
    pp, vp = init_policy(2, 128, 64, seed=3), init_value(8, 2, seed=4)
    lr1, lr2 = 1e-4, 3e-5
    tr = _trainer(ctx, pp, vp)
    tr.set_optimizer(POLICY, "adam", lr1)
    tr.iterate(1)
    g1 = tr.buffer(BUF_POLICY_GRADS).copy()
    tr.set_learning_rate(POLICY, lr2)
    tr.iterate(1)
    g2 = tr.buffer(BUF_POLICY_GRADS).copy()
    opt = po.Opt(po.OPT_ADAM, lr1)
    want = pp.astype(np.float32).copy()
    for g in g1:
        opt.step(want, g)
    opt.lr = lr2
    for g in g2:
        opt.step(want, g)
    grads = np.concatenate([g1, g2])
    mask = noise_mask(grads)
    assert_params_close(tr.params(POLICY), want, mask, 2 * lr1 * 8,
                        "adam after a rate change")
