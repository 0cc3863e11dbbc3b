"""Wide-range policy parameters on the f16-pair kernels.

The f16-pair operands (csrc/xh_split.h) are scaled per launch by a power of
two from the operand's maximum, so |S x| <= 2^14.  The split
S x = hi + lo + e has |e| <= 2^-22 |S x| only while lo is a normal f16;
below |S x| = 2^-3 (2^17 under the launch maximum) lo is subnormal and e is an
absolute <= 2^-25 in scaled units.  An operand entry far below its launch's
maximum therefore loses relative accuracy that the reference's fp32
matmul_transposed (/root/reference/xylo/tensor.cc:218-227) keeps.  These
cases put parts of the policy 2^20 below the rest and hold the epoch-0
gradients to the tight budget of conftest against the oracle's double sums
(logged as `range ...` in grad_units.jsonl)."""
import numpy as np
import pytest

from conftest import assert_close, assert_grad_units

pytestmark = pytest.mark.gpu

SMALL = 2.0 ** -20


def _scaled(pp, D, H1, H2, how):
    """Reference flat layout (nn.h:499-508): W1 [H1][2D], b1, W2 [H2][H1],
    b2, w3 [H2], b3."""
    p = pp.copy()
    f0 = 2 * D
    oW1, ob1 = 0, H1 * f0
    oW2 = ob1 + H1
    ob2 = oW2 + H2 * H1
    ow3 = ob2 + H2
    if how == "w2_rows":      # half the layer-2 units 2^20 smaller
        p[oW2:oW2 + (H2 // 2) * H1] *= SMALL
    elif how == "w2_cols":    # every W2 row spans 2^20 (K direction)
        w2 = p[oW2:ob2].reshape(H2, H1)
        w2[:, ::2] *= SMALL
    elif how == "h1_units":   # half the layer-1 units (H1 features) tiny
        w1 = p[oW1:ob1].reshape(H1, f0)
        w1[: H1 // 2] *= SMALL
        p[ob1:ob1 + H1 // 2] *= SMALL
    elif how == "w3":         # layer 3 weights 2^20 apart (W2' = diag(w3) W2)
        p[ow3:ow3 + H2 // 2] *= SMALL
    return p.astype(np.float32)


@pytest.mark.parametrize("how", ["w2_rows", "w2_cols", "h1_units", "w3"])
@pytest.mark.parametrize("algo,B,D,N,T", [("ppo", 64, 2, 32, 4),
                                         ("ac", 128, 3, 8, 8)])
def test_wide_range_parameters(ctx, how, algo, B, D, N, T):
    from oracle import pyoracle as po
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import BUF_ACTION, BUF_POLICY_GRADS
    H1 = H2 = 128
    x0 = 8642
    pp = _scaled(init_policy(D, H1, H2, seed=61), D, H1, H2, how)
    vp = init_value(B, D, seed=62)
    tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                 widths=(H1, H2), rng_state=x0)
    tr.set_params(POLICY, pp)
    tr.set_params(VALUE, vp)
    head = po.OR_SOFTMAX_XENT if algo == "ac" else po.OR_SOFTMAX
    orc = po.Trainer({"ppo": po.OR_PPO, "ac": po.OR_AC}[algo], B, D, N, T,
                     po.perbin_model(2 * D, [H1, H2], head), pp,
                     po.full_model(B * 2 * D, [64, 32], 1), vp,
                     lr_pi=1e-5 if algo == "ac" else 1e-4,
                     lr_v=1e-4 if algo == "ac" else 1e-5, x0=x0)
    tr.rollout()
    orc.rollout()
    np.testing.assert_array_equal(tr.buffer(BUF_ACTION),
                                  orc.buf(po.BUF_STEP_CHOICE).reshape(N, T).T)
    tr.learn()
    orc.learn()
    npi = tr.num_params(POLICY)
    dev = tr.buffer(BUF_POLICY_GRADS).reshape(-1, npi)
    ref = np.asarray(orc.buf(po.BUF_POLICY_GRADS)).reshape(-1, npi)
    mag = np.asarray(orc.buf(po.BUF_POLICY_GRADS_MAG)).reshape(-1, npi)
    assert_grad_units(dev[0], ref[0], mag[0],
                      what="range %s %s B%d D%d N%d T%d epoch0" % (how, algo, B,
                                                                   D, N, T))
    if algo == "ac":
        assert_close(tr.params(POLICY), orc.params(0), what="policy params")
