"""model::eval on the device (xh_model_eval): the drop-in layer's host-side
model::eval (nn.h:473-479) runs there.  Against the reference's own logits for
weights.20 (deep_w20 golden: conv1d_1 4->128->64->1 on 64 observations) and
against the oracle for the value net, a softmax head and REINFORCE's full
MLP.  Tolerance: conftest.RTOL."""
import numpy as np
import pytest

from conftest import assert_close, golden

pytestmark = pytest.mark.gpu


def test_weights20_logits_match_reference(ctx):
    from dependence_free_rl_amd.trainer import model_eval
    g = golden("deep_w20")
    layers = [("conv1d_1", 4, 128), ("relu", 0, 0), ("conv1d_1", 128, 64),
              ("relu", 0, 0), ("conv1d_1", 64, 1)]
    z = model_eval(ctx, layers, g["params"], g["obs"])
    assert_close(z, g["logits"], what="weights.20 logits")
    p = model_eval(ctx, layers + [("softmax", 0, 0)], g["params"], g["obs"])
    e = np.exp(g["logits"].astype(np.float64))
    assert_close(p, e / e.sum(1, keepdims=True), what="softmax head")


@pytest.mark.parametrize("kind", ["value", "pg"])
def test_full_mlps_match_oracle(ctx, kind):
    from oracle import pyoracle as po
    from dependence_free_rl_amd import init_full_policy, init_value
    from dependence_free_rl_amd.trainer import model_eval
    B, D = 64, 2
    rng = np.random.default_rng(3)
    x = (rng.integers(0, 9, size=(300, B * 2 * D)) / 8.0).astype(np.float32)
    if kind == "value":
        p = init_value(B, D, seed=5)
        layers = [("full", 256, 64), ("relu", 0, 0), ("full", 64, 32),
                  ("relu", 0, 0), ("full", 32, 1)]
        om = po.full_model(256, [64, 32], 1)
    else:
        p = init_full_policy(B, D, (256, 128), seed=6) * 3.0
        layers = [("full", 256, 256), ("relu", 0, 0), ("full", 256, 128),
                  ("relu", 0, 0), ("full", 128, B), ("softmax_xent", 0, 0)]
        om = po.full_model(256, [256, 128], B, po.OR_SOFTMAX_XENT)
    y = model_eval(ctx, layers, p, x)
    assert_close(y, po.model_eval(om, p, x), what=kind)


def test_model_eval_rejects_bad_shapes(ctx):
    from dependence_free_rl_amd import XhError
    from dependence_free_rl_amd.trainer import model_eval
    with pytest.raises(XhError):
        model_eval(ctx, [("full", 10, 4)], np.zeros(44, np.float32),
                   np.zeros((2, 9), np.float32))
    with pytest.raises(XhError):  # parameter count
        model_eval(ctx, [("full", 9, 4)], np.zeros(41, np.float32),
                   np.zeros((2, 9), np.float32))
