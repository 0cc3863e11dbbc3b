"""The reference's generic training API on the device (include/xylo_hip.h
"layer / model / optimizer / loss"), the pieces a caller assembles a learner
from: model::forward / gradient (nn.h:481-528), layer::backward / gradient
(nn.h:20-33), the discrete-action loss gradients (rl.h:33-74,
policy_gradient.h:24-85) and optimizer::next_parameters (nn.h:616-698).

Pinned by the reference itself: on golden ppo_b8d2 (the reference's
ppo_learner on its own bp::environment), model_forward -> surrogate loss
-> model_gradient reproduces the reference's first-epoch policy gradient, and
the value net's square-loss step its value gradient (row-summed fp32 bound,
sides = 2); against the oracle's double sums the same gradients hold the
tight budget of conftest.  The composed-learner C++ program
(tests/compat/composed_learner.cc) runs whole learn() calls from these
pieces and reproduces the golden's parameters iteration by iteration."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, assert_close, assert_grad_close, assert_grad_units, golden

pytestmark = pytest.mark.gpu

POLICY_LAYERS = [("conv1d_1", 4, 128), ("relu", 0, 0), ("conv1d_1", 128, 64),
                 ("relu", 0, 0), ("conv1d_1", 64, 1), ("softmax", 0, 0)]
VALUE_LAYERS = [("full", 32, 64), ("relu", 0, 0), ("full", 64, 32),
                ("relu", 0, 0), ("full", 32, 1)]


def _rows_distrib(g, p="it0_"):
    """Each learner row's action distribution (the end rows repeat the last
    transition's action, policy_gradient.h:173-178)."""
    dist = {(int(e), int(s)): d for e, s, d in zip(g[p + "step_env"],
                                                   g[p + "step_index"],
                                                   g[p + "step_distrib"])}
    out = []
    for e, s, end in zip(g[p + "row_env"], g[p + "row_step"], g[p + "row_is_end"]):
        out.append(out[-1] if end else dist[(int(e), int(s))])
    return np.asarray(out, np.float32)


def test_policy_epoch_from_pieces_matches_the_reference(ctx):
    from oracle import pyoracle as po
    from dependence_free_rl_amd.trainer import (action_loss_grad, model_forward,
                                                model_gradient)
    g = golden("ppo_b8d2")
    x = g["it0_rows"]
    choice = g["it0_row_choice"]
    adv = g["it0_advantages"]
    params = g["init_policy"]
    distrib = _rows_distrib(g)
    acts = model_forward(ctx, POLICY_LAYERS, params, x)
    pm = po.perbin_model(4, [128, 64], po.OR_SOFTMAX)
    assert len(acts) == len(POLICY_LAYERS) + 1
    assert_close(acts[-1], po.model_eval(pm, params, x), tol=1e-5,
                 what="model_forward output")
    target = action_loss_grad(ctx, "surrogate_loss", choice, adv, acts[-1],
                              distrib)
    grad = model_gradient(ctx, POLICY_LAYERS, params, acts[:-1], target)
    pold = distrib[np.arange(len(choice)), choice]
    ref, mag = po.policy_grad_rows_mag(pm, params, x, choice, pold, adv, po.OR_PPO)
    n_terms = x.shape[0] * 8
    # the reference's own fp32 gradient of its first epoch (sides = 2)
    assert_grad_close(grad, g["it0_policy_grads"][0], mag, n_terms, sides=2,
                      what="pieces vs reference epoch 0")
    assert_grad_units(grad, ref, mag, what="model_api ppo_b8d2 policy epoch0")


def test_value_step_from_pieces_matches_the_reference(ctx):
    """update_value_model (policy_gradient.h:196-218): V over the rows, TD
    targets r + gamma V(next) (end rows keep their value), square-loss
    gradient (nn.h:535-537) through model_gradient."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd.trainer import model_forward, model_gradient
    g = golden("ppo_b8d2")
    x = g["it0_rows"]
    params = g["init_value"]
    acts = model_forward(ctx, VALUE_LAYERS, params, x)
    v = acts[-1].ravel()
    assert_close(v, g["it0_values_before"], what="value forward")
    reward = g["it0_row_reward"].astype(np.float32)
    end = g["it0_row_is_end"].astype(bool)
    targets = np.empty_like(v)
    for r in range(len(v)):
        targets[r] = v[r] if end[r] else np.float32(reward[r] + np.float32(0.99) * v[r + 1])
    target = (acts[-1].ravel() - targets).reshape(-1, 1)
    grad = model_gradient(ctx, VALUE_LAYERS, params, acts[:-1], target)
    vm = po.full_model(32, [64, 32], 1)
    ref, mag = po.value_grad_rows_mag(vm, params, x, targets)
    assert_grad_close(grad, g["it0_value_grad"], mag, len(v), sides=2,
                      what="value gradient vs reference")
    assert_close(grad, g["it0_value_grad"], what="value gradient")


def test_layer_backward_and_gradient(ctx):
    """One layer at a time (layer::backward / gradient) against numpy in
    float64: Dense (full and per-point), relu (gated by the input's sign),
    softmax (the Jacobian product) and softmax_cross_entropy (backprop
    passed through)."""
    from dependence_free_rl_amd.trainer import layer_backward, layer_gradient
    rng = np.random.default_rng(5)
    rows = 37
    # full_layer 24 -> 10
    x = rng.normal(size=(rows, 24)).astype(np.float32)
    W = rng.normal(size=(10, 24)).astype(np.float32)
    b = rng.normal(size=10).astype(np.float32)
    bp = rng.normal(size=(rows, 10)).astype(np.float32)
    p = np.concatenate([W.ravel(), b])
    got = layer_backward(ctx, ("full", 24, 10), p, x, bp)
    np.testing.assert_allclose(got, bp.astype(np.float64) @ W, rtol=1e-5, atol=1e-5)
    gw = layer_gradient(ctx, ("full", 24, 10), x, bp)
    want = np.concatenate([(bp.T.astype(np.float64) @ x).ravel(), bp.sum(0)])
    np.testing.assert_allclose(gw, want, rtol=1e-5, atol=1e-4)
    # convolution1d_1 4 -> 6 over 8 points per row
    x = rng.normal(size=(rows, 32)).astype(np.float32)
    W = rng.normal(size=(6, 4)).astype(np.float32)
    bp = rng.normal(size=(rows, 48)).astype(np.float32)
    p = np.concatenate([W.ravel(), np.zeros(6, np.float32)])
    got = layer_backward(ctx, ("conv1d_1", 4, 6), p, x, bp)
    want = (bp.reshape(-1, 6).astype(np.float64) @ W).reshape(rows, 32)
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5)
    gw = layer_gradient(ctx, ("conv1d_1", 4, 6), x, bp)
    want = np.concatenate([(bp.reshape(-1, 6).T.astype(np.float64) @
                            x.reshape(-1, 4)).ravel(), bp.reshape(-1, 6).sum(0)])
    np.testing.assert_allclose(gw, want, rtol=1e-5, atol=1e-4)
    # relu: exact
    x = rng.normal(size=(rows, 16)).astype(np.float32)
    bp = rng.normal(size=(rows, 16)).astype(np.float32)
    np.testing.assert_array_equal(layer_backward(ctx, ("relu", 0, 0), [], x, bp),
                                  np.where(x > 0, bp, 0))
    assert layer_gradient(ctx, ("relu", 0, 0), x, bp).size == 0
    # softmax: (diag(s) - s s^T) g per row (nn.h:393-417)
    z = rng.normal(size=(rows, 8)).astype(np.float32)
    s = np.exp(z.astype(np.float64))
    s /= s.sum(1, keepdims=True)
    want = np.stack([(np.diag(si) - np.outer(si, si)) @ gi
                     for si, gi in zip(s, bp[:, :8].astype(np.float64))])
    np.testing.assert_allclose(layer_backward(ctx, ("softmax", 0, 0), [], z,
                                              bp[:, :8]), want, atol=1e-6)
    np.testing.assert_array_equal(
        layer_backward(ctx, ("softmax_xent", 0, 0), [], z, bp[:, :8]), bp[:, :8])


def test_action_loss_gradients_are_the_reference_expressions(ctx):
    """Every element equals the reference's host expression in float32
    (rl.h:33-74; kl: policy_gradient.h:55-74's gradient part)."""
    from dependence_free_rl_amd.trainer import action_loss_grad
    rng = np.random.default_rng(9)
    rows, B = 50, 16
    p = rng.random((rows, B)).astype(np.float32) + np.float32(0.01)
    p /= p.sum(1, keepdims=True)
    q = rng.random((rows, B)).astype(np.float32) + np.float32(0.01)
    q /= q.sum(1, keepdims=True)
    ch = rng.integers(0, B, rows).astype(np.int32)
    adv = rng.normal(size=rows).astype(np.float32)
    f = np.float32
    want = {k: np.zeros((rows, B), np.float32) for k in
            ("gradient_log", "policy_loss", "surrogate_loss", "kl_regulated")}
    beta = f(0.05)
    for r in range(rows):
        c, a = ch[r], adv[r]
        want["policy_loss"][r] = p[r] * a
        want["policy_loss"][r, c] = f(p[r, c] * a) - a
        want["kl_regulated"][r] = want["policy_loss"][r] + (p[r] - q[r]) * beta
        ratio = f(p[r, c] / q[r, c])
        clipped = min(max(ratio, f(1) - f(0.2)), f(1) + f(0.2))
        imp = min(f(clipped * a), f(ratio * a)) * f(-1)
        want["surrogate_loss"][r, c] = f(imp / p[r, c])
        weighted = f(f(f(1) / p[r, c]) * a) * f(-1)
        want["gradient_log"][r, c] = f(f(p[r, c] / q[r, c]) * weighted)
    for kind, w in want.items():
        got = action_loss_grad(ctx, kind, ch, adv, p, None if kind == "policy_loss"
                               else q, param=0.2 if kind != "kl_regulated" else beta)
        np.testing.assert_array_equal(got, w, err_msg=kind)


@pytest.mark.parametrize("kind", ["sgd", "momentum", "adam"])
def test_optimizer_apply_matches_the_oracle(ctx, kind):
    """next_parameters (nn.h:616-698) for three steps, the optimizer state
    carried by the caller, against the oracle's or_opt_step: bit for bit."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd.trainer import optimizer_apply
    rng = np.random.default_rng(3)
    n = 1000
    p0 = rng.normal(size=n).astype(np.float32)
    lr, wd = 1e-3, (1e-5 if kind == "sgd" else 0.0)
    o = po.Opt({"sgd": 0, "momentum": 1, "adam": 2}[kind], lr, wd)
    ref = p0.copy()
    dev, m, v = p0.copy(), None, None
    for t in range(1, 4):
        grad = rng.normal(size=n).astype(np.float32)
        o.step(ref, grad)
        dev, m, v = optimizer_apply(ctx, kind, dev, grad, lr, wd, t=float(t),
                                    m=m, v=v)
        np.testing.assert_array_equal(dev, ref, err_msg="%s step %d" % (kind, t))


@pytest.mark.parametrize("mode", ["subclass", "pieces", "fused"])
def test_composed_learner_program_matches_golden(tmp_path, mode):
    """A C++ program built against include/xylo_compat assembles PPO from the
    public pieces (a ppo_learner subclass overriding optimize_action with
    optimizer::step(surrogate_loss), or a learn() written from
    update_value_model / calculate_advantage / optimizer::step) and trains
    the reference's bp::environment agents on the device: after every one of
    the golden's 5 iterations both nets' parameters equal the reference's
    within 1e-4 (golden ppo_b8d2).  The library's fused learner is run as
    the control."""
    exe = os.path.join(REPO, "build", "compat", "composed_learner")
    if not os.path.exists(exe):
        pytest.skip("build/compat/composed_learner not built (make compat)")
    g = golden("ppo_b8d2")
    out = str(tmp_path / "run")
    r = subprocess.run([exe, "mode=" + mode, "N=8", "T=8", "iters=5", "seed=42",
                        "widths=128,64", "out=" + out], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    for it in range(5):
        pol = np.fromfile("%s.it%d.policy.bin" % (out, it), np.float32)
        val = np.fromfile("%s.it%d.value.bin" % (out, it), np.float32)
        assert_close(pol, g["it%d_policy_params" % it],
                     what="%s it%d policy" % (mode, it))
        assert_close(val, g["it%d_value_params" % it],
                     what="%s it%d value" % (mode, it))
