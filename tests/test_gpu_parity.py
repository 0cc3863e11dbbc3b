"""GPU parity: the HIP path (through the C ABI) against the golden vectors of
the real reference and against the CPU oracle.  Run on the MI355X box:

    python -m pytest tests -m gpu -x -q

Bit-exact: env states, items, dones, actions, RNG states.  Tolerance
(|x - y| <= 1e-4 * max(1, |y|), conftest.RTOL): logits, probabilities,
values, advantages, gradients, parameters.
"""
import numpy as np
import pytest

from conftest import (GRAD_UNITS_P99_DRIFT, assert_close, assert_grad_close,
                      assert_grad_units, assert_params_close, golden, noise_mask)
from gpu_helpers import (default_lr, meta, row_index, step_major,
                         trainer_from_golden)

pytestmark = pytest.mark.gpu



ENV_CASES = ["ppo_b8d2", "ppo_b32d1", "ppo_b64d2", "ppo_b64d2_n160", "ac_b8d2",
             "ac_b128d3", "ac_b128d3_n96", "ppo_b32d1_n768",
             "klppo_b8d2"]


@pytest.mark.parametrize("name", ENV_CASES)
def test_env_construction_bit_exact(ctx, name):
    from dependence_free_rl_amd.trainer import BUF_BINS, BUF_ITEMS
    tr, g, kv = trainer_from_golden(ctx, name)
    N, T, D = tr.N, tr.T, tr.D
    bins = tr.buffer(BUF_BINS)[0]
    items = tr.buffer(BUF_ITEMS)[0, :, :D]
    s_bins = step_major(g["it0_step_bins"], N, T)[0]
    s_item = step_major(g["it0_step_item"], N, T)[0]
    np.testing.assert_array_equal(bins, s_bins)
    np.testing.assert_array_equal(items, s_item)


@pytest.mark.parametrize("name", ENV_CASES)
def test_rollout_teacher_forced_bit_exact(ctx, name):
    """Given the reference's actions, every env transition, item draw, reset
    and RNG state matches the reference bit for bit."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd.trainer import (BUF_BINS, BUF_DONE, BUF_ITEMS,
                                                BUF_POLD, BUF_RNG, POLICY)
    tr, g, kv = trainer_from_golden(ctx, name)
    N, T, B, D = tr.N, tr.T, tr.B, tr.D
    x0 = int(g["x0"][0])
    for it in range(int(kv["iters"])):
        p = "it%d_" % it
        if it > 0:
            tr.set_params(POLICY, g["it%d_policy_params" % (it - 1)])
        tr.set_forced_actions(step_major(g[p + "step_choice"], N, T))
        tr.rollout()
        bins = tr.buffer(BUF_BINS)
        np.testing.assert_array_equal(bins[:T], step_major(g[p + "step_bins"], N, T))
        np.testing.assert_array_equal(bins[T], g[p + "final_bins"])
        items = tr.buffer(BUF_ITEMS)[:, :, :D]
        np.testing.assert_array_equal(items[:T], step_major(g[p + "step_item"], N, T))
        np.testing.assert_array_equal(items[T], g[p + "final_item"])
        np.testing.assert_array_equal(tr.buffer(BUF_DONE),
                                      step_major(g[p + "step_done"], N, T))
        dist = g[p + "step_distrib"]
        pch = dist[np.arange(len(dist)), g[p + "step_choice"]]
        assert_close(tr.buffer(BUF_POLD), step_major(pch, N, T), what="p_old")
        # per-env engine states: reference-order positions
        rng = tr.buffer(BUF_RNG)
        for e in (0, N - 1):
            pos = 2 * N + 4 * T * N * (it + 1) + 4 * T * e
            assert rng[e] == po.minstd_jump(x0, pos)
        assert po.minstd_jump(int(g[p + "x_end"][0]), 4 * T * (N - 1)) == rng[N - 1]
        tr.learn()  # advance the batch window (forget())


@pytest.mark.parametrize("name", ["ppo_b8d2", "ac_b8d2", "ppo_b64d2", "ac_b128d3"])
def test_rollout_sampling_matches_reference(ctx, name):
    """Free-running: the GPU's own softmax + categorical sampler picks the
    reference's actions (no fixture step lies on a probability near-tie)."""
    from dependence_free_rl_amd.trainer import BUF_ACTION, BUF_BINS, POLICY, VALUE
    tr, g, kv = trainer_from_golden(ctx, name)
    N, T = tr.N, tr.T
    for it in range(int(kv["iters"])):
        p = "it%d_" % it
        if it > 0:  # re-sync parameters so only sampling is under test
            tr.set_params(POLICY, g["it%d_policy_params" % (it - 1)])
            tr.set_params(VALUE, g["it%d_value_params" % (it - 1)])
        tr.rollout()
        np.testing.assert_array_equal(tr.buffer(BUF_ACTION),
                                      step_major(g[p + "step_choice"], N, T))
        np.testing.assert_array_equal(tr.buffer(BUF_BINS)[T], g[p + "final_bins"])
        tr.learn()


def _magnitude_oracle(g, kv):
    """The CPU oracle on the golden's initial state, teacher-forced in lockstep
    with the test: it supplies sum|terms| of every policy-gradient entry
    (or_model_grad_mag) for the row-summed gradient bound."""
    from oracle import pyoracle as po
    B, D, N, T = (int(kv["B"]), int(kv["D"]), int(kv["N"]), int(kv.get("T", 4)))
    widths = [int(w) for w in kv["widths"].split(",")]
    algo = kv["algo"]
    head = po.OR_SOFTMAX_XENT if algo == "ac" else po.OR_SOFTMAX
    code = {"ppo": po.OR_PPO, "ac": po.OR_AC, "klppo": po.OR_KLPPO}[algo]
    orc = po.Trainer(code, B, D, N, T, po.perbin_model(2 * D, widths, head),
                     g["init_policy"], po.full_model(B * 2 * D, [64, 32], 1),
                     g["init_value"], lr_pi=default_lr(algo, 0),
                     lr_v=default_lr(algo, 1), wd_pi=float(kv.get("wd_pi", 0.0)),
                     x0=int(g["x0"][0]))
    kinds = {"sgd": po.OPT_SGD, "momentum": po.OPT_MOMENTUM, "adam": po.OPT_ADAM}
    for which, key in ((0, "opt_pi"), (1, "opt_v")):
        if key in kv:
            orc.set_optimizer(which, kinds[kv[key]], default_lr(algo, which))
    return orc


@pytest.mark.parametrize("name", ["ppo_b8d2", "ppo_b32d1", "ppo_b64d2", "ac_b8d2",
                                  "ac_b128d3", "klppo_b8d2", "ppo_adam_b8d2",
                                  "ac_mom_b8d2", "ppo_b64d2_n160",
                                  # >= 3 row groups per train workgroup at
                                  # the config-5 / config-2 shapes
                                  "ac_b128d3_n96", "ppo_b32d1_n768"])
def test_learn_matches_reference(ctx, name):
    """Teacher-forced iterations: V, advantages, per-epoch policy gradients,
    value gradient and updated parameters vs the reference learner (sgd, and
    momentum / adam optimizers with their state carried across learn();
    adam's noise-level entries per conftest.noise_mask).  Policy gradients
    are row sums under heavy cancellation: they are held to the stated
    row-summed bound (conftest.assert_grad_close, both sides fp32), with
    sum|terms| from the oracle run in lockstep."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd.trainer import (BUF_ADV, BUF_POLICY_GRADS,
                                                BUF_V_STATE0, BUF_V_TERM,
                                                BUF_VALUE_GRAD, POLICY, VALUE)
    tr, g, kv = trainer_from_golden(ctx, name)
    orc = _magnitude_oracle(g, kv)
    N, T, B = tr.N, tr.T, tr.B
    worst = {}
    adam = {w: kv.get(k) == "adam" for w, k in ((POLICY, "opt_pi"),
                                               (VALUE, "opt_v"))}
    mask, nsteps = {POLICY: None, VALUE: None}, {POLICY: 0, VALUE: 0}
    for it in range(int(kv["iters"])):
        p = "it%d_" % it
        tr.set_forced_actions(step_major(g[p + "step_choice"], N, T))
        # the lockstep oracle learns from the device trainer's own parameters
        # (assert_grad_units measures one learn()'s arithmetic, not drift)
        orc.set_params(0, tr.params(POLICY))
        orc.set_params(1, tr.params(VALUE))
        tr.rollout()
        tr.learn()
        orc.rollout(forced=np.asarray(g[p + "step_choice"]).reshape(N, T))
        orc.learn()
        rows = row_index(g, it, T)
        v0, vt, adv = tr.buffer(BUF_V_STATE0), tr.buffer(BUF_V_TERM), tr.buffer(BUF_ADV)
        vrow, arow = [], []
        for kind, t, e in rows:
            if kind == 0:
                vrow.append(v0[t, e]); arow.append(adv[t, e])
            elif kind == 1:
                vrow.append(v0[T, e]); arow.append(0.0)
            else:
                vrow.append(vt[t, e]); arow.append(0.0)
        checks = [
            ("values", np.array(vrow), g[p + "values_before"]),
            ("advantages", np.array(arow), g[p + "advantages"]),
            ("value_grad", tr.buffer(BUF_VALUE_GRAD), g[p + "value_grad"]),
        ]
        for what, x, y in checks:
            worst[what] = max(worst.get(what, 0.0),
                              assert_close(x, y, what=p + what))
        worst["policy_grads"] = max(worst.get("policy_grads", 0.0), assert_grad_close(
            tr.buffer(BUF_POLICY_GRADS).ravel(), np.asarray(g[p + "policy_grads"]).ravel(),
            orc.buf(po.BUF_POLICY_GRADS_MAG), n_terms=N * T * B, sides=2,
            what=p + "policy_grads"))
        # the tight check against the lockstep oracle's double sums (the
        # same teacher-forced batch; conftest.assert_grad_units).  Under adam
        # the two sides' noise-level entries step apart after the first
        # update (conftest.noise_mask): there only the first epoch's
        # gradient, which both compute on the same parameters.
        # Epoch 0 runs on identical parameters on both sides: the tight
        # budget.  Epochs 1..k-1 start from parameters each side updated
        # itself (f32 steps of gradients that differ by the units above), so
        # a cancelled entry also carries that drift: the drift budget.
        npi = tr.num_params(POLICY)
        dev = tr.buffer(BUF_POLICY_GRADS).reshape(-1, npi)
        ref = np.asarray(orc.buf(po.BUF_POLICY_GRADS)).reshape(-1, npi)
        mag = np.asarray(orc.buf(po.BUF_POLICY_GRADS_MAG)).reshape(-1, npi)
        for ep in range(1 if adam[POLICY] else dev.shape[0]):
            if adam[POLICY] and it > 0:
                break
            budget = {} if ep == 0 else {"p99_units": GRAD_UNITS_P99_DRIFT}
            assert_grad_units(dev[ep], ref[ep], mag[ep],
                              what="golden %s %sepoch%d_policy_grads" % (name, p, ep),
                              **budget)
        for w, what, gk in ((VALUE, "value_params", "value_grad"),
                            (POLICY, "policy_params", "policy_grads")):
            gr = g[p + gk]
            nsteps[w] += gr.reshape(-1, gr.shape[-1]).shape[0]
            if adam[w]:
                mask[w] = noise_mask(gr, mask[w])
            worst[what] = max(worst.get(what, 0.0), assert_params_close(
                tr.params(w), g[p + what], mask[w],
                2 * default_lr(kv["algo"], w) * nsteps[w], what=p + what))
    print(name, {k: "%.2e" % v for k, v in worst.items()})


def test_weights20_logits(ctx):
    """deep_agent.cc's trained policy (weights.20): GPU logits vs the
    reference's model::eval for 64 fixed observations."""
    from dependence_free_rl_amd import Trainer
    from dependence_free_rl_amd.trainer import (BUF_BINS, BUF_ITEMS, BUF_LOGITS,
                                                POLICY)
    g = golden("deep_w20")
    tr = Trainer(ctx, algo="ppo", bins=8, dims=2, num_envs=64, steps=1,
                 widths=(128, 64), record_last_step=True)
    tr.set_params(POLICY, g["params"])
    obs = g["obs"].reshape(64, 8, 4)
    bins = np.zeros((2, 64, 8, 2), np.int8)
    bins[0] = np.rint(obs[:, :, :2] * 8).astype(np.int8)
    items = np.zeros((2, 64, 4), np.int8)
    items[0, :, :2] = np.rint(obs[:, 0, 2:] * 8).astype(np.int8)
    tr.set_buffer(BUF_BINS, bins)
    tr.set_buffer(BUF_ITEMS, items)
    tr.set_forced_actions(np.zeros((1, 64), np.int32))
    tr.rollout()
    z = tr.buffer(BUF_LOGITS)
    assert_close(z, g["logits"], what="weights.20 logits")
    assert abs(z[0, 0] - 2.76766) < 1e-4 and np.allclose(z[0], z[0, 0], atol=1e-6)


def test_deep_agent_argmax_episodes(ctx):
    """deep_agent.cc: weights.20, seed 1, 1000 argmax episodes -> total reward
    26600 (apps/bin_packing/deep_agent.cc:21-41), every episode length equal
    to the reference's; the other 7 envs of the group run on their own
    streams."""
    from dependence_free_rl_amd import Trainer
    from dependence_free_rl_amd.trainer import POLICY
    g = golden("deep_w20")
    tr = Trainer(ctx, algo="ppo", bins=8, dims=2, num_envs=8, steps=1,
                 widths=(128, 64))
    tr.set_params(POLICY, g["params"])
    r = tr.evaluate(8, 1000, int(g["x0"][0]), trace_cap=40)
    tot, steps = r["totals"], r["steps"]
    assert tot[0] == float(g["total_reward"][0]) == 26600.0
    assert steps[0] == int(g["episode_len"].sum()) == 27600
    # env 0's engine advanced by 2 (construction) + 2 per step
    from oracle import pyoracle as po
    assert r["rng"][0] == po.minstd_jump(int(g["x0"][0]), 2 + 2 * 27600)
    # first episode's actions: replay through the oracle env and its argmax
    # policy gives the same choices
    L0 = int(g["episode_len"][0])
    assert (r["trace"][:L0] >= 0).all() and (r["trace"][:L0] < 8).all()
    assert np.all(np.abs(tot / 1000.0 - 26.55) < 0.5)


def test_evaluate_from_given_items(ctx):
    """init_items: an env constructed earlier (item already drawn) plays from
    the engine's current state; splitting 1000 episodes into 10 x 100 calls,
    chaining final item and engine state, reproduces the one-call run."""
    from dependence_free_rl_amd import Trainer
    from dependence_free_rl_amd.trainer import POLICY
    from oracle import pyoracle as po
    g = golden("deep_w20")
    tr = Trainer(ctx, algo="ppo", bins=8, dims=2, num_envs=8, steps=1,
                 widths=(128, 64))
    tr.set_params(POLICY, g["params"])
    x0 = int(g["x0"][0])
    whole = tr.evaluate(8, 1000, x0)
    # construction draws by hand: bernoulli(0.4) on the first two draws
    rng = po.Rng(x0)
    first = rng.canonical() < 0.4
    item = [4, 2] if first else [1, 2]
    x, tot, n = po.minstd_jump(x0, 2), 0.0, 0
    for _ in range(10):
        r = tr.evaluate(8, 100, x, init_items=np.tile(item, (8, 1)))
        tot += r["totals"][0]
        n += int(r["steps"][0])
        x, item = int(r["rng"][0]), list(r["final_items"][0])
    assert tot == whole["totals"][0] and n == whole["steps"][0]
    assert x == whole["rng"][0]


def test_klppo_beta_and_old_distributions(ctx):
    """kl_ppo_learner specifics: the rollout keeps each step's whole sampled
    distribution (action.distrib, rl.h:27-30), and beta adapts per epoch
    from the mean KL over ALL rows (end rows included) as the oracle's
    restatement of kl_regulated_loss does (policy_gradient.h:41-85)."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd.trainer import BUF_KL, BUF_QOLD
    tr, g, kv = trainer_from_golden(ctx, "klppo_b8d2")
    N, T, B = tr.N, tr.T, tr.B
    from test_oracle_golden import models_for
    pol, val = models_for(kv)
    orc = po.Trainer(po.OR_KLPPO, B, 2, N, T, pol, g["init_policy"], val,
                     g["init_value"], wd_pi=1e-5, x0=int(g["x0"][0]))
    for it in range(int(kv["iters"])):
        p = "it%d_" % it
        tr.set_forced_actions(step_major(g[p + "step_choice"], N, T))
        tr.rollout()
        assert_close(tr.buffer(BUF_QOLD),
                     step_major(g[p + "step_distrib"], N, T), what="q_old")
        tr.learn()
        orc.rollout(forced=g[p + "step_choice"])
        orc.learn()
        okl = orc.buf(po.BUF_KL).reshape(-1, 3)
        gkl = tr.buffer(BUF_KL)
        np.testing.assert_array_equal(gkl[:, 0], okl[:, 0])   # beta used
        np.testing.assert_array_equal(gkl[:, 2], okl[:, 2])   # beta after
        assert_close(gkl[:, 1], okl[:, 1], what="mean KL")
