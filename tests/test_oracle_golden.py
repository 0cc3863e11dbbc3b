"""Pin the CPU oracle (oracle/oracle.c) to the real reference's golden vectors.

The golden .npz fixtures were produced by oracle/_ref/ref_harness -- the
reference compiled from /root/reference with its own flags -- via
tests/golden/make_golden.py.  CPU only.
"""
import numpy as np
import pytest

from conftest import assert_close, assert_params_close, golden, noise_mask
from oracle import pyoracle as po


def parse_meta(d):
    kv = dict(a.split("=", 1) for a in str(d["meta_args"]).split())
    return kv


def models_for(kv):
    B, D = int(kv["B"]), int(kv["D"])
    widths = [int(w) for w in kv["widths"].split(",")]
    algo = kv["algo"]
    if algo == "pg":
        pol = po.full_model(B * 2 * D, widths, B, po.OR_SOFTMAX_XENT)
        return pol, None
    head = po.OR_SOFTMAX_XENT if algo == "ac" else po.OR_SOFTMAX
    pol = po.perbin_model(2 * D, widths, head)
    val = po.full_model(B * 2 * D, [64, 32], 1)
    return pol, val


# ------------------------------------------------------------------ RNG ----
def test_minstd_raw_and_canonical():
    g = golden("rng")
    r = po.Rng.seeded(42)
    raw = np.array([r.next() for _ in range(len(g["raw"]))], np.uint32)
    np.testing.assert_array_equal(raw, g["raw"])
    r = po.Rng.seeded(42)
    can = np.array([r.canonical() for _ in range(len(g["canonical"]))])
    np.testing.assert_array_equal(can, g["canonical"])  # bit-exact doubles


def test_bernoulli():
    g = golden("rng")
    r = po.Rng.seeded(42)
    b = np.array([r.bernoulli(0.4) for _ in range(len(g["bernoulli"]))])
    np.testing.assert_array_equal(b, g["bernoulli"])


@pytest.mark.parametrize("width", [8, 32, 64, 128])
def test_discrete_distribution(width):
    g = golden("rng")
    probs, picks = g["disc_probs_%d" % width], g["disc_pick_%d" % width]
    r = po.Rng.seeded(42 + width)
    got = np.array([r.discrete(p) for p in probs])
    np.testing.assert_array_equal(got, picks)
    assert r.state == int(g["disc_state_after_%d" % width][0])


def test_jump_ahead():
    r = po.Rng.seeded(123)
    for _ in range(1000):
        r.next()
    assert po.minstd_jump(po.lib().or_minstd_seed(123), 1000) == r.state


# ------------------------------------------------------------------ env ----
def test_env_trajectory_bit_exact():
    """bp::environment + bp::agent + random_policy, 3000 steps, seed 7."""
    g = golden("env8")
    cfg = po.env_cfg(8, 2)
    rng = po.Rng(int(g["x0"][0]))
    env = po.Env(cfg, rng)
    uniform = np.full(8, np.float32(1.0) / np.float32(8), np.float32)
    n = len(g["choice"])
    for k in range(n):
        np.testing.assert_array_equal(env.bins, g["start_bins"][k])
        np.testing.assert_array_equal(env.item[:2], g["start_item"][k])
        c = rng.discrete(uniform)
        assert c == g["choice"][k]
        env.apply(c)
        np.testing.assert_array_equal(env.bins, g["end_bins"][k])
        np.testing.assert_array_equal(env.item[:2], g["end_item"][k])
        over = bool((env.bins < 0).any())
        assert int(not over) == g["reward"][k]
        if over:
            env.reset()
    assert rng.state == int(g["x_end"][0])
    assert int(g["gen_env_identical"][0]) == 1
    # the benchmark-shape envs (64 / 128 bins) reproduce the reference env on
    # 8 injected bins, the rest staying full (ref_harness.cc envcheck_injected)
    assert int(g["gen_env64_identical"][0]) == 1
    assert int(g["gen_env128_identical"][0]) == 1


# ---------------------------------------------------------- deep agent ----
def test_weights20_logits_and_argmax_episodes():
    g = golden("deep_w20")
    m = po.perbin_model(4, [128, 64], None)
    assert po.nparams(m) == 8961 == g["params"].size
    z = po.model_eval(m, g["params"], g["obs"])
    assert_close(z, g["logits"], what="weights.20 logits")
    # empty bins, item (4,2): every bin scores the same
    assert np.allclose(z[0], z[0, 0])
    total, _ = po.eval_argmax(8, 2, m, g["params"], 1000, int(g["x0"][0]))
    assert total == float(g["total_reward"][0]) == 26600.0


# ------------------------------------------------------------- learners ----
LEARN = ["ppo_b8d2", "ppo_b32d1", "ppo_b64d2", "ac_b8d2", "ac_b128d3", "pg_b8d1",
         "klppo_b8d2", "ppo_adam_b8d2", "ac_mom_b8d2", "pg_b8d2",
         "ppo_b64d2_n160"]
ALGO = {"ppo": po.OR_PPO, "ac": po.OR_AC, "pg": po.OR_PG, "klppo": po.OR_KLPPO}
OPT = {"sgd": po.OPT_SGD, "momentum": po.OPT_MOMENTUM, "adam": po.OPT_ADAM}


def run_oracle_against(name, forced=True):
    g = golden(name)
    kv = parse_meta(g)
    B, D, N = int(kv["B"]), int(kv["D"]), int(kv["N"])
    T = int(kv.get("T", 4))
    algo = ALGO[kv["algo"]]
    pol, val = models_for(kv)
    lr_pi = 1e-5 if kv["algo"] == "ac" else 1e-4
    lr_v = 1e-4 if kv["algo"] == "ac" else 1e-5
    tr = po.Trainer(algo, B, D, N, T, pol, g["init_policy"], val,
                    g["init_value"] if val is not None else None, lr_pi=lr_pi,
                    lr_v=lr_v, wd_pi=float(kv.get("wd_pi", 0.0)), gamma=0.99,
                    x0=int(g["x0"][0]),
                    episodes=int(kv.get("episodes", 1)))
    for which, key, lr in ((0, "opt_pi", lr_pi), (1, "opt_v", lr_v)):
        if key in kv:
            tr.set_optimizer(which, OPT[kv[key]], lr)
    iters = int(kv["iters"])
    worst = {}
    adam = {w: kv.get(k) == "adam" for w, k in ((0, "opt_pi"), (1, "opt_v"))}
    lrs = {0: lr_pi, 1: lr_v}
    mask = {0: None, 1: None}
    nsteps = {0: 0, 1: 0}
    for it in range(iters):
        p = "it%d_" % it
        f = g[p + "step_choice"] if (forced and algo != po.OR_PG) else None
        tr.rollout(forced=f)
        ns = len(g[p + "step_choice"])
        np.testing.assert_array_equal(
            tr.buf(po.BUF_STEP_BINS).reshape(ns, B, D), g[p + "step_bins"])
        np.testing.assert_array_equal(
            tr.buf(po.BUF_STEP_ITEM).reshape(ns, D), g[p + "step_item"])
        np.testing.assert_array_equal(tr.buf(po.BUF_STEP_CHOICE), g[p + "step_choice"])
        np.testing.assert_array_equal(tr.buf(po.BUF_STEP_DONE), g[p + "step_done"])
        pch = g[p + "step_distrib"][np.arange(ns), g[p + "step_choice"]]
        worst["p_old"] = max(worst.get("p_old", 0),
                             assert_close(tr.buf(po.BUF_STEP_PCHOICE), pch, what="p_old"))
        np.testing.assert_array_equal(
            tr.buf(po.BUF_FINAL_BINS).reshape(N, B, D), g[p + "final_bins"])
        tr.learn()
        rows = g[p + "rows"]
        np.testing.assert_array_equal(tr.buf(po.BUF_ROWS).reshape(rows.shape), rows)
        np.testing.assert_array_equal(tr.buf(po.BUF_ROW_ENV), g[p + "row_env"])
        np.testing.assert_array_equal(tr.buf(po.BUF_ROW_STEP), g[p + "row_step"])
        np.testing.assert_array_equal(tr.buf(po.BUF_ROW_IS_END), g[p + "row_is_end"])
        checks = [("advantages", tr.buf(po.BUF_ADVANTAGES), g[p + "advantages"]),
                  ("policy_grads", tr.buf(po.BUF_POLICY_GRADS),
                   g[p + "policy_grads"].ravel())]
        if algo != po.OR_PG:
            checks += [("values", tr.buf(po.BUF_VALUES), g[p + "values_before"]),
                       ("value_grad", tr.buf(po.BUF_VALUE_GRAD), g[p + "value_grad"])]
        for what, x, y in checks:
            worst[what] = max(worst.get(what, 0), assert_close(x, y, what=p + what))
        params = [(0, "policy_params", "policy_grads")]
        if algo != po.OR_PG:
            params.append((1, "value_params", "value_grad"))
        for w, what, gk in params:
            gr = g[p + gk]
            nsteps[w] += gr.reshape(-1, gr.shape[-1]).shape[0]
            if adam[w]:
                mask[w] = noise_mask(gr, mask[w])
            worst[what] = max(worst.get(what, 0), assert_params_close(
                tr.params(w), g[p + what], mask[w], 2 * lrs[w] * nsteps[w],
                what=p + what))
        assert tr.rng == int(g[p + "x_end"][0])
    return worst


@pytest.mark.parametrize("name", LEARN)
def test_learner_matches_reference(name):
    worst = run_oracle_against(name, forced=True)
    print(name, {k: "%.2e" % v for k, v in worst.items()})


def test_env_streams_single_env_is_reference_stream():
    """or_trainer_set_env_streams (the device REINFORCE convention: env g on
    the stream advanced by g * 2^26) leaves env 0 on the reference's engine:
    pg_b8d1's one-worker run is reproduced with it on."""
    g = golden("pg_b8d1")
    kv = parse_meta(g)
    pol, _ = models_for(kv)
    tr = po.Trainer(po.OR_PG, 8, 1, 1, 1, pol, g["init_policy"],
                    x0=int(g["x0"][0]), episodes=int(kv["episodes"]))
    tr.set_env_streams(1 << 26)
    for it in range(int(kv["iters"])):
        tr.rollout()
        np.testing.assert_array_equal(tr.buf(po.BUF_STEP_CHOICE),
                                      g["it%d_step_choice" % it])
        tr.learn()
        assert int(tr.env_streams()[0]) == int(g["it%d_x_end" % it][0])
        assert_close(tr.params(0), g["it%d_policy_params" % it])


@pytest.mark.parametrize("name", ["ppo_adam_b8d2", "ac_mom_b8d2", "klppo_b8d2"])
def test_optimizer_restatement_on_reference_gradients(name):
    """or_opt_step fed the reference's own recorded gradients reproduces the
    reference's parameters after every step (momentum / adam / sgd with weight
    decay, state carried across learn() calls)."""
    g = golden(name)
    kv = parse_meta(g)
    ac = kv["algo"] == "ac"
    for w, pk, gk, ok, lr, wd in (
            (0, "policy_params", "policy_grads", "opt_pi", 1e-5 if ac else 1e-4,
             float(kv.get("wd_pi", 0))),
            (1, "value_params", "value_grad", "opt_v", 1e-4 if ac else 1e-5, 0.0)):
        p = np.array(g["init_policy" if w == 0 else "init_value"], np.float32)
        opt = po.Opt(OPT[kv.get(ok, "sgd")], lr, wd)
        for it in range(int(kv["iters"])):
            gr = g["it%d_%s" % (it, gk)]
            for row in gr.reshape(-1, gr.shape[-1]):
                opt.step(p, row)
            assert_close(p, g["it%d_%s" % (it, pk)], tol=1e-6, what=pk)


@pytest.mark.parametrize("name", ["ppo_b8d2", "ac_b8d2", "pg_b8d1", "klppo_b8d2"])
def test_free_running_sampling_matches_reference(name):
    """Without teacher forcing the oracle's own sampler reproduces the
    reference's actions (no probability near-ties in these fixtures)."""
    run_oracle_against(name, forced=False)


# ----------------------------------------------------------- heuristics ----
@pytest.mark.parametrize("kind", ["firstfit", "bestfit", "minwaste", "random"])
def test_heuristic_agents_match_reference(kind):
    """or_heuristic_eval vs the reference's own agent programs' policies
    (heur_* fixtures: 2 rounds x 1000 episodes, seed 3)."""
    g = golden("heur_" + kind)
    for r in range(2):
        total, lens, _ = po.heuristic_eval(8, 2, kind, 1000, int(g["x_round"][r]))
        assert np.float32(total / 1000.0) == g["round_avg"][r]
        if r == 0:
            np.testing.assert_array_equal(lens, g["episode_len"])


def test_venv_driver_matches_reference():
    """or_venv_run (the vectorised env's checker): one agent with a 2-draw
    policy replays the reference's env8 trajectory given its choices, and a
    shard of a many-env run equals that part of the whole run."""
    g = golden("env8")
    n = len(g["choice"])
    out = po.venv_run(8, 2, 1, int(g["x0"][0]),
                      np.asarray(g["choice"], np.int32).reshape(n, 1))
    np.testing.assert_array_equal(out["bins"][:n, 0], g["start_bins"])
    np.testing.assert_array_equal(out["item"][:n, 0], g["start_item"])
    np.testing.assert_array_equal(out["reward"][:, 0], g["reward"])
    assert out["x_end"] == int(g["x_end"][0])
    rng = np.random.default_rng(3)
    acts = rng.integers(0, 16, size=(6, 12)).astype(np.int32)
    full = po.venv_run(16, 3, 12, 99, acts)
    part = po.venv_run(16, 3, 4, 99, acts[:, 5:9], n_global=12, offset=5)
    for k in ("bins", "item", "reward", "done"):
        np.testing.assert_array_equal(part[k], full[k][:, 5:9])
    assert part["x_end"] == full["x_end"]


def test_reference_env_pins_the_d2_goldens():
    """Every learner golden of a D = 2 shape the reference's env can take was
    driven by the reference's own bp::environment / bp::agent: 8 bins from
    apps/bin_packing/bin_packing.h as it is, BASELINE config 3's 64 bins from
    the same header compiled with num_bins = 64 (oracle/Makefile,
    ref_harness_bp64).  The other shapes (1-D, 3-D, 32 / 128 bins) are
    gen_env's and say so."""
    for name in ("ppo_b64d2", "ppo_b64d2_n160"):
        g = golden(name)
        assert int(g["env_is_reference"][0]) == 1, name
        assert "bp::environment" in str(g["meta_env"]), name
        assert "num_bins = 64" in str(g["meta_env"]), name
    for name in ("ppo_b8d2", "ac_b8d2", "klppo_b8d2", "ppo_adam_b8d2",
                 "ac_mom_b8d2", "pg_b8d2"):
        assert int(golden(name)["env_is_reference"][0]) == 1, name
    for name in ("ppo_b32d1", "ac_b128d3", "pg_b8d1"):
        g = golden(name)
        assert int(g["env_is_reference"][0]) == 0 and "gen_env" in str(g["meta_env"])
