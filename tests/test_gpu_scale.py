"""GPU vs CPU oracle at the benchmark shape (64 bins, 2-D, [128,128]) and
size-independent properties at the full BASELINE config-3 size."""
import numpy as np
import pytest

from conftest import (assert_close, assert_grad_close, assert_grad_units,
                      log_record)

pytestmark = pytest.mark.gpu



def _oracle_trainer(B, D, N, T, widths, pp, vp, x0, algo):
    from oracle import pyoracle as po
    head = po.OR_SOFTMAX_XENT if algo == "ac" else po.OR_SOFTMAX
    pol = po.perbin_model(2 * D, list(widths), head)
    val = po.full_model(B * 2 * D, [64, 32], 1)
    code = {"ppo": po.OR_PPO, "ac": po.OR_AC, "klppo": po.OR_KLPPO}[algo]
    return po.Trainer(code, B, D, N, T, pol, pp, val, vp,
                      lr_pi=1e-5 if algo == "ac" else 1e-4,
                      lr_v=1e-4 if algo == "ac" else 1e-5,
                      wd_pi=1e-5 if algo == "klppo" else 0.0, x0=x0)


@pytest.mark.parametrize("algo,B,D,widths,N,T", [
    ("ppo", 64, 2, (128, 128), 32, 4),   # BASELINE config 3 shape
    ("ppo", 64, 2, (128, 128), 160, 4),  # 640 groups: multi-group train blocks
    ("ppo", 32, 1, (64, 64), 64, 4),     # config 2 shape
    # config 2 shape, 1536 two-env groups: 3 per train workgroup (2 x 256)
    ("ppo", 32, 1, (64, 64), 768, 4),
    ("ac", 32, 1, (64, 64), 96, 4),      # AC through the config-2 split kernel
    # an odd number of two-env groups (15)
    ("ppo", 32, 1, (64, 64), 10, 3),
    ("ac", 16, 2, (64, 64), 64, 8),
    ("ac", 128, 3, (128, 128), 8, 8),    # config 5 shape
    # config 5 shape, 768 row groups: 3 per train workgroup (256)
    ("ac", 128, 3, (128, 128), 96, 8),
    ("klppo", 64, 2, (128, 128), 16, 4),  # KL-PPO at the config-3 shape
])
def test_gpu_vs_oracle(ctx, algo, B, D, widths, N, T):
    from oracle import pyoracle as po
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_ADV, BUF_BINS,
                                                BUF_DONE, BUF_POLD,
                                                BUF_POLICY_GRADS, BUF_VALUE_GRAD)
    x0 = 987654321
    pp = init_policy(D, *widths, seed=3)
    vp = init_value(B, D, seed=4)
    tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                 widths=widths, rng_state=x0)
    tr.set_params(POLICY, pp)
    tr.set_params(VALUE, vp)
    orc = _oracle_trainer(B, D, N, T, widths, pp, vp, x0, algo)
    for it in range(2):
        tr.rollout()
        acts = tr.buffer(BUF_ACTION)            # [T][N]
        if it > 0:  # learn() from the device trainer's own parameters
            orc.set_params(0, tr.params(POLICY))
            orc.set_params(1, tr.params(VALUE))
        orc.rollout()                           # free-running oracle sampler
        o_choice = orc.buf(po.BUF_STEP_CHOICE).reshape(N, T).T
        np.testing.assert_array_equal(acts, o_choice)
        bins = tr.buffer(BUF_BINS)
        np.testing.assert_array_equal(
            bins[:T], orc.buf(po.BUF_STEP_BINS).reshape(N, T, B, D).swapaxes(0, 1))
        np.testing.assert_array_equal(
            bins[T], orc.buf(po.BUF_FINAL_BINS).reshape(N, B, D))
        np.testing.assert_array_equal(
            tr.buffer(BUF_DONE), orc.buf(po.BUF_STEP_DONE).reshape(N, T).T)
        assert_close(tr.buffer(BUF_POLD),
                     orc.buf(po.BUF_STEP_PCHOICE).reshape(N, T).T, what="p_old")
        tr.learn()
        orc.learn()
        # advantages of transition rows, in (t, env) order
        env = orc.buf(po.BUF_ROW_ENV)
        step = orc.buf(po.BUF_ROW_STEP) - it * T
        is_end = orc.buf(po.BUF_ROW_IS_END)
        oadv = orc.buf(po.BUF_ADVANTAGES)
        adv = tr.buffer(BUF_ADV)
        m = is_end == 0
        assert_close(adv[step[m], env[m]], oadv[m], what="advantages")
        assert_close(tr.buffer(BUF_VALUE_GRAD), orc.buf(po.BUF_VALUE_GRAD),
                     what="value_grad")
        assert_close(tr.params(VALUE), orc.params(1), what="value params")
        # every row of the batch contributes B per-bin rows to each sum
        assert_grad_close(tr.buffer(BUF_POLICY_GRADS).ravel(),
                          orc.buf(po.BUF_POLICY_GRADS),
                          orc.buf(po.BUF_POLICY_GRADS_MAG),
                          n_terms=len(env) * B, what="policy_grads")
        # the tight check against the oracle's double sums (conftest)
        assert_grad_units(tr.buffer(BUF_POLICY_GRADS).ravel(),
                          orc.buf(po.BUF_POLICY_GRADS),
                          orc.buf(po.BUF_POLICY_GRADS_MAG),
                          what="vs_oracle %s B%d D%d N%d T%d it%d" % (
                              algo, B, D, N, T, it))
        assert_close(tr.params(POLICY), orc.params(0), what="policy params")


def test_c3_full_size_properties(ctx):
    """BASELINE config 3 (32768 envs x 64 bins x 2-D, [128,128], T=4): env
    transition invariants on every env, probability normalisation, finite
    learner state, and bitwise run-to-run determinism."""
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_ADV, BUF_BINS,
                                                BUF_DONE, BUF_ITEMS, BUF_POLD,
                                                BUF_PROBS)
    N, B, D, T = 32768, 64, 2, 4
    pp, vp = init_policy(D, 128, 128, seed=1), init_value(B, D, seed=2)

    def make():
        tr = Trainer(ctx, bins=B, dims=D, num_envs=N, steps=T, widths=(128, 128),
                     rng_state=20241008, record_last_step=True)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        return tr

    tr = make()
    tr.iterate(2)
    tr.rollout()
    bins = tr.buffer(BUF_BINS).astype(np.int32)
    items = tr.buffer(BUF_ITEMS)[:, :, :D].astype(np.int32)
    act = tr.buffer(BUF_ACTION)
    done = tr.buffer(BUF_DONE)
    assert bins.min() >= 0 and bins.max() <= 8  # stored states never negative
    assert act.min() >= 0 and act.max() < B
    ok_items = ((items == [4, 2]).all(-1) | (items == [1, 2]).all(-1))
    assert ok_items.all()
    for t in range(T):
        nxt = bins[t].copy()
        idx = np.arange(N)
        nxt[idx, act[t]] -= items[t]
        over = (nxt[idx, act[t]] < 0).any(-1)
        np.testing.assert_array_equal(over.astype(np.uint8), done[t])
        keep = ~over
        np.testing.assert_array_equal(bins[t + 1][keep], nxt[keep])
        assert (bins[t + 1][over] == 8).all()
    probs = tr.buffer(BUF_PROBS)
    np.testing.assert_allclose(probs.sum(1), 1.0, atol=1e-5)
    pold = tr.buffer(BUF_POLD)
    assert (pold > 0).all() and (pold <= 1).all()
    tr.learn()
    p1 = tr.params(POLICY)
    assert np.isfinite(p1).all() and np.isfinite(tr.params(VALUE)).all()
    assert np.isfinite(tr.buffer(BUF_ADV)).all()
    # determinism: same seed, same params -> bitwise identical result
    tr2 = make()
    tr2.iterate(3)
    np.testing.assert_array_equal(tr2.params(POLICY), p1)


def test_c3_rng_positions_full_size(ctx):
    """Every env's minstd state after 2 iterations at full config-3 size sits
    at its reference-order position: 2 construction draws per
    env, then 4 draws per env step in worker order, i.e.
    jump(x0, 2N + 4TN*its + 4T*e)."""
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import BUF_RNG
    N, B, D, T, its, x0 = 32768, 64, 2, 4, 2, 1234567
    tr = Trainer(ctx, bins=B, dims=D, num_envs=N, steps=T, widths=(128, 128),
                 rng_state=x0)
    tr.set_params(POLICY, init_policy(D, 128, 128, seed=7))
    tr.set_params(VALUE, init_value(B, D, seed=8))
    tr.iterate(its)
    rng = tr.buffer(BUF_RNG).astype(np.int64)
    m, a = 2147483647, 16807
    base = 2 * N + 4 * T * N * its
    want = np.array([x0 * pow(a, base + 4 * T * e, m) % m for e in range(N)],
                    dtype=np.int64)
    np.testing.assert_array_equal(rng, want)


@pytest.mark.parametrize("algo,N,B,D,T", [("ppo", 32768, 64, 2, 4),
                                         ("ac", 16384, 128, 3, 8)])
def test_wave_rollout_matches_4wave(ctx, monkeypatch, algo, N, B, D, T):
    """Full config-3 / config-5 size: the wave-per-env rollouts (default at
    B=64 and B=128, [128,128]) and the 4-wave rollouts (XH_ROLLOUT_KERNEL=4)
    produce the same trajectories (actions, states, items, dones) and RNG
    states on the same parameters; logits / probabilities agree to the last
    place."""
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_BINS, BUF_DONE,
                                                BUF_ITEMS, BUF_LOGITS, BUF_POLD,
                                                BUF_PROBS, BUF_RNG)
    pp, vp = init_policy(D, 128, 128, seed=11), init_value(B, D, seed=12)
    bufs = (BUF_ACTION, BUF_BINS, BUF_DONE, BUF_ITEMS, BUF_LOGITS, BUF_POLD,
            BUF_PROBS, BUF_RNG)
    got = {}
    for kern in ("wave", "4"):
        # the f32-MFMA wave kernel (at 64 bins the default rollout is the
        # bf16-split one: test_split_rollout_matches_f32)
        monkeypatch.setenv("XH_ROLLOUT_KERNEL", "4" if kern == "4" else "f32")
        tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                     widths=(128, 128), rng_state=99, record_last_step=True)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        tr.rollout()
        got[kern] = [tr.buffer(b).copy() for b in bufs]
        tr.close()
    exact = (BUF_ACTION, BUF_BINS, BUF_DONE, BUF_ITEMS, BUF_RNG)
    for b, x, y in zip(bufs, got["wave"], got["4"]):
        if b in exact:
            np.testing.assert_array_equal(x, y, err_msg="buffer %d" % b)
        else:  # ~0.03% of the logits differ in the last place
            np.testing.assert_allclose(x, y, rtol=2e-6, atol=1e-7,
                                       err_msg="buffer %d" % b)


@pytest.mark.gpu
@pytest.mark.parametrize("algo,N,B,D,T,items", [
    ("ppo", 4096, 32, 1, 4, ([4], [1])),                    # BASELINE config 2
    ("ac", 16384, 128, 3, 8, ([4, 2, 2], [1, 2, 1])),      # config 5 per GPU
])
def test_other_configs_full_size_properties(ctx, algo, N, B, D, T, items):
    """BASELINE configs 2 and 5 at their per-GPU sizes: env transition
    invariants on every env and step, probability normalisation, finite
    learner state, and bitwise run-to-run determinism (as config 3 above)."""
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_ADV, BUF_BINS,
                                                BUF_DONE, BUF_ITEMS, BUF_POLD)
    H = (64, 64) if B == 32 else (128, 128)
    pp, vp = init_policy(D, *H, seed=3), init_value(B, D, seed=4)

    def make():
        tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                     widths=H, rng_state=777)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        return tr

    tr = make()
    tr.iterate(1)
    tr.rollout()
    bins = tr.buffer(BUF_BINS).astype(np.int32).reshape(T + 1, N, B, D)
    it = tr.buffer(BUF_ITEMS).reshape(T + 1, N, 4)[:, :, :D].astype(np.int32)
    act = tr.buffer(BUF_ACTION).reshape(T, N)
    done = tr.buffer(BUF_DONE).reshape(T, N)
    assert bins.min() >= 0 and bins.max() <= 8
    assert act.min() >= 0 and act.max() < B
    ok = (it == items[0]).all(-1) | (it == items[1]).all(-1)
    assert ok.all()
    idx = np.arange(N)
    for t in range(T):
        nxt = bins[t].copy()
        nxt[idx, act[t]] -= it[t]
        over = (nxt[idx, act[t]] < 0).any(-1)
        np.testing.assert_array_equal(over.astype(np.uint8), done[t])
        np.testing.assert_array_equal(bins[t + 1][~over], nxt[~over])
        assert (bins[t + 1][over] == 8).all()
    pold = tr.buffer(BUF_POLD)
    assert (pold > 0).all() and (pold <= 1).all()
    tr.learn()
    p1 = tr.params(POLICY)
    assert np.isfinite(p1).all() and np.isfinite(tr.params(VALUE)).all()
    assert np.isfinite(tr.buffer(BUF_ADV)).all()
    tr2 = make()
    tr2.iterate(2)
    np.testing.assert_array_equal(tr2.params(POLICY), p1)


def test_bench_json_line(tmp_path):
    """bench.py end to end at a small size: one JSON line with the driver's
    keys, the roofline / HBM objects, and whole-job arithmetic."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run(
        [sys.executable, os.path.join(repo, "bench.py"), "--steps", "2",
         "--warmup", "1", "--envs", "256", "--no-cpu-baseline"],
        capture_output=True, text=True, timeout=110, check=True, cwd=repo)
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup",
              "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
              "dtype", "data", "config", "roofline", "hbm_roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["scaling"] == "weak"
    assert d["config"]["envs_per_gpu"] == 256
    # value = env-steps / time: 256 envs x T=4 per step
    assert abs(d["value"] * d["ms_per_step"] / 1e3 - 256 * 4) < 1e-3 * 256 * 4 + 1
    r = d["roofline"]
    # the config-3 train kernel: f16 pairs in layer 2 / dH1, the bf16 split
    # in dW2 (peak = dense 2500 / (8/3)), as the library reports it
    assert r["bound"] == "mfma" and 0 < r["frac"] < 1 and r["peak"] == 937.5
    assert r["math"] == "f16_pair_bf16_split" and r["math_source"] == "xh_trainer_kernel_info"
    assert 0 < d["iteration_roofline"]["frac"] < 1


def _c3_health_run(ctx, iters, **kw):
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import BUF_ADV
    N, B, D, T = 32768, 64, 2, 4
    tr = Trainer(ctx, bins=B, dims=D, num_envs=N, steps=T, widths=(128, 128),
                 rng_state=20241008, record_last_step=True, **kw)
    tr.set_params(POLICY, init_policy(D, 128, 128, seed=0))
    tr.set_params(VALUE, init_value(B, D, seed=1))
    log = []
    for k in range(iters // 5):
        tr.iterate(5)
        h = tr.health()
        h["finite"] = h["finite"] and bool(np.isfinite(tr.buffer(BUF_ADV)).all())
        log.append((5 * (k + 1), h))
    tr.close()
    return log


def test_c3_numerics_over_bench_length(ctx):
    """The bench workload (BASELINE config 3 with lr_scale_rows, the
    documented opt-in the bench runs) stays numerically healthy over 25
    iterations: finite parameters, probabilities and advantages after every
    5, and real episodes (mean length between 1 step and the longest
    possible episode)."""
    log = _c3_health_run(ctx, 25, lr_scale_rows=True)
    for it, h in log:
        assert h["finite"], (it, h)
        assert h["done_rate"] > 0 and 1.0 <= h["mean_episode_len"] <= 64 * 8 * 2 + 1, (it, h)
    print("lr_scale_rows: (iteration, mean episode length, max prob)",
          [(it, round(h["mean_episode_len"], 2), round(h["max_prob"], 4))
           for it, h in log])


def test_c3_reference_lr_on_row_sums_diverges(ctx):
    """Why the bench needs lr_scale_rows: the reference applies the raw lr
    to gradients SUMMED over the batch rows (nn.h:94-98, 624) and its softmax
    has no max shift (nn.h:382-392).  At 131072 env-steps x 64 bins per
    batch that step is ~10^4 x the reference drivers' and the policy's
    probabilities turn non-finite within 25 iterations; health() detects it
    (the bench reports it as `health.finite`)."""
    log = _c3_health_run(ctx, 25)
    first = next((it for it, h in log if not h["finite"]), None)
    print("reference semantics: first non-finite check at iteration", first,
          [(it, h["finite"]) for it, h in log])
    assert first is not None


@pytest.mark.parametrize("algo,B,D,N,T,widths", [("ppo", 64, 2, 160, 4, (128, 128)),
                                                ("ac", 128, 3, 24, 8, (128, 128)),
                                                ("ppo", 32, 1, 768, 4, (64, 64))])
def test_split_train_kernel_accuracy(ctx, monkeypatch, algo, B, D, N, T, widths):
    """The config-3, config-5 and config-2 train kernels run their GEMMs on
    exactly split operands (f16 pairs for layer 2 and dH1, the three-part
    bf16 split for dW2; csrc/xh_split.h).  Their policy gradients stay
    within the stated row-summed bound and within a small factor of the
    f32-MFMA kernel's distance to the oracle's double-precision sums on the
    same batch (several row groups per workgroup), error per entry in units
    of u * sum|terms| (round 2, config 3: max 435 vs 272, median 0.37 vs 0.18
    -- both under one rounding unit of the terms' magnitude, against a bound
    of n + 8 = 40968 units)."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import BUF_POLICY_GRADS
    x0 = 24681357
    pp = init_policy(D, *widths, seed=11)
    vp = init_value(B, D, seed=12)
    orc = _oracle_trainer(B, D, N, T, widths, pp, vp, x0, algo)
    orc.rollout()
    orc.learn()
    ref = orc.buf(po.BUF_POLICY_GRADS)
    mag = orc.buf(po.BUF_POLICY_GRADS_MAG)
    ratios = {}
    # the superseded split forms live in the variant library only
    # (`make variants`); the product library has the default and f32 kernels
    kernels = ("f32", "split")
    for kernel in kernels:
        if kernel != "split":
            monkeypatch.setenv("XH_TRAIN_KERNEL", kernel)
        else:
            monkeypatch.delenv("XH_TRAIN_KERNEL", raising=False)
        tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                     widths=widths, rng_state=x0)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        tr.rollout()
        tr.learn()
        g = tr.buffer(BUF_POLICY_GRADS).ravel().astype(np.float64)
        tr.close()
        assert_grad_close(g, ref, mag, n_terms=N * T * B, what=kernel)
        units = np.abs(g - ref) / np.maximum(mag * 2.0 ** -24, 1e-30)
        ratios[kernel] = (float(units.max()), float(np.median(units[mag > 0])))
    print("policy-gradient error in u * sum|terms| (max, median):", ratios)
    for k in kernels[1:]:
        assert ratios[k][0] <= 3 * ratios["f32"][0] + 8, ratios
        assert ratios[k][1] <= 3 * ratios["f32"][1] + 1, ratios


@pytest.mark.parametrize("algo,N,B,D,T", [("ppo", 32768, 64, 2, 4),
                                         ("ac", 16384, 128, 3, 8),
                                         ("ppo", 4096, 32, 1, 4)])
def test_split_rollout_matches_f32(ctx, monkeypatch, algo, N, B, D, T):
    """Config-3 / config-5 / config-2 size: the default 64-, 128- and 32-bin
    rollouts run layer 2 on the f16 matrix cores with exactly split f32
    operands (rollout_split_kernel, all T slots in one launch, /
    rollout_split128_kernel).
    Teacher-forced with the f32 wave kernel's actions, it reproduces the
    states, items, dones and RNG streams bit for bit and the logits /
    probabilities / p_old within f32-class rounding; free-running, it picks
    the same action at all but a rare near-tie."""
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_BINS, BUF_DONE,
                                                BUF_ITEMS, BUF_LOGITS, BUF_POLD,
                                                BUF_PROBS, BUF_RNG)
    H = (64, 64) if B == 32 else (128, 128)
    pp, vp = init_policy(D, *H, seed=21), init_value(B, D, seed=22)
    bufs = (BUF_ACTION, BUF_BINS, BUF_DONE, BUF_ITEMS, BUF_LOGITS, BUF_POLD,
            BUF_PROBS, BUF_RNG)

    def run(kernel, forced=None):
        if kernel == "f32":
            monkeypatch.setenv("XH_ROLLOUT_KERNEL", "f32")
        else:
            monkeypatch.delenv("XH_ROLLOUT_KERNEL", raising=False)
        tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                     widths=H, rng_state=77, record_last_step=True)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        if forced is not None:
            tr.set_forced_actions(forced)
        tr.rollout()
        out = {b: tr.buffer(b).copy() for b in bufs}
        tr.close()
        return out

    ref = run("f32")
    free = run("split")
    forced = run("split", forced=ref[BUF_ACTION])
    for b in (BUF_ACTION, BUF_BINS, BUF_DONE, BUF_ITEMS, BUF_RNG):
        np.testing.assert_array_equal(forced[b], ref[b], err_msg="buffer %d" % b)
    for b in (BUF_LOGITS, BUF_PROBS, BUF_POLD):
        np.testing.assert_allclose(forced[b], ref[b], rtol=2e-5, atol=1e-7,
                                   err_msg="buffer %d" % b)
    diff = free[BUF_ACTION] != ref[BUF_ACTION]
    mism = int(diff.sum())
    envs = int(diff.any(0).sum())  # an env diverges from its first mismatch on
    print("free-running split vs f32 rollout: %d of %d actions differ (%d envs)"
          % (mism, ref[BUF_ACTION].size, envs))
    log_record("sampling_agreement.jsonl", {
        "test": "split_vs_f32_rollout", "algo": algo, "N": N, "B": B, "D": D,
        "T": T, "actions": int(ref[BUF_ACTION].size), "differ": mism,
        "envs_differ": envs})
    assert mism <= 1e-4 * ref[BUF_ACTION].size
