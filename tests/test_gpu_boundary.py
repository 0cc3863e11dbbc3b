"""Boundary checks of the C ABI that need a device: input validation of the
state setters and the kernel report (xh_trainer_kernel_info)."""
import numpy as np
import pytest

from conftest import HEADLINE_TRAIN_KERNEL

pytestmark = pytest.mark.gpu


def _trainer(ctx, B=64, D=2, N=64, T=4, widths=(128, 128)):
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    tr = Trainer(ctx, bins=B, dims=D, num_envs=N, steps=T, widths=widths,
                 rng_state=11)
    tr.set_params(POLICY, init_policy(D, *widths, seed=1))
    tr.set_params(VALUE, init_value(B, D, seed=2))
    return tr


def test_learn_refuses_items_outside_the_item_table(ctx):
    """The train kernels fold the item's layer-1 contribution into
    per-item-table-entry biases, so a batch slot holding any other item is
    refused by learn() (XH_ERR_STATE) instead of being trained as item_b;
    rollouts from such a slot still run, and a rollout's own items (drawn from
    the table) make the later slots valid again."""
    from dependence_free_rl_amd import XhError
    from dependence_free_rl_amd.trainer import BUF_ITEMS
    tr = _trainer(ctx)
    tr.rollout()
    tr.learn()
    items = tr.buffer(BUF_ITEMS).copy()
    items[0, 5, :2] = (3, 3)  # not {4,2} / {1,2}
    tr.set_buffer(BUF_ITEMS, items)
    with pytest.raises(XhError, match="item-table entry"):
        tr.learn()
    items[0, 5, :2] = (4, 2)
    tr.set_buffer(BUF_ITEMS, items)
    tr.learn()
    with pytest.raises(XhError):  # item values outside [0, capacity]
        items[1, 0, 0] = -1
        tr.set_buffer(BUF_ITEMS, items)
    tr.close()


def test_state_setters_reject_out_of_range_bins(ctx):
    """Bin values above the capacity are refused by set_env_state,
    set_buffer(BINS) and the venv's BINS.  Every negative int8 value stays
    legal: an apply by hand past game over keeps subtracting
    (bin_packing.h:53-63), so -4, -8, -12, ... are reachable states the
    drop-in layer uploads (tests/compat/bound_env_by_hand.cc)."""
    from dependence_free_rl_amd import VecEnv, XhError
    from dependence_free_rl_amd.trainer import BUF_BINS
    tr = _trainer(ctx)
    bins, items = tr.env_state(0, 2)
    bad = bins.copy()
    bad[1, 3, 0] = 9
    with pytest.raises(XhError, match="above the capacity"):
        tr.set_env_state(0, bad, items)
    bad[1, 3, 0] = -12  # overflowed twice: accepted
    tr.set_env_state(0, bad, items)
    b = tr.buffer(BUF_BINS).copy()
    b[0, 0, 0, 1] = 9
    with pytest.raises(XhError, match="above the capacity"):
        tr.set_buffer(BUF_BINS, b)
    b[0, 0, 0, 1] = -100
    tr.set_buffer(BUF_BINS, b)
    tr.close()
    env = VecEnv(ctx, num_envs=8, bins=8, dims=2, rng_state=1)
    vb, _ = env.view()
    vb[2, 1, 1] = 10
    with pytest.raises(XhError, match="above the capacity"):
        env.set(3, vb)  # VENV_BINS
    vb[2, 1, 1] = -100
    env.set(3, vb)
    env.close()


@pytest.mark.parametrize("B,D,algo", [(64, 2, "ppo"), (128, 3, "ac")])
def test_overflowed_start_states_run_the_f32_kernels(ctx, monkeypatch, B, D,
                                                     algo):
    """A start state with a bin below -capacity (|bins / capacity| > 1, beyond
    the f16-pair kernels' H1 bound) is rolled out and
    learned by the f32-MFMA kernels: the iteration equals, bit for bit, the
    same iteration run with XH_TRAIN_KERNEL=f32 XH_ROLLOUT_KERNEL=f32, and the
    next iteration (states >= 0 again) is back on the f16-pair kernels."""
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_BINS,
                                                BUF_POLICY_GRADS, BUF_PROBS)
    # T = 1: the whole batch is the overflowed slot 0
    N, T, widths = 16, 1, (128, 128)
    pp, vp = init_policy(D, *widths, seed=5), init_value(B, D, seed=6)

    def run(f32):
        if f32:
            monkeypatch.setenv("XH_TRAIN_KERNEL", "f32")
            monkeypatch.setenv("XH_ROLLOUT_KERNEL", "f32")
        else:
            monkeypatch.delenv("XH_TRAIN_KERNEL", raising=False)
            monkeypatch.delenv("XH_ROLLOUT_KERNEL", raising=False)
        tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                     widths=widths, rng_state=77, record_last_step=True)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        bins, items = tr.env_state()
        bins[3, 7, 0] = -20   # overflowed (game over) start states
        bins[9, 0, :] = -128
        tr.set_env_state(0, bins, items)
        tr.rollout()
        tr.learn()
        out = {b: tr.buffer(b).copy()
               for b in (BUF_ACTION, BUF_BINS, BUF_POLICY_GRADS, BUF_PROBS)}
        out["params"] = tr.params(POLICY)
        out["kinfo"] = tr.kernel_info()
        tr.rollout()
        tr.learn()
        out["kinfo2"] = tr.kernel_info()
        tr.close()
        return out

    wide, ref = run(False), run(True)
    f32_train = "policy_train8_kernel"
    assert wide["kinfo"]["policy_train"]["kernel"] == f32_train, wide["kinfo"]
    assert wide["kinfo2"]["policy_train"]["kernel"] != f32_train, wide["kinfo2"]
    assert wide["kinfo2"]["policy_train"]["math"] == "f16_pair_bf16_split"
    assert (wide[BUF_BINS][0] < -8).any()
    for k in (BUF_ACTION, BUF_BINS, BUF_POLICY_GRADS, BUF_PROBS, "params"):
        np.testing.assert_array_equal(wide[k], ref[k], err_msg=str(k))
    assert np.isfinite(wide["params"]).all()


@pytest.mark.parametrize("kind", ["bin", "item"])
@pytest.mark.parametrize("B,D,widths", [(64, 2, (128, 128)), (32, 1, (64, 64)),
                                        (128, 3, (128, 128))])
def test_wide_slot0_then_register_stepping(ctx, monkeypatch, B, D, widths, kind):
    """T = 4 with a slot 0 the split rollouts cannot take -- an overflowed
    bin, or an item outside the item table (they fold the item into
    per-entry biases): slot 0 runs on the f32 rollout, slots 1-3 in one
    launch of the register-stepping split kernel.  Teacher-forced with the
    all-f32 run's actions, every state, item, done and RNG state is
    bit-identical to that run, and p_old agrees to f32 rounding."""
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_BINS, BUF_DONE,
                                                BUF_ITEMS, BUF_POLD, BUF_RNG)
    N, T = 64, 4
    pp, vp = init_policy(D, *widths, seed=15), init_value(B, D, seed=16)

    def run(f32, forced=None):
        if f32:
            monkeypatch.setenv("XH_ROLLOUT_KERNEL", "f32")
        else:
            monkeypatch.delenv("XH_ROLLOUT_KERNEL", raising=False)
        tr = Trainer(ctx, algo="ppo", bins=B, dims=D, num_envs=N, steps=T,
                     widths=widths, rng_state=91)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        if kind == "bin":
            bins, items = tr.env_state()
            bins[5, 3, 0] = -40
            tr.set_env_state(0, bins, items)
        else:
            it = tr.buffer(BUF_ITEMS).copy()
            it[0, 5, :D] = 3  # not an item-table entry
            tr.set_buffer(BUF_ITEMS, it)
        if forced is not None:
            tr.set_forced_actions(forced)
        tr.rollout()
        out = {b: tr.buffer(b).copy()
               for b in (BUF_ACTION, BUF_BINS, BUF_DONE, BUF_ITEMS, BUF_POLD, BUF_RNG)}
        out["kinfo"] = tr.kernel_info()
        tr.close()
        return out

    ref = run(True)
    got = run(False, forced=ref[BUF_ACTION])
    assert got["kinfo"]["rollout_step"]["kernel"] == (
        "rollout_split128_kernel" if B == 128 else "rollout_split_kernel")
    for b in (BUF_ACTION, BUF_BINS, BUF_DONE, BUF_ITEMS, BUF_RNG):
        np.testing.assert_array_equal(got[b], ref[b], err_msg="buffer %d" % b)
    np.testing.assert_allclose(got[BUF_POLD], ref[BUF_POLD], rtol=2e-5, atol=1e-7)


def test_env_overrides_of_many_envs(ctx):
    """xh_trainer_set_env_state for every env (one run of consecutive envs)
    and for scattered envs: the next rollout starts from exactly those
    states."""
    from dependence_free_rl_amd.trainer import BUF_BINS, BUF_ITEMS
    N = 256
    tr = _trainer(ctx, N=N)
    tr.rollout()
    tr.learn()
    bins, items = tr.env_state(0, N)
    rng = np.random.default_rng(0)
    nb = rng.integers(0, 9, size=bins.shape).astype(np.int8)
    ni = np.where(rng.random(N)[:, None] < 0.5, [[4, 2]], [[1, 2]]).astype(np.int8)
    tr.set_env_state(0, nb, ni)
    # scattered overrides on top: envs 3, 4, 5 and 200
    for e in (3, 4, 5, 200):
        nb[e] = 8 - nb[e]
        tr.set_env_state(e, nb[e:e + 1], ni[e:e + 1])
    tr.rollout()
    np.testing.assert_array_equal(tr.buffer(BUF_BINS)[0], nb)
    np.testing.assert_array_equal(tr.buffer(BUF_ITEMS)[0, :, :2], ni)
    tr.close()


@pytest.mark.parametrize("B,D,widths,train,roll,prod,f32_train", [
    (64, 2, (128, 128), HEADLINE_TRAIN_KERNEL, "rollout_split_kernel", 8.0 / 3.0,
     "policy_train8_kernel"),
    # config 2's shape: the split train kernel and the split rollout (two
    # envs per wave)
    (32, 1, (64, 64), "policy_train_split4h_kernel", "rollout_split_kernel", 8.0 / 3.0,
     "policy_train_kernel"),
    (8, 2, (128, 64), None, None, None, None),
])
def test_kernel_info_names_what_ran(ctx, monkeypatch, B, D, widths, train, roll,
                                    prod, f32_train):
    """xh_trainer_kernel_info reports the kernels the last rollout step and
    policy epoch launched, their arithmetic and its MFMA peak; an override
    variable shows up in the report and changes what runs."""
    tr = _trainer(ctx, B=B, D=D, widths=widths)
    k = tr.kernel_info()
    assert k["policy_train"]["kernel"] is None  # nothing launched yet
    tr.rollout()
    tr.learn()
    k = tr.kernel_info()
    kt, kr = k["policy_train"], k["rollout_step"]
    if train:
        assert kt["kernel"] == train and kr["kernel"] == roll
        # f16 pairs in layer 2 (three products) and dH1 (two), the bf16
        # split in dW2 (three): 8 MFMA products per 3 f32 products
        assert kt["math"] == "f16_pair_bf16_split"
        assert kt["products_per_f32_product"] == pytest.approx(prod, rel=1e-5)
        assert kt["peak_tflops"] == pytest.approx(2500.0 / prod, rel=1e-5)
        if roll.startswith("rollout_split"):
            assert kr["math"] == "f16_pair"
            assert kr["peak_tflops"] == pytest.approx(2500.0 / 3)
        else:
            assert kr["math"] == "f32_mfma"
    else:
        assert kt["math"] == "f32_mfma" and kt["peak_tflops"] == 157.3
        assert kt["kernel"].startswith("policy_train")
    assert k["overrides"] == {"XH_TRAIN_KERNEL": None, "XH_ROLLOUT_KERNEL": None,
                            "XH_VALUE_KERNEL": None}
    assert k["value"] == "vnet_bf16"
    tr.close()
    if train:
        monkeypatch.setenv("XH_TRAIN_KERNEL", "f32")
        tr = _trainer(ctx, B=B, D=D, widths=widths)
        tr.rollout()
        tr.learn()
        k = tr.kernel_info()
        assert k["overrides"]["XH_TRAIN_KERNEL"] == "f32"
        assert k["policy_train"]["math"] == "f32_mfma"
        assert k["policy_train"]["kernel"] == f32_train
        tr.close()
