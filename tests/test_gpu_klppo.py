"""KL-PPO on the f16-pair train kernels (64, 128 and 32 bins), against the oracle.

kl_ppo_learner (/root/reference/xylo/policy_gradient.h:310-335) trains on
every row of its state matrix: the transitions, the open trajectories' end
rows and the terminal end rows (rl.h:336-343), with kl_regulated_loss
(policy_gradient.h:41-85) and beta adapted between epochs from the mean KL.
At the 64-bin 2-D [128,128] shape (BASELINE config 3's) the epoch runs
policy_train_spec8_kl_kernel, the KL-PPO build of the wave-specialised
headline train kernel (its round-4 predecessor policy_train_split8wh_kl_kernel
under XH_TRAIN_KERNEL=split8wh), at the 128-bin 3-D shape (config 5's) policy_train_split8x_kl_kernel
and at the 32-bin 1-D [64,64] shape (config 2's, two rows per 64-row group)
policy_train_split4h_kl_kernel (f16 pairs + the exact bf16 split, DESIGN.md
§3.0a-d).  Lockstep iterations: the oracle learns from the
device trainer's parameters each iteration, samples its own actions and the
device replays them, so the comparison measures one learn()'s arithmetic.
Several iterations carry the envs into terminal end rows (a 64-bin episode
ends when an item overflows its bin).  Epoch-0 gradients are held to the
tight budget (conftest), later epochs to the drift budget; beta (used and
after) must equal the oracle's, the mean KL within 1e-4.
"""
import numpy as np
import pytest

from conftest import GRAD_UNITS_P99_DRIFT, assert_close, assert_grad_units
from gpu_helpers import step_major

pytestmark = pytest.mark.gpu

KL_KERNEL = {64: "policy_train_spec8_kl_kernel", 128: "policy_train_split8x_kl_kernel",
             32: "policy_train_split4h_kl_kernel"}


@pytest.mark.parametrize("B,D,N,T,iters,cap,kernel",
                         [(64, 2, 48, 4, 5, 0, "split"), (64, 2, 32, 4, 4, 1, "split"),
                          (64, 2, 48, 4, 5, 0, "f32"), (64, 2, 48, 4, 5, 0, "split8wh"),
                          (128, 3, 24, 8, 5, 0, "split"), (128, 3, 24, 8, 5, 1, "split"),
                          (32, 1, 64, 4, 5, 0, "split"), (32, 1, 48, 4, 5, 1, "split"),
                          (32, 1, 64, 4, 5, 0, "f32")],
                         ids=["b64_n48", "b64_n32_cap1", "b64_n48_f32", "b64_n48_8wh", "b128_n24",
                              "b128_n24_cap1", "b32_n64", "b32_n48_cap1", "b32_n64_f32"])
def test_klppo_split_matches_oracle(ctx, monkeypatch, B, D, N, T, iters, cap, kernel):
    """kernel "f32": the same iterations on the f32-MFMA KL kernel
    (XH_TRAIN_KERNEL=f32), the accuracy reference the split kernel's logged
    error units are read against."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import BUF_KL, BUF_POLICY_GRADS
    widths, x0, wd = ((64, 64) if B == 32 else (128, 128)), 777001, 1e-5
    want = KL_KERNEL[B]
    if kernel == "f32":
        monkeypatch.setenv("XH_TRAIN_KERNEL", "f32")
        want = "policy_train_kernel<kl>"
    elif kernel == "split8wh":  # the round-4 KL build, kept for A/B
        monkeypatch.setenv("XH_TRAIN_KERNEL", "split8wh")
        want = "policy_train_split8wh_kl_kernel"
    pp, vp = init_policy(D, *widths, seed=61), init_value(B, D, seed=62)
    tr = Trainer(ctx, algo="klppo", bins=B, dims=D, num_envs=N, steps=T,
                 widths=widths, rng_state=x0, wd_policy=wd, train_grid_cap=cap)
    tr.set_params(POLICY, pp)
    tr.set_params(VALUE, vp)
    orc = po.Trainer(po.OR_KLPPO, B, D, N, T,
                     po.perbin_model(2 * D, list(widths), po.OR_SOFTMAX), pp,
                     po.full_model(B * 2 * D, [64, 32], 1), vp, wd_pi=wd, x0=x0)
    npi = tr.num_params(POLICY)
    terminal_rows = 0
    for it in range(iters):
        orc.set_params(0, tr.params(POLICY))
        orc.set_params(1, tr.params(VALUE))
        orc.rollout()
        tr.set_forced_actions(step_major(orc.buf(po.BUF_STEP_CHOICE), N, T))
        tr.rollout()
        tr.learn()
        orc.learn()
        k = tr.kernel_info()
        assert k["policy_train"]["kernel"] == want, k
        is_end = orc.buf(po.BUF_ROW_IS_END)
        rows = len(is_end)
        terminal_rows += int(rows - N * T - N) if rows > N * T + N else 0
        dev = tr.buffer(BUF_POLICY_GRADS).reshape(-1, npi)
        ref = np.asarray(orc.buf(po.BUF_POLICY_GRADS)).reshape(-1, npi)
        mag = np.asarray(orc.buf(po.BUF_POLICY_GRADS_MAG)).reshape(-1, npi)
        for ep in range(dev.shape[0]):
            budget = {} if ep == 0 else {"p99_units": GRAD_UNITS_P99_DRIFT}
            assert_grad_units(dev[ep], ref[ep], mag[ep],
                              what="klppo %s B%d N%d cap%d it%d epoch%d"
                                   % (kernel, B, N, cap, it, ep), **budget)
        okl = orc.buf(po.BUF_KL).reshape(-1, 3)
        gkl = tr.buffer(BUF_KL)
        np.testing.assert_array_equal(gkl[:, 0], okl[:, 0])   # beta used
        np.testing.assert_array_equal(gkl[:, 2], okl[:, 2])   # beta after
        assert_close(gkl[:, 1], okl[:, 1], what="mean KL it%d" % it)
        assert_close(tr.params(POLICY), orc.params(0), what="policy it%d" % it)
    # the batches reached the terminal end rows (E_t of ended trajectories)
    assert terminal_rows > 0, terminal_rows
    tr.close()


@pytest.mark.parametrize("B,D,widths", [(64, 2, (128, 128)), (128, 3, (128, 128))])
def test_recorded_distributions(ctx, B, D, widths):
    """record_distrib (the composed learner's q, rl.h:27-30) on the split
    rollouts: every step's distribution sums to 1, the last step's equals the
    probabilities output, and each step's p_old is its entry at the chosen
    bin."""
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import BUF_ACTION, BUF_POLD, BUF_PROBS, BUF_QOLD
    N, T = 32, 4
    tr = Trainer(ctx, algo="ac" if B == 128 else "ppo", bins=B, dims=D, num_envs=N,
                 steps=T, widths=widths, rng_state=99001, record_distrib=True,
                 record_last_step=True)
    tr.set_params(POLICY, init_policy(D, *widths, seed=71))
    tr.set_params(VALUE, init_value(B, D, seed=72))
    tr.rollout()
    q = tr.buffer(BUF_QOLD)
    assert q.shape == (T, N, B)
    np.testing.assert_allclose(q.sum(axis=2), 1.0, rtol=0, atol=1e-5)
    np.testing.assert_array_equal(q[T - 1], tr.buffer(BUF_PROBS))
    act = tr.buffer(BUF_ACTION)
    pold = tr.buffer(BUF_POLD)
    pick = np.take_along_axis(q, act[:, :, None].astype(np.int64), axis=2)[:, :, 0]
    np.testing.assert_array_equal(pick, pold)
    tr.close()
