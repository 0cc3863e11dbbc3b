"""GPU parity of the vectorised env boundary (xh_venv_*, include/xylo_hip.h):
a caller's own actions step N bp::environment instances on the device.

Bit-exact against the reference's env8 golden (3000 steps of the real
bp::environment + random_policy) and against the oracle's sequential
reference-order driver (or_venv_run) at the full BASELINE config-3 shape
(32768 envs x 64 bins x 2-D)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _venv(ctx, **kw):
    from dependence_free_rl_amd import VecEnv
    return VecEnv(ctx, **kw)


@pytest.mark.parametrize("B", [8, 64, 128])
def test_venv_replays_reference_env8(ctx, B):
    """One env, the reference's 3000 random-policy choices: every state,
    item, reward and the final engine state equal the real reference's.  At
    64 / 128 bins the choices land on 8 random distinct bins (the benchmark
    shapes; the reference env has 8): those bins follow the reference's, the
    others stay full (the same check the harness makes of gen_env<64|128,2>,
    oracle/ref_harness.cc envcheck_injected)."""
    from dependence_free_rl_amd._lib import VENV_RNG
    g = golden("env8")
    slot = (np.arange(8) if B == 8 else
            np.random.default_rng(B).permutation(B)[:8])
    env = _venv(ctx, num_envs=1, bins=B, dims=2, rng_state=int(g["x0"][0]),
                policy_draws=2)

    def placed(b8):
        full = np.full((B, 2), 8, dtype=b8.dtype)
        full[slot] = b8
        return full

    n = len(g["choice"])
    for k in range(n):
        bins, item = env.view()
        np.testing.assert_array_equal(bins[0], placed(g["start_bins"][k]))
        np.testing.assert_array_equal(item[0], g["start_item"][k])
        env.set_actions([slot[g["choice"][k]]])
        reward, done = env.step()
        assert reward[0] == g["reward"][k] and done[0] == (g["reward"][k] == 0)
        if not done[0]:
            np.testing.assert_array_equal(env.view()[0][0],
                                          placed(g["end_bins"][k]))
    assert env.get(VENV_RNG)[0] == int(g["x_end"][0])
    env.close()


@pytest.mark.parametrize("B,D,N,offset,Ng", [(64, 2, 32768, 0, 32768),
                                            (64, 2, 4096, 8192, 32768),
                                            (128, 3, 2048, 0, 2048),
                                            (32, 1, 4096, 0, 4096),
                                            (8, 2, 1000, 0, 1000)])
def test_venv_matches_reference_order_driver(ctx, B, D, N, offset, Ng):
    """External (random) actions at full size: states, items, rewards, dones
    after every step and the engine positions equal the sequential driver
    stepping the Ng agents in env order on one engine."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd._lib import VENV_DONE, VENV_REWARD, VENV_RNG
    S, x0 = 5, 4242
    rng = np.random.default_rng(B * 7 + D)
    acts = rng.integers(0, B, size=(S, N)).astype(np.int32)
    # every other env packs into its first 3 bins, so overflows / resets
    # happen often
    acts[:, ::2] = rng.integers(0, 3, size=(S, (N + 1) // 2))
    ref = po.venv_run(B, D, N, x0, acts, policy_draws=2, n_global=Ng,
                      offset=offset)
    env = _venv(ctx, num_envs=N, bins=B, dims=D, rng_state=x0,
                env_offset=offset, num_envs_global=Ng, policy_draws=2)
    for s in range(S):
        bins, item = env.view()
        np.testing.assert_array_equal(bins, ref["bins"][s])
        np.testing.assert_array_equal(item, ref["item"][s])
        env.set_actions(acts[s])
        env.step(fetch=False)
        np.testing.assert_array_equal(env.get(VENV_REWARD), ref["reward"][s])
        np.testing.assert_array_equal(env.get(VENV_DONE), ref["done"][s])
    bins, item = env.view()
    np.testing.assert_array_equal(bins, ref["bins"][S])
    np.testing.assert_array_equal(item, ref["item"][S])
    assert ref["done"].sum() > 0  # resets were exercised
    if offset == 0:  # env 0 stands where the sequential engine ended
        assert env.get(VENV_RNG)[0] == ref["x_end"]
    env.close()


def test_venv_observation_layout(ctx):
    """observe() and step(write_obs) = observation::to_vector per env."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd._lib import VENV_OBS
    B, D, N = 16, 3, 256
    env = _venv(ctx, num_envs=N, bins=B, dims=D, rng_state=11)
    rng = np.random.default_rng(5)
    cfg = po.env_cfg(B, D)
    for s in range(4):
        env.set_actions(rng.integers(0, B, N))
        env.step(write_obs=True, fetch=False)
        obs_step = env.get(VENV_OBS)
        obs = env.observe()
        np.testing.assert_array_equal(obs, obs_step)
        bins, item = env.view()
        for e in (0, 17, N - 1):
            want = np.zeros(B * 2 * D, np.float32)
            b32 = np.ascontiguousarray(bins[e], np.int32)
            i32 = np.zeros(3, np.int32)
            i32[:D] = item[e]
            po.lib().or_obs(po.C.byref(cfg), po._ptr(b32), po._ptr(i32),
                            po._ptr(want))
            np.testing.assert_array_equal(obs[e].reshape(-1), want)
    env.close()


@pytest.mark.parametrize("B,D", [(8, 2), (128, 3)])
def test_venv_apply_reset_masks(ctx, B, D):
    """environment::apply / reset on masked subsets: each env draws from its
    own stream where it stands, exactly as the oracle env does; apply leaves
    an overflowed env un-reset (game_over reported, no item drawn)."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd._lib import VENV_DONE, VENV_RNG
    N = 64
    env = _venv(ctx, num_envs=N, bins=B, dims=D, rng_state=77, policy_draws=0)
    cfg = po.env_cfg(B, D)
    rng = np.random.default_rng(B + D)
    bins, item = env.view()
    xs = env.get(VENV_RNG).astype(np.uint32)
    st = [(np.ascontiguousarray(bins[e], np.int32),
           np.concatenate([item[e], np.zeros(3 - D, np.int8)]).astype(np.int32))
          for e in range(N)]
    for it in range(12):
        mask = (rng.random(N) < 0.5).astype(np.uint8)
        if it % 3 == 2:
            env.reset(mask)
            for e in np.nonzero(mask)[0]:
                x = po.C.c_uint32(int(xs[e]))
                po.lib().or_env_reset(po.C.byref(cfg), po._ptr(st[e][0]),
                                      po._ptr(st[e][1]), po.C.byref(x))
                xs[e] = x.value
            continue
        acts = rng.integers(0, B, N).astype(np.int32)
        env.set_actions(acts)
        done = env.apply(mask)
        assert (done[mask == 0] == 0).all()  # only this call's verdicts
        for e in np.nonzero(mask)[0]:
            x = po.C.c_uint32(int(xs[e]))
            po.lib().or_env_apply(po.C.byref(cfg), po._ptr(st[e][0]),
                                  po._ptr(st[e][1]), int(acts[e]), po.C.byref(x))
            xs[e] = x.value
            assert done[e] == int((st[e][0] < 0).any())
        bins, item = env.view()
        for e in range(N):
            np.testing.assert_array_equal(bins[e], st[e][0])
            np.testing.assert_array_equal(item[e], st[e][1][:D])
        np.testing.assert_array_equal(env.get(VENV_RNG), xs)
    env.close()


def test_venv_rejects_out_of_range_actions(ctx):
    from dependence_free_rl_amd import XhError
    env = _venv(ctx, num_envs=8, bins=8, dims=2, rng_state=1)
    with pytest.raises(XhError):
        env.set_actions([0, 1, 2, 3, 4, 5, 6, 8])
    env.close()


def test_trainer_env_state_round_trip(ctx):
    """xh_trainer_get/set_env_state: the states the next rollout starts from
    (the batch's final states after learn()); a replaced state is where that
    env's next rollout starts, and the learner's batch is untouched."""
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import BUF_ADV, BUF_BINS, BUF_ITEMS
    B, D, N, T = 64, 2, 64, 4
    tr = Trainer(ctx, bins=B, dims=D, num_envs=N, steps=T, widths=(128, 128),
                 rng_state=9)
    tr.set_params(POLICY, init_policy(D, 128, 128, seed=1))
    tr.set_params(VALUE, init_value(B, D, seed=2))
    bins0, items0 = tr.env_state()
    np.testing.assert_array_equal(bins0, tr.buffer(BUF_BINS)[0])
    tr.rollout()
    batch = tr.buffer(BUF_BINS)
    nb = np.full((2, B, D), 8, np.int8)
    nb[0, 5] = (1, 3)
    ni = np.array([[1, 2], [4, 2]], np.int8)
    tr.set_env_state(10, nb, ni)        # pending until the next rollout
    b, i = tr.env_state(10, 2)
    np.testing.assert_array_equal(b, nb)
    np.testing.assert_array_equal(i, ni)
    tr.learn()                          # reads the untouched batch
    np.testing.assert_array_equal(tr.buffer(BUF_BINS), batch)
    b, i = tr.env_state()
    want_b = batch[T].copy()
    want_b[10:12] = nb
    np.testing.assert_array_equal(b, want_b)
    tr.rollout()
    np.testing.assert_array_equal(tr.buffer(BUF_BINS)[0], want_b)
    np.testing.assert_array_equal(tr.buffer(BUF_ITEMS)[0, 10:12, :D], ni)
    assert np.isfinite(tr.buffer(BUF_ADV)).all()
    tr.close()


def test_trainer_env_state_rejects_mixed_items(ctx):
    """set_env_state takes whole item-table entries only: at D = 3 the item
    (4, 2, 1) passes a per-dimension check against (4, 2, 2) / (1, 2, 1) but
    is neither entry (the train kernels carry dW1's item columns as sums per
    table entry)."""
    from dependence_free_rl_amd import Trainer, XhError
    B, D, N = 128, 3, 8
    tr = Trainer(ctx, algo="ac", bins=B, dims=D, num_envs=N, steps=2,
                 widths=(128, 128), rng_state=3)
    nb = np.full((1, B, D), 8, np.int8)
    tr.set_env_state(0, nb, np.array([[1, 2, 1]], np.int8))  # item_b: fine
    with pytest.raises(XhError, match="item-table entry"):
        tr.set_env_state(0, nb, np.array([[4, 2, 1]], np.int8))
    tr.close()
