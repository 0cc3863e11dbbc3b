"""BASELINE configs 4 and 5 as GLOBAL workloads on one device.

Config 4 is 262144 envs (64 bins, 2-D, [128,128], PPO, T=4) over 8 ranks of
32768; config 5 is 131072 envs (128 bins, 3-D, [128,128], actor-critic, T=8)
over 8 ranks of 16384.  A rank is a trainer with num_envs_global = 8n and
env_offset = r n; the only exchange between ranks is the SUM all-reduce of
the flat gradients (the reference's loss is a row sum, nn.h:94-98).  Here
the 8 rank trainers and one 8n-env trainer run side by side on one device:

* every rank's trajectories (states, items, actions, p_old, dones) are
  bit-identical to its slice of the 8n-env trainer's, and its advantages;
* every env's minstd_rand0 state sits at its reference-order position
  jump(x0, 2 Ng + 4 T Ng its + 4 T e) for e up to Ng - 1 (SURVEY App. B;
  the worker order of rl.h:325-349 run sequentially);
* the host sum of the 8 ranks' value and policy gradients (what
  ncclAllReduce forms) equals the 8n-env gradient up to fp32 summation
  order (no oracle at this size: relative L2 and worst-entry limits, the
  oracle-pinned check of the same kernels is tests/test_gpu_shards.py).

Learning rates are 0, so each epoch sees the same parameters on every side.

The full-size sampling check: a 256-env sample of the config-3 job
(32768 envs, reference-order streams) run through the oracle's sequential
sampler at two shard offsets picks the same actions as the device's
default (f16-pair) rollout.
"""
import numpy as np
import pytest

from conftest import log_record

pytestmark = pytest.mark.gpu

M31, A = 2147483647, 16807

# (relative L2, worst entry / max |g|) of the 8-rank sum against the 8n-env
# gradient, fp32 sums over 8n * T * B rows in two orders at the same slab
# depth.  About 3x the values measured (policy gradient, the larger of the two
# iterations; profiles/r05b_global_sums.jsonl: config 4 9.0e-5 / 1.8e-4,
# config 5 1.1e-4 / 2.2e-4; the value gradients agree to 2e-6)
GLOBAL_SUM_LIMITS = {64: (3e-4, 6e-4), 128: (4e-4, 7e-4)}


def _positions(x0, base, step, n):
    """x0 * A^(base + step * e) mod M31 for e in [0, n)."""
    out = np.empty(n, np.int64)
    x = x0 * pow(A, base, M31) % M31
    m = pow(A, step, M31)
    for e in range(n):
        out[e] = x
        x = x * m % M31
    return out


@pytest.mark.parametrize("cfg", [
    # BASELINE config 4: 262144 envs over 8 ranks of 32768 (= config 3 each)
    dict(name="config4", algo="ppo", B=64, D=2, n=32768, T=4, widths=(128, 128)),
    # BASELINE config 5: 131072 envs over 8 ranks of 16384
    dict(name="config5", algo="ac", B=128, D=3, n=16384, T=8,
         widths=(128, 128)),
])
def test_global_workload_8_ranks(ctx, cfg):
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_ADV, BUF_BINS,
                                                BUF_DONE, BUF_ITEMS, BUF_POLD,
                                                BUF_POLICY_GRADS, BUF_RNG,
                                                BUF_VALUE_GRAD)
    algo, B, D, n, T, widths = (cfg[k] for k in ("algo", "B", "D", "n", "T",
                                                 "widths"))
    W, x0 = 8, 20241008
    Ng = W * n
    pp, vp = init_policy(D, *widths, seed=41), init_value(B, D, seed=42)

    def make(num, off):
        tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=num, steps=T,
                     widths=widths, lr_policy=0.0, lr_value=0.0,
                     rng_state=x0, num_envs_global=Ng, env_offset=off)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        return tr

    full = make(Ng, 0)
    ranks = [make(n, r * n) for r in range(W)]
    # the 8n-env batch trains on 8x the workgroups of one rank, so that no
    # gradient slab sums more row groups than a rank's (the bench depth);
    # at 4096 groups per slab the f32 sums of the full batch drifted 2e-2
    # (relative L2) from the ranks' (profiles/r05a_global_sums.jsonl)
    for tr in [full] + ranks:
        tr.rollout()
        tr.learn()
    grid = [tr.kernel_info()["train_grid"] for tr in [full] + ranks]
    assert grid[0] == W * grid[1] and len(set(grid[1:])) == 1, grid
    full = make(Ng, 0)
    ranks = [make(n, r * n) for r in range(W)]
    for it in range(2):
        for tr in [full] + ranks:
            tr.rollout()
        for buf in (BUF_ACTION, BUF_POLD, BUF_BINS, BUF_ITEMS, BUF_DONE):
            f = full.buffer(buf)
            for r, tr in enumerate(ranks):
                np.testing.assert_array_equal(
                    f[:, r * n:(r + 1) * n], tr.buffer(buf),
                    err_msg="%s it%d rank %d buffer %d" % (cfg["name"], it, r, buf))
        rng = full.buffer(BUF_RNG).astype(np.int64)
        for r, tr in enumerate(ranks):
            np.testing.assert_array_equal(rng[r * n:(r + 1) * n],
                                          tr.buffer(BUF_RNG).astype(np.int64))
        # reference-order positions of every env of the job after it + 1
        # rollouts (each stream stored at its next iteration's first draw):
        # construction 2 Ng, then 4 T draws per env per iteration in env order
        want = _positions(x0 % M31, 2 * Ng + 4 * T * Ng * (it + 1), 4 * T, Ng)
        np.testing.assert_array_equal(rng, want)
        for tr in [full] + ranks:
            tr.learn()
        a = full.buffer(BUF_ADV)
        for r, tr in enumerate(ranks):
            np.testing.assert_array_equal(a[:, r * n:(r + 1) * n], tr.buffer(BUF_ADV))
        # the all-reduce's sum, formed on the host (float64 over the ranks)
        vg = sum(tr.buffer(BUF_VALUE_GRAD).astype(np.float64) for tr in ranks)
        vf = full.buffer(BUF_VALUE_GRAD).astype(np.float64)
        pg = sum(tr.buffer(BUF_POLICY_GRADS)[0].astype(np.float64) for tr in ranks)
        pf = full.buffer(BUF_POLICY_GRADS)[0].astype(np.float64)
        rec = {"config": cfg["name"], "it": it, "envs": Ng, "ranks": W}
        for what, g, f in (("value", vg, vf), ("policy", pg, pf)):
            rel = float(np.linalg.norm(g - f) / np.linalg.norm(f))
            worst = float(np.abs(g - f).max() / np.abs(f).max())
            rec[what] = {"rel_l2": rel, "worst_rel": worst}
        print(rec)
        log_record("global_sums.jsonl", rec)
        lim = GLOBAL_SUM_LIMITS[B]
        for what in ("value", "policy"):
            assert rec[what]["rel_l2"] <= lim[0], rec
            assert rec[what]["worst_rel"] <= lim[1], rec
    for tr in [full] + ranks:
        tr.close()


@pytest.mark.parametrize("off", [0, 32768 - 256])
def test_c3_full_size_sampling_vs_oracle(ctx, off):
    """The default config-3 rollout (rollout_split_kernel: layer 2 on f16
    pairs) at full size, free-running: envs [off, off + 256) of the 32768-env
    job against the oracle's sequential reference-order sampler
    (discrete_distribution on the model's probabilities, rl.h:27-30,
    tensor.cc:467-470) on the same streams.  Actions, states and dones match
    bit for bit, p_old within 1e-4.  An env whose sampled bin differs
    diverges from there on; it is allowed only as a PROVEN near-tie: at its
    first differing step (same state on both sides) the draw u, recomputed
    from the env's reference-order stream position, lies between the
    oracle's and the device's cumulative probability at the boundary they
    resolve differently, and those two differ by at most TIE_TOL = 1e-4 (the
    stated probability tolerance p_old is held to).  Anything else fails."""
    from oracle import pyoracle as po
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_BINS, BUF_DONE,
                                                BUF_POLD, BUF_QOLD)
    N, S, B, D, T, x0 = 32768, 256, 64, 2, 4, 1357911
    pp, vp = init_policy(D, 128, 128, seed=51), init_value(B, D, seed=52)
    tr = Trainer(ctx, bins=B, dims=D, num_envs=N, steps=T, widths=(128, 128),
                 rng_state=x0, record_distrib=True)
    tr.set_params(POLICY, pp)
    tr.set_params(VALUE, vp)
    tr.rollout()
    assert tr.kernel_info()["rollout_step"]["kernel"] == "rollout_split_kernel"
    act = tr.buffer(BUF_ACTION)[:, off:off + S]
    bins = tr.buffer(BUF_BINS)[:T, off:off + S]
    done = tr.buffer(BUF_DONE)[:, off:off + S]
    pold = tr.buffer(BUF_POLD)[:, off:off + S]
    q = tr.buffer(BUF_QOLD)[:, off:off + S]  # every sampled distribution
    tr.close()
    # the oracle sample: env i constructed at engine position 2 (off + i),
    # its step draws from 2 N + 4 T (off + i) on
    orc = po.Trainer(po.OR_PPO, B, D, S, T,
                     po.perbin_model(2 * D, [128, 128], po.OR_SOFTMAX), pp,
                     po.full_model(B * 2 * D, [64, 32], 1), vp,
                     x0=po.minstd_jump(x0, 2 * off))
    orc.set_stream_states([po.minstd_jump(x0, 2 * N + 4 * T * (off + i))
                           for i in range(S)])
    orc.rollout()
    o_act = orc.buf(po.BUF_STEP_CHOICE).reshape(S, T).T
    o_bins = orc.buf(po.BUF_STEP_BINS).reshape(S, T, B, D).swapaxes(0, 1)
    o_done = orc.buf(po.BUF_STEP_DONE).reshape(S, T).T
    o_pold = orc.buf(po.BUF_STEP_PCHOICE).reshape(S, T).T
    diff = act != o_act
    bad = diff.any(0)
    o_item = orc.buf(po.BUF_STEP_ITEM).reshape(S, T, -1).swapaxes(0, 1)
    from sampling_ties import near_tie
    ties = [near_tie(po, pp, B, D, N, T, x0, off + i, t, o_bins[t, i],
                      o_item[t, i], q[t, i], int(act[t, i]), int(o_act[t, i]))
            for i in np.flatnonzero(bad)
            for t in [int(np.flatnonzero(diff[:, i])[0])]]
    rec = {"test": "c3_full_size_vs_oracle", "offset": off, "envs": S,
           "actions": int(act.size), "differ": int(diff.sum()),
           "envs_differ": int(bad.sum()), "near_ties": ties}
    print(rec)
    log_record("sampling_agreement.jsonl", rec)
    for tie in ties:
        assert tie["proven"], rec
    ok = ~bad
    np.testing.assert_array_equal(act[:, ok], o_act[:, ok])
    np.testing.assert_array_equal(bins[:, ok], o_bins[:, ok])
    np.testing.assert_array_equal(done[:, ok], o_done[:, ok])
    err = np.abs(pold[:, ok] - o_pold[:, ok]) / np.maximum(1, np.abs(o_pold[:, ok]))
    assert err.max() <= 1e-4, float(err.max())
