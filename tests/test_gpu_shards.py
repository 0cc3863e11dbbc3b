"""The multi-GPU data path on one device.

Shards: two trainers owning envs [0, n) and [n, 2n) of a 2n-env job
(num_envs_global, env_offset) roll out exactly the corresponding halves of
the full trainer's trajectories (reference-order RNG positions), and their
per-shard gradients sum to the full batch's gradient -- the sum ncclAllReduce
forms across ranks.  Learning rates are 0 so every epoch sees the same
parameters.

RCCL: a one-rank communicator (world = 1 with a unique id) routes every
gradient through ncclAllReduce (1 value + k policy all-reduces per
iteration) and leaves the result bit-identical."""
import numpy as np
import pytest

from conftest import assert_close, assert_grad_close

pytestmark = pytest.mark.gpu



@pytest.mark.parametrize("n", [64, 16384])
def test_two_shards_sum_to_full_batch(ctx, n):
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ACTION, BUF_ADV, BUF_BINS,
                                                BUF_POLD, BUF_POLICY_GRADS,
                                                BUF_VALUE_GRAD)
    B, D, T = 8, 2, 4
    pp, vp = init_policy(D, 128, 64, seed=21), init_value(B, D, seed=22)

    def make(num, off):
        tr = Trainer(ctx, bins=B, dims=D, num_envs=num, steps=T,
                     widths=(128, 64), lr_policy=0.0, lr_value=0.0,
                     rng_state=31337, num_envs_global=2 * n, env_offset=off)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        return tr

    full, s0, s1 = make(2 * n, 0), make(n, 0), make(n, n)
    orc = None
    if n <= 64:  # the oracle's sum|terms| per entry states the fp32 bound
        from oracle import pyoracle as po
        orc = po.Trainer(po.OR_PPO, B, D, 2 * n, T,
                         po.perbin_model(2 * D, [128, 64], po.OR_SOFTMAX), pp,
                         po.full_model(B * 2 * D, [64, 32], 1), vp,
                         lr_pi=0.0, lr_v=0.0, x0=31337)
    for it in range(2):
        for tr in (full, s0, s1):
            tr.rollout()
        for buf in (BUF_ACTION, BUF_POLD):
            f = full.buffer(buf)
            np.testing.assert_array_equal(f[:, :n], s0.buffer(buf))
            np.testing.assert_array_equal(f[:, n:], s1.buffer(buf))
        f = full.buffer(BUF_BINS)
        np.testing.assert_array_equal(f[:, :n], s0.buffer(BUF_BINS))
        np.testing.assert_array_equal(f[:, n:], s1.buffer(BUF_BINS))
        for tr in (full, s0, s1):
            tr.learn()
        if orc is not None:
            orc.rollout()
            orc.learn()
        a = full.buffer(BUF_ADV)
        np.testing.assert_array_equal(a[:, :n], s0.buffer(BUF_ADV))
        np.testing.assert_array_equal(a[:, n:], s1.buffer(BUF_ADV))
        assert_close(s0.buffer(BUF_VALUE_GRAD) + s1.buffer(BUF_VALUE_GRAD),
                     full.buffer(BUF_VALUE_GRAD), what="value grad sum")
        g = s0.buffer(BUF_POLICY_GRADS)[0] + s1.buffer(BUF_POLICY_GRADS)[0]
        f = full.buffer(BUF_POLICY_GRADS)[0]
        if orc is not None:
            # two fp32 evaluation orders of the same sums (sides = 2)
            mag = orc.buf(po.BUF_POLICY_GRADS_MAG)[:g.size]
            rows = len(orc.buf(po.BUF_ROW_ENV))
            assert_grad_close(g, f, mag, n_terms=rows * B, sides=2,
                              what="policy grad sum")
        else:  # fp32 sums over 131k env-steps in different orders
            rel = np.linalg.norm(g - f) / np.linalg.norm(f)
            worst = np.abs(g - f).max() / np.abs(f).max()
            assert rel <= 1e-5 and worst <= 1e-4, (rel, worst)


def test_rccl_one_rank_communicator(ctx):
    from dependence_free_rl_amd import (POLICY, VALUE, Context, Trainer,
                                        init_policy, init_value)
    B, D, N, T, its = 8, 2, 256, 4, 2
    pp, vp = init_policy(D, 128, 64, seed=5), init_value(B, D, seed=6)
    rc = Context(device=0, rank=0, world=1, uid=Context.unique_id())
    try:
        out = []
        for c in (ctx, rc):
            tr = Trainer(c, bins=B, dims=D, num_envs=N, steps=T,
                         widths=(128, 64), rng_state=777)
            tr.set_params(POLICY, pp)
            tr.set_params(VALUE, vp)
            tr.set_timing(True)
            tr.iterate(its)
            out.append((tr.params(POLICY), tr.params(VALUE),
                        tr.kernel_time("allreduce")[1]))
            tr.close()
        (p0, v0, n0), (p1, v1, n1) = out
        assert n0 == 0 and n1 == its * (1 + tr.epochs), (n0, n1)
        np.testing.assert_array_equal(p0, p1)
        np.testing.assert_array_equal(v0, v1)
        x = np.arange(7, dtype=np.float32)
        np.testing.assert_array_equal(rc.allreduce_host(x), x)
    finally:
        rc.close()
