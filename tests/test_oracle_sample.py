"""The oracle's env sample of a larger reference-order job (CPU).

tests/test_gpu_global.py checks a 256-env sample of the full-size config-3
rollout against the oracle: envs [off, off + S) of an N-env job are an S-env
oracle trainer constructed from the engine advanced by 2 off draws, with env
i's stream set to the job's position 2 N + 4 T (off + i)
(or_trainer_set_stream_states).  Here that sample is held to the full
sequential N-env oracle run (the reference's worker order, rl.h:325-360) on
the same seed: identical trajectories."""
import numpy as np

from oracle import pyoracle as po


def test_sample_matches_full_sequential_run():
    from dependence_free_rl_amd.trainer import init_policy, init_value
    B, D, N, S, off, T, x0 = 8, 2, 48, 12, 20, 4, 424242
    pp, vp = init_policy(D, 32, 32, seed=3), init_value(B, D, seed=4)
    pol = po.perbin_model(2 * D, [32, 32], po.OR_SOFTMAX)
    val = po.full_model(B * 2 * D, [64, 32], 1)
    full = po.Trainer(po.OR_PPO, B, D, N, T, pol, pp, val, vp, x0=x0)
    full.rollout()
    sample = po.Trainer(po.OR_PPO, B, D, S, T, pol, pp, val, vp,
                        x0=po.minstd_jump(x0, 2 * off))
    sample.set_stream_states([po.minstd_jump(x0, 2 * N + 4 * T * (off + i))
                              for i in range(S)])
    sample.rollout()
    for buf, shape in ((po.BUF_STEP_CHOICE, (T,)), (po.BUF_STEP_DONE, (T,)),
                       (po.BUF_STEP_BINS, (T, B, D)), (po.BUF_STEP_ITEM, (T, D))):
        f = full.buf(buf).reshape((N,) + shape)[off:off + S]
        s = sample.buf(buf).reshape((S,) + shape)
        np.testing.assert_array_equal(f, s, err_msg="buffer %d" % buf)
    np.testing.assert_array_equal(
        full.buf(po.BUF_STEP_PCHOICE).reshape(N, T)[off:off + S],
        sample.buf(po.BUF_STEP_PCHOICE).reshape(S, T))
