"""The fused value net (dense_kernels.hip: mlp3_forward_kernel,
mlp3_backward_data_kernel, mlp3_weight_grad_kernel) against the layer-by-
layer Dense GEMMs it replaces (XH_VALUE_KERNEL=gemm): update_value_model and
calculate_advantage (policy_gradient.h:196-281) give the same bits."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo,B,D,widths,N,T", [
    ("ppo", 32, 1, (64, 64), 512, 4),      # config 2 shape (Fin 64)
    ("ppo", 64, 2, (128, 128), 256, 4),    # config 3 (reduced layer 0, Fin 256)
    ("ac", 128, 3, (128, 128), 96, 8),     # config 5 (Fin 768)
])
def test_fused_value_net_bit_identical(ctx, monkeypatch, algo, B, D, widths, N, T):
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ADV, BUF_TARGETS, BUF_V_STATE,
                                                BUF_V_STATE0, BUF_V_TERM,
                                                BUF_VALUE_GRAD)
    pp, vp = init_policy(D, *widths, seed=31), init_value(B, D, seed=32)
    bufs = (BUF_V_STATE0, BUF_V_TERM, BUF_TARGETS, BUF_VALUE_GRAD, BUF_V_STATE,
            BUF_ADV)

    def run(kernel):
        if kernel:
            monkeypatch.setenv("XH_VALUE_KERNEL", kernel)
        else:
            monkeypatch.delenv("XH_VALUE_KERNEL", raising=False)
        tr = Trainer(ctx, algo=algo, bins=B, dims=D, num_envs=N, steps=T,
                     widths=widths, rng_state=5)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        out = []
        for _ in range(3):  # three iterations: episodes end (terminal rows)
            tr.rollout()
            tr.learn()
            out.append([tr.buffer(b).copy() for b in bufs] + [tr.params(VALUE)])
        k = tr.kernel_info()["value"]
        tr.close()
        return out, k

    ref, kr = run("gemm")
    got, kg = run(None)
    assert (kr, kg) == ("gemm", "mlp3_fused")
    for it, (x, y) in enumerate(zip(got, ref)):
        for i, (a, b) in enumerate(zip(x, y)):
            np.testing.assert_array_equal(a, b, err_msg="iteration %d item %d" % (it, i))
