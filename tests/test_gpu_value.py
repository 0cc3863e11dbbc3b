"""The value net's kernels: the bf16 pair of value_net_kernels.hip (the
default, "vnet_bf16") and the f32 fused kernels of dense_kernels.hip
(mlp3_forward_kernel, mlp3_backward_data_kernel, mlp3_weight_grad_kernel;
XH_VALUE_KERNEL=mlp3) against the layer-by-layer Dense GEMMs they replace
(XH_VALUE_KERNEL=gemm), through update_value_model and calculate_advantage
(policy_gradient.h:196-281) over three iterations (episodes end: terminal
rows).  The f32 fused kernels give the same bits.  The bf16 kernels take
layer 0 as exact bf16 products (integer observations, W0 / 8 in three exact
bf16 parts) summed in another order: values, terminal values, TD targets,
value gradients, advantages and updated parameters within the parity
tolerance (RTOL, conftest.py) of the GEMMs'."""
import numpy as np
import pytest

from conftest import RTOL, assert_close, log_record

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo,B,D,widths,N,T", [
    ("ppo", 32, 1, (64, 64), 512, 4),      # config 2 shape (Fin 64)
    ("ppo", 64, 2, (128, 128), 256, 4),    # config 3 (reduced layer 0, Fin 256)
    ("ac", 128, 3, (128, 128), 96, 8),     # config 5 (Fin 768)
    ("ac", 128, 3, (128, 128), 7, 3),      # fewer rows than one 64-row tile per split
])
def test_value_kernels_against_gemm(ctx, monkeypatch, algo, B, D, widths, N, T):
    from dependence_free_rl_amd import POLICY, VALUE, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import (BUF_ADV, BUF_TARGETS, BUF_V_STATE,
                                                BUF_V_STATE0, BUF_V_TERM,
                                                BUF_VALUE_GRAD)
    pp, vp = init_policy(D, *widths, seed=31), init_value(B, D, seed=32)
    names = ("v_state0", "v_term", "targets", "value_grad", "v_state", "adv")
    bufs = (BUF_V_STATE0, BUF_V_TERM, BUF_TARGETS, BUF_VALUE_GRAD, BUF_V_STATE,
            BUF_ADV)

    def run(kernel, w0_fuse=None):
        if w0_fuse is None:
            monkeypatch.delenv("XH_W0_FUSE", raising=False)
        else:
            monkeypatch.setenv("XH_W0_FUSE", w0_fuse)
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
    m3, km = run("mlp3")
    got, kg = run(None)
    assert (kr, km, kg) == ("gemm", "mlp3_fused", "vnet_bf16")
    if B <= 64:
        # the W0 fragments split inside the forward (the default up to 64 bins
        # and 3 k blocks per half) and by w0_frag_kernel with its own item
        # sums (XH_W0_FUSE=1) have the bits of w0_item_kernel +
        # w0_frag_kernel (XH_W0_FUSE=0)
        sep, _ = run(None, w0_fuse="0")
        frk, _ = run(None, w0_fuse="1")
        for mode, other in (("default", got), ("1", frk)):
            for it, (x, y) in enumerate(zip(other, sep)):
                for i, (a, b) in enumerate(zip(x, y)):
                    np.testing.assert_array_equal(
                        a, b, err_msg="w0 mode %s iteration %d item %d" % (mode, it, i))
    worst = {}
    for it, (x, y, z) in enumerate(zip(got, ref, m3)):
        for i, (a, b, c) in enumerate(zip(x, y, z)):
            np.testing.assert_array_equal(c, b, err_msg="mlp3 iteration %d item %d" % (it, i))
            name = names[i] if i < len(names) else "value_params"
            err = assert_close(a, b, tol=RTOL, what="vnet %s iteration %d" % (name, it))
            worst[name] = max(worst.get(name, 0.0), err)
    print("vnet_bf16 vs gemm, max scaled error:", worst)
    log_record("value_kernels.jsonl", {"B": B, "D": D, "N": N, "T": T, "algo": algo,
                                       "max_scaled_err": worst})
