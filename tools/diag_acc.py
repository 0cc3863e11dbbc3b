#!/usr/bin/env python3
"""Diagnostic (GPU box): per-entry policy-gradient error of the default and
an override train kernel against the oracle's double sums, at the
test_gpu_scale accuracy case of a shape; prints the worst entries with the
parameter block they belong to (flat model::parameters() layout).
    python tools/diag_acc.py [B D N T H] [override]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    B, D, N, T, H = [int(x) for x in (sys.argv[1:6] or [32, 1, 768, 4, 64])]
    over = sys.argv[6] if len(sys.argv) > 6 else "split4h"
    from oracle import pyoracle as po
    from dependence_free_rl_amd import POLICY, VALUE, Context, Trainer, init_policy, init_value
    from dependence_free_rl_amd.trainer import BUF_POLICY_GRADS
    x0 = 24681357
    pp, vp = init_policy(D, H, H, seed=11), init_value(B, D, seed=12)
    orc = po.Trainer(po.OR_PPO, B, D, N, T, po.perbin_model(2 * D, [H, H], po.OR_SOFTMAX), pp,
                     po.full_model(B * 2 * D, [64, 32], 1), vp, x0=x0)
    orc.rollout()
    orc.learn()
    ref = np.asarray(orc.buf(po.BUF_POLICY_GRADS), np.float64)
    mag = np.asarray(orc.buf(po.BUF_POLICY_GRADS_MAG), np.float64)
    F0 = 2 * D
    blocks = [("W1", H * F0), ("b1", H), ("W2", H * H), ("b2", H), ("w3", H), ("b3", 1)]
    npi = sum(n for _, n in blocks)

    def block_of(i):
        i %= npi
        for name, n in blocks:
            if i < n:
                return name, i
            i -= n
        return "?", i
    ctx = Context(0)
    for kern in ("default", over, "f32"):
        if kern == "default":
            os.environ.pop("XH_TRAIN_KERNEL", None)
        else:
            os.environ["XH_TRAIN_KERNEL"] = kern
        tr = Trainer(ctx, bins=B, dims=D, num_envs=N, steps=T, widths=(H, H), rng_state=x0)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        tr.rollout()
        tr.learn()
        name = tr.kernel_info()["policy_train"]["kernel"]
        g = tr.buffer(BUF_POLICY_GRADS).ravel().astype(np.float64)
        tr.close()
        units = np.abs(g - ref) / np.maximum(mag * 2.0 ** -24, 1e-30)
        order = np.argsort(-units)[:8]
        print(name, "max %.0f median %.3f p99 %.1f" % (
            units.max(), np.median(units[mag > 0]), np.percentile(units[mag > 0], 99)))
        for i in order:
            print("   epoch %d %s[%d] units %.0f x %.6g ref %.6g mag %.3g" % (
                i // npi, *block_of(i), units[i], g[i], ref[i], mag[i]))
    ctx.close()


if __name__ == "__main__":
    main()
