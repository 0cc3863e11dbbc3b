"""Diagnostic: run-to-run determinism of the 128-bin rollout kernels."""
import os
import sys
import numpy as np
sys.path.insert(0, ".")
from dependence_free_rl_amd import POLICY, VALUE, Context, Trainer, init_policy, init_value
from dependence_free_rl_amd.trainer import BUF_ACTION, BUF_LOGITS
ctx = Context(0)
B, D, T = 128, 3, 8
pp, vp = init_policy(D, 128, 128, seed=11), init_value(B, D, seed=12)
for kern in ("wave", "4"):
    if kern == "4":
        os.environ["XH_ROLLOUT_KERNEL"] = "4"
    else:
        os.environ.pop("XH_ROLLOUT_KERNEL", None)
    for N in (8192, 16384):
        ref = None
        for rep in range(4):
            tr = Trainer(ctx, algo="ac", bins=B, dims=D, num_envs=N, steps=T,
                         widths=(128, 128), rng_state=99)
            tr.set_params(POLICY, pp)
            tr.set_params(VALUE, vp)
            tr.rollout()
            got = (tr.buffer(BUF_ACTION), tr.buffer(BUF_LOGITS))
            tr.close()
            if ref is None:
                ref = got
            print(kern, N, rep, "actions differ", int((got[0] != ref[0]).sum()),
                  "logit maxdiff", float(np.abs(got[1] - ref[1]).max()), flush=True)
