"""Diagnostic: 128-bin rollouts (wave vs 4-wave vs oracle)."""
import os
import sys
import numpy as np
sys.path.insert(0, ".")
from dependence_free_rl_amd import POLICY, VALUE, Context, Trainer, init_policy, init_value
from dependence_free_rl_amd.trainer import BUF_ACTION, BUF_LOGITS
from oracle import pyoracle as po
ctx = Context(0)
B, D, T = 128, 3, 8
pp, vp = init_policy(D, 128, 128, seed=11), init_value(B, D, seed=12)
for N in (4104, 8192, 16384):
    got = {}
    for kern in ("wave", "4"):
        if kern == "4":
            os.environ["XH_ROLLOUT_KERNEL"] = "4"
        else:
            os.environ.pop("XH_ROLLOUT_KERNEL", None)
        tr = Trainer(ctx, algo="ac", bins=B, dims=D, num_envs=N, steps=T,
                     widths=(128, 128), rng_state=99, record_last_step=True)
        tr.set_params(POLICY, pp)
        tr.set_params(VALUE, vp)
        tr.rollout()
        got[kern] = (tr.buffer(BUF_ACTION), tr.buffer(BUF_LOGITS))
        tr.close()
    a, b = got["wave"][0], got["4"][0]
    bad_env = np.nonzero((a != b).any(0))[0]
    bad_t = np.nonzero((a != b).any(1))[0]
    print(N, "bad envs", len(bad_env), bad_env[:8].tolist(), "bad steps", bad_t.tolist())
    print(N, "actions differ", int((a != b).sum()), "of", a.size,
          "first", np.argwhere(a != b)[:3].tolist(),
          "logit maxdiff", float(np.abs(got["wave"][1] - got["4"][1]).max()))
    if N <= 64:
        orc = po.Trainer(po.OR_AC, B, D, N, T,
                         po.perbin_model(2 * D, [128, 128], po.OR_SOFTMAX_XENT), pp,
                         po.full_model(B * 2 * D, [64, 32], 1), vp, x0=99)
        orc.rollout()
        oc = orc.buf(po.BUF_STEP_CHOICE).reshape(N, T).T
        print("   vs oracle: wave", int((a != oc).sum()), "4wave", int((b != oc).sum()))
