"""Diagnostic: GPU argmax evaluation (weights.20, seed 1, 10000 episodes) vs
the oracle, step by step: first step where the oracle's argmax differs from
the GPU's choice, with the logit gap there."""
import sys

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from conftest import golden  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from dependence_free_rl_amd import Context, Trainer  # noqa: E402
from dependence_free_rl_amd.trainer import POLICY  # noqa: E402

g = golden("deep_w20")
ctx = Context(0)
tr = Trainer(ctx, algo="ppo", bins=8, dims=2, num_envs=8, steps=1,
             widths=(128, 64))
tr.set_params(POLICY, g["params"])
E = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
r = tr.evaluate(8, E, 1, trace_cap=400000)
print("gpu total", r["totals"][0], "steps", r["steps"][0])
trace = r["trace"][: r["steps"][0]]
cfg = po.env_cfg(8, 2)
rng = po.Rng(1)
env = po.Env(cfg, rng)
m = po.perbin_model(4, [128, 64], None)
ep = 0
for i, a in enumerate(trace):
    obs = env.obs().reshape(1, 32)
    z = po.model_eval(m, g["params"], obs)[0]
    c = int(np.argmax(z))
    if c != a:
        zs = np.sort(z)[::-1]
        print("step", i, "episode", ep, "gpu", a, "oracle", c, "z", z[a], z[c],
              "gap", z[c] - z[a], "bins", env.bins.tolist(), "item",
              env.item[:2].tolist())
        break
    over = env.apply(a)
    if over:
        env.reset()
        ep += 1
else:
    print("no divergence over", len(trace), "steps")
