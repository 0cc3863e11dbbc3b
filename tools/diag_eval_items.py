"""Diagnostic: determinism of evaluate() (one call vs repeated, chained)."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import golden
from dependence_free_rl_amd import Context, Trainer
from dependence_free_rl_amd.trainer import POLICY
from oracle import pyoracle as po
ctx = Context(0)
g = golden("deep_w20")
tr = Trainer(ctx, algo="ppo", bins=8, dims=2, num_envs=8, steps=1, widths=(128, 64))
tr.set_params(POLICY, g["params"])
x0 = int(g["x0"][0])
ref = None
for rep in range(4):
    w = tr.evaluate(8, 1000, x0, trace_cap=30000)
    if ref is None:
        ref = w
    d = np.nonzero(w["trace"] != ref["trace"])[0]
    print("whole", rep, w["totals"], w["steps"][0], w["rng"][0], "trace diff", d[:4], len(d))
for rep in range(3):
    rng = po.Rng(x0)
    first = rng.canonical() < 0.4
    item = [4, 2] if first else [1, 2]
    x, tot, n = po.minstd_jump(x0, 2), 0.0, 0
    tr_all = []
    for c in range(10):
        r = tr.evaluate(8, 100, x, init_items=np.tile(item, (8, 1)), trace_cap=3000)
        k = int(r["steps"][0])
        tr_all.append(r["trace"][:k])
        tot += r["totals"][0]
        n += k
        x, item = int(r["rng"][0]), list(r["final_items"][0])
    t = np.concatenate(tr_all)
    d = np.nonzero(t != ref["trace"][:len(t)])[0]
    print("chained", rep, tot, n, x, "trace diff vs whole", d[:4], len(d))
