"""Diagnostic: evaluate() traces across trace_cap values."""
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
w = tr.evaluate(8, 100, x0, trace_cap=3000)
rng = po.Rng(x0)
first = rng.canonical() < 0.4
item = [4, 2] if first else [1, 2]
x = po.minstd_jump(x0, 2)
bad = 0
for cap in (1, 7, 2048, 2049, 3000, 4096, 10000, 12345):
    for init in (None, np.tile(item, (8, 1))):
        r2 = tr.evaluate(8, 100, x0 if init is None else x, init_items=init, trace_cap=cap)
        k = min(cap, 2748)
        d = np.nonzero(r2["trace"][:k] != w["trace"][:k])[0]
        bad += len(d)
        print(cap, init is None, r2["totals"][0], d[:5])
whole = tr.evaluate(8, 1000, x0)
x, tot = po.minstd_jump(x0, 2), 0.0
for _ in range(10):
    r = tr.evaluate(8, 100, x, init_items=np.tile(item, (8, 1)))
    tot += r["totals"][0]
    x, item = int(r["rng"][0]), list(r["final_items"][0])
print("chained", tot, whole["totals"][0], "BAD" if bad or tot != whole["totals"][0] else "OK")
