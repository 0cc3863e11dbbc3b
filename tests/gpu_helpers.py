"""Shared helpers for the GPU parity tests (tests only)."""
import numpy as np

from conftest import golden


def meta(g):
    return dict(a.split("=", 1) for a in str(g["meta_args"]).split())


def trainer_from_golden(ctx, name, **kw):
    from dependence_free_rl_amd import POLICY, VALUE, Trainer
    g = golden(name)
    kv = meta(g)
    B, D, N, T = int(kv["B"]), int(kv["D"]), int(kv["N"]), int(kv.get("T", 4))
    widths = tuple(int(w) for w in kv["widths"].split(","))
    if "wd_pi" in kv:
        kw.setdefault("wd_policy", float(kv["wd_pi"]))
    kw.setdefault("wd_policy", 0.0)
    tr = Trainer(ctx, algo=kv["algo"], bins=B, dims=D, num_envs=N, steps=T,
                 widths=widths, rng_state=int(g["x0"][0]), **kw)
    tr.set_params(POLICY, g["init_policy"])
    tr.set_params(VALUE, g["init_value"])
    for which, key in ((POLICY, "opt_pi"), (VALUE, "opt_v")):
        if key in kv:
            tr.set_optimizer(which, kv[key], default_lr(kv["algo"], which))
    return tr, g, kv


def default_lr(algo, which):
    """Drivers' learning rates: ppo_training.cc:17,26 / ac_training.cc:17,26."""
    if algo == "ac":
        return 1e-5 if which == 0 else 1e-4
    return 1e-4 if which == 0 else 1e-5


def step_major(arr, N, T):
    """Golden per-step logs are env-major ([env][t]); GPU buffers are [t][env]."""
    a = np.asarray(arr)
    return a.reshape((N, T) + a.shape[1:]).swapaxes(0, 1)


def row_index(g, it, T):
    """Map golden learn rows -> (kind, t, env): kind 0 transition, 1 open end
    row (S_T), 2 terminal end row (E_t)."""
    p = "it%d_" % it
    env = g[p + "row_env"]
    step = g[p + "row_step"] - it * T
    is_end = g[p + "row_is_end"]
    frozen = g[p + "row_frozen"]
    out = []
    for k in range(len(env)):
        if not is_end[k]:
            out.append((0, int(step[k]), int(env[k])))
        elif frozen[k]:
            out.append((2, int(step[k]) - 1, int(env[k])))
        else:
            out.append((1, T, int(env[k])))
    return out
