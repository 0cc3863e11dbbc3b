"""The near-tie proof of a free-running sample that differs between the
device and the oracle (tests/test_gpu_global.py): discrete_distribution's
pick (rl.h:27-30, tensor.cc:467-470; libstdc++ random.tcc:2654-2713) is the
lower_bound of the draw u in the cumulative table, so two f32-class
evaluations of one state can pick neighbouring bins only when u falls between
their two tables' entries at that boundary.  CPU only (the oracle)."""
import numpy as np

TIE_TOL = 1e-4


def cumulative(p):
    """discrete_distribution's cumulative table (libstdc++ random.tcc:2654-2713,
    as or_discrete): p / sum in double, partial sums, last entry 1."""
    p = np.asarray(p, np.float64)
    total = 0.0
    for x in p:  # the sequential double sum (numpy's sum is pairwise)
        total += float(x)
    cp = np.cumsum(p / total)
    cp[-1] = 1.0
    return cp


def near_tie(po, pp, B, D, N, T, x0, g, t, bins, item, q_dev, c_dev, c_orc):
    """Is env g's first differing pick at step t a near-tie?  Both sides saw
    the same state (every earlier step agreed); u is the step's draw from the
    env's reference-order stream (construction 2 N, then 4 draws per step);
    the oracle's distribution is its model on that state."""
    import ctypes as C
    cfg = po.env_cfg(B, D)
    b = np.ascontiguousarray(bins, np.int32).reshape(B, D)
    it = np.zeros(3, np.int32)
    it[:D] = np.asarray(item, np.int32).ravel()[:D]
    obs = np.zeros(B * 2 * D, np.float32)
    po.lib().or_obs(C.byref(cfg), po._ptr(b), po._ptr(it), po._ptr(obs))
    p_orc = po.model_eval(po.perbin_model(2 * D, [128, 128], po.OR_SOFTMAX), pp,
                          obs[None, :])[0]
    u = po.Rng(po.minstd_jump(x0, 2 * N + 4 * T * g + 4 * t)).canonical()
    cp_o, cp_d = cumulative(p_orc), cumulative(q_dev)
    k = min(c_dev, c_orc)
    lo, hi = sorted((float(cp_o[k]), float(cp_d[k])))
    rec = {"env": int(g), "step": int(t), "device_pick": c_dev,
           "oracle_pick": c_orc, "u": u, "cp_oracle": float(cp_o[k]),
           "cp_device": float(cp_d[k]), "gap": hi - lo}
    # each side's pick is the lower_bound of u in its own table, and u falls
    # in the sliver between the two tables' boundary k
    rec["proven"] = bool(int(np.searchsorted(cp_o, u, side="left")) == c_orc and
                         int(np.searchsorted(cp_d, u, side="left")) == c_dev and
                         abs(c_dev - c_orc) >= 1 and lo <= u <= hi and
                         hi - lo <= TIE_TOL)
    return rec
