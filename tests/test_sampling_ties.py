"""The near-tie proof used by the full-size sampling test (sampling_ties.py)
on constructed cases: a device distribution that moves the boundary at the
oracle's pick just past the draw u is a proven tie when the move is within
TIE_TOL, and not beyond it; equal picks or a u outside the sliver are never
ties."""
import ctypes as C

import numpy as np

from sampling_ties import TIE_TOL, cumulative, near_tie


def _setup():
    from oracle import pyoracle as po
    B, D, N, T, x0, g, t = 64, 2, 32768, 4, 1357911, 77, 1
    rng = np.random.default_rng(3)
    from dependence_free_rl_amd.trainer import init_policy
    pp = init_policy(D, 128, 128, seed=51)
    bins = rng.integers(0, 9, (B, D)).astype(np.int32)
    item = np.array([4, 2], np.int32)
    cfg = po.env_cfg(B, D)
    it = np.zeros(3, np.int32)
    it[:D] = item
    obs = np.zeros(B * 2 * D, np.float32)
    po.lib().or_obs(C.byref(cfg), po._ptr(bins), po._ptr(it), po._ptr(obs))
    p = po.model_eval(po.perbin_model(2 * D, [128, 128], po.OR_SOFTMAX), pp,
                      obs[None, :])[0]
    u = po.Rng(po.minstd_jump(x0, 2 * N + 4 * T * g + 4 * t)).canonical()
    return po, pp, B, D, N, T, x0, g, t, bins, item, p, u


def _shifted(p, c, u, extra):
    """a device table whose boundary c sits `extra` below u (it picks c + 1)"""
    cp = cumulative(p)
    delta = cp[c] - u + extra  # mass moved from bin c to bin c + 1
    q = np.asarray(p, np.float64).copy()
    q[c] -= delta
    q[c + 1] += delta
    return q.astype(np.float32)


def test_near_tie_proof():
    po, pp, B, D, N, T, x0, g, t, bins, item, p, u = _setup()
    cp = cumulative(p)
    c = int(np.searchsorted(cp, u, side="left"))
    if c == B - 1:
        c -= 1
    # the same distribution: the same pick, no tie to prove
    r = near_tie(po, pp, B, D, N, T, x0, g, t, bins, item, p, c, c)
    assert not r["proven"]
    # a table whose boundary c lies just below u picks c + 1: proven when
    # the oracle's boundary is within TIE_TOL of u, whichever it is here
    q = _shifted(p, c, u, 1e-7)
    qc = cumulative(q)
    cd = int(np.searchsorted(qc, u, side="left"))
    r = near_tie(po, pp, B, D, N, T, x0, g, t, bins, item, q, cd, c)
    assert r["proven"] == (cd != c and abs(qc[c] - cp[c]) <= TIE_TOL and
                           qc[c] <= u <= cp[c]), r
    # a made-up tie: the oracle's own u with a device table far off
    far = p.astype(np.float64).copy()
    far[c] *= 0.5
    far = far.astype(np.float32)
    fc = cumulative(far)
    cf = int(np.searchsorted(fc, u, side="left"))
    if cf != c and abs(fc[min(c, cf)] - cp[min(c, cf)]) > TIE_TOL:
        r = near_tie(po, pp, B, D, N, T, x0, g, t, bins, item, far, cf, c)
        assert not r["proven"], r
