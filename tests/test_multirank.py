"""Multi-rank semantics on CPU (gloo, world_size 2): the env shards and the
SUM all-reduce that the RCCL path relies on.

* Sharded gradients: each rank computes the loss gradient of the rows of its
  own envs (oracle, the reference's row losses); the gloo SUM all-reduce of
  the shard gradients equals the full-batch gradient of the single process.
* Env streams: rank r's envs, started at the reference-order positions the
  GPU uses (construction 2g, steps 2*Ng + 4*T*g), reproduce exactly the states
  of the single-process sequential run.
"""
import os
import socket

import numpy as np
import pytest

from conftest import REPO

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _full_run(B=8, D=2, N=8, T=8, x0=123457):
    from oracle import pyoracle as po
    from dependence_free_rl_amd.trainer import init_policy, init_value
    pol = po.perbin_model(2 * D, [64, 32], po.OR_SOFTMAX)
    val = po.full_model(B * 2 * D, [64, 32], 1)
    pp, vp = init_policy(D, 64, 32, seed=5), init_value(B, D, seed=6)
    tr = po.Trainer(po.OR_PPO, B, D, N, T, pol, pp, val, vp, x0=x0)
    tr.rollout()
    step_bins = tr.buf(po.BUF_STEP_BINS).reshape(N, T, B, D)
    step_choice = tr.buf(po.BUF_STEP_CHOICE).reshape(N, T)
    tr.learn()
    return dict(pol=pol, val=val, pp=pp, vp=vp, rows=tr.buf(po.BUF_ROWS).reshape(-1, B * 2 * D),
                env=tr.buf(po.BUF_ROW_ENV), choice=tr.buf(po.BUF_ROW_CHOICE),
                pold=tr.buf(po.BUF_ROW_POLD), adv=tr.buf(po.BUF_ADVANTAGES),
                targets=tr.buf(po.BUF_TARGETS), is_end=tr.buf(po.BUF_ROW_IS_END),
                pgrad0=tr.buf(po.BUF_POLICY_GRADS)[:pp.size],
                vgrad=tr.buf(po.BUF_VALUE_GRAD), step_bins=step_bins,
                step_choice=step_choice, B=B, D=D, N=N, T=T, x0=x0)


def _worker(rank, port, out):
    import sys
    sys.path.insert(0, REPO)
    import torch
    import torch.distributed as dist
    from oracle import pyoracle as po
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port,
                            rank=rank, world_size=WORLD)
    f = _full_run()
    N = f["N"]
    lo, hi = rank * N // WORLD, (rank + 1) * N // WORLD
    m = (f["env"] >= lo) & (f["env"] < hi)
    # this rank's rows only (its envs' trajectories, end rows included)
    pg = po.policy_grad_rows(f["pol"], f["pp"], f["rows"][m], f["choice"][m],
                             f["pold"][m], f["adv"][m], po.OR_PPO)
    vm = m & (f["is_end"] == 0)
    vg = po.value_grad_rows(f["val"], f["vp"], f["rows"][vm], f["targets"][vm])
    # end rows of the value step have target == V(self): zero gradient
    pg_t, vg_t = torch.from_numpy(pg.astype(np.float64)), torch.from_numpy(vg.astype(np.float64))
    dist.all_reduce(pg_t, op=dist.ReduceOp.SUM)
    dist.all_reduce(vg_t, op=dist.ReduceOp.SUM)
    # env streams of this shard, restarted from reference-order positions
    B, D, T, x0 = f["B"], f["D"], f["T"], f["x0"]
    cfg = po.env_cfg(B, D)
    ok_streams = True
    for g in range(lo, hi):
        rng = po.Rng(po.minstd_jump(x0, 2 * g))
        env = po.Env(cfg, rng)
        rng.x.value = po.minstd_jump(x0, 2 * N + 4 * T * g)
        for t in range(T):
            ok_streams &= bool((env.bins == f["step_bins"][g, t]).all())
            rng.canonical()  # the sampler's draws
            over = env.apply(f["step_choice"][g, t])
            if over:
                env.reset()
    res = torch.tensor([float(ok_streams)])
    dist.all_reduce(res, op=dist.ReduceOp.MIN)
    if rank == 0:
        np.savez(out, pg=pg_t.numpy(), vg=vg_t.numpy(), pfull=f["pgrad0"],
                 vfull=f["vgrad"], streams=res.numpy())
    dist.destroy_process_group()


def test_two_rank_gloo_shards_sum_to_the_single_process_batch(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(_free_port(), out), nprocs=WORLD, join=True)
    r = np.load(out)
    assert r["streams"][0] == 1.0
    # shard sums equal the full-batch gradients (fp32 summation-order noise)
    for what, x, y in (("policy", r["pg"], r["pfull"]), ("value", r["vg"], r["vfull"])):
        err = np.abs(x - y) / np.maximum(1.0, np.abs(y))
        assert err.max() <= 1e-5, (what, err.max())
