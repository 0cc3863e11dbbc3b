"""Is the host ahead of the GPU?  For a bench configuration, the time
xh_trainer_iterate(1) takes to return (host enqueue only: no synchronisation
inside the product loop) against the GPU time per iteration; if enqueueing
an iteration takes about as long as running it, the GPU idles between
launches waiting for the host.

    python tools/host_ahead.py --config 5
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--timing", default="off", choices=["off", "train"],
                    help="train: HIP events around the policy-train launches, as "
                         "bench.py's timed region")
    ap.add_argument("--lr-scale-rows", action="store_true",
                    help="bench.py's default learning-rate scaling (lr / rows)")
    args = ap.parse_args()
    import bench
    from dependence_free_rl_amd import (POLICY, VALUE, Context, Trainer, init_policy,
                                        init_value)
    k = bench.select_config(args.config)
    ctx = Context(0)
    tr = Trainer(ctx, algo=k["algo"], bins=k["B"], dims=k["D"], num_envs=k["N"],
                 steps=k["T"], widths=k["H"], value_widths=(bench.V1, bench.V2),
                 rng_state=20241008, lr_scale_rows=args.lr_scale_rows)
    tr.set_params(POLICY, init_policy(k["D"], *k["H"], seed=0))
    tr.set_params(VALUE, init_value(k["B"], k["D"], bench.V1, bench.V2, seed=1))
    tr.iterate(2)
    tr.synchronize()
    if args.timing == "train":
        tr.set_timing("train")
    enq = []
    t0 = time.perf_counter()
    for _ in range(args.iters):
        a = time.perf_counter()
        tr.iterate(1)
        enq.append(time.perf_counter() - a)
    b = time.perf_counter()
    tr.synchronize()
    t1 = time.perf_counter()
    print("config %d timing %s lr_scale_rows %d: host enqueue per iteration %.3f ms (first %.3f, max %.3f); "
          "wall per iteration %.3f ms; wait at the end %.3f ms"
          % (args.config, args.timing, args.lr_scale_rows, 1e3 * sum(enq) / len(enq), 1e3 * enq[0], 1e3 * max(enq),
             1e3 * (t1 - t0) / args.iters, 1e3 * (t1 - b)))
    tr.close()


if __name__ == "__main__":
    main()
