"""Wall time of bench-config iterations with per-launch HIP-event timing on
and off (is the phase instrumentation inside the timed region free?)."""
import sys
import time

sys.path.insert(0, ".")
import bench  # noqa: E402
from dependence_free_rl_amd import (POLICY, VALUE, Context, Trainer,  # noqa: E402
                                    init_policy, init_value)

for c in [int(x) for x in (sys.argv[1:] or ["2", "3"])]:
    k = bench.select_config(c)
    ctx = Context(device=0)
    tr = Trainer(ctx, algo=k["algo"], bins=k["B"], dims=k["D"], num_envs=k["N"],
                 steps=k["T"], widths=k["H"], value_widths=(64, 32),
                 rng_state=20241008, lr_scale_rows=True)
    tr.set_params(POLICY, init_policy(k["D"], *k["H"], seed=0))
    tr.set_params(VALUE, init_value(k["B"], k["D"], 64, 32, seed=1))
    tr.iterate(2)
    tr.synchronize()
    for rep in range(3):
        for timing in (False, True):
            tr.set_timing(timing)
            tr.reset_timing()
            t0 = time.perf_counter()
            tr.iterate(10)
            tr.synchronize()
            dt = (time.perf_counter() - t0) / 10 * 1e3
            print("config %d timing %-5s %.3f ms/iteration" % (c, timing, dt), flush=True)
    tr.close()
