#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (container only).

Runs oracle/_ref/ref_harness -- the real reference compiled from
/root/reference by `make -C oracle ref` -- and converts its record files into
small .npz fixtures.  Re-run after changing the harness:

    make -C oracle ref && python tests/golden/make_golden.py

The fixtures are data only (inputs and expected outputs).  Each entry in
FIXTURES says which reference code path produced it.
"""
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
# the same harness compiled against the reference's bin_packing.h with
# num_bins = 64 (oracle/Makefile): the config-3 shape on bp::environment
HARNESS_BP64 = os.path.join(REPO, "oracle", "_ref", "ref_harness_bp64")
BP64 = ("ppo_b64d2", "ppo_b64d2_n160")
REF = "/root/reference"

_DT = {b"f": np.float32, b"d": np.float64, b"i": np.int32, b"u": np.uint32}


def read_records(path):
    out = {}
    with open(path, "rb") as f:
        data = f.read()
    off = 0
    while off < len(data):
        (nl,) = struct.unpack_from("<I", data, off)
        off += 4
        name = data[off:off + nl].decode()
        off += nl
        dt = data[off:off + 1]
        off += 1
        (nd,) = struct.unpack_from("<I", data, off)
        off += 4
        dims = struct.unpack_from("<%dQ" % nd, data, off)
        off += 8 * nd
        dtype = np.dtype(_DT[dt])
        n = int(np.prod(dims)) if nd else 1
        arr = np.frombuffer(data, dtype=dtype, count=n, offset=off).reshape(dims)
        off += n * dtype.itemsize
        out[name] = arr.copy()
    return out


# name -> (harness mode, args, small-ification)
FIXTURES = {
    # minstd_rand0 / generate_canonical / bernoulli / discrete_distribution
    # (xylo/tensor.cc:71-75, 467-470; apps/bin_packing/bin_packing.h:81)
    "rng": ("rng", ["seed=42", "n=8000"]),
    # bp::environment + bp::agent + random_policy (bin_packing.h:46-107,
    # rl.h:305-349), and gen_env<8,2> equivalence; gen_env<64,2> and
    # gen_env<128,2> reproduce it on 8 injected bins
    "env8": ("envcheck", ["seed=7", "steps=3000"]),
    # deep_agent.cc with weights.20, seed 1, 1000 argmax episodes
    "deep_w20": ("deep", ["seed=1", "episodes=1000",
                          "weights=%s/apps/bin_packing/weights.20" % REF]),
    # ppo_training.cc shapes: conv 4->128->64->1 + softmax, value 32->64->32->1
    "ppo_b8d2": ("learn", ["algo=ppo", "B=8", "D=2", "widths=128,64", "N=8",
                           "T=8", "iters=5", "seed=42"]),
    # BASELINE config 2 shape (1-D, 32 bins, [64,64])
    "ppo_b32d1": ("learn", ["algo=ppo", "B=32", "D=1", "widths=64,64", "N=6",
                            "T=4", "iters=2", "seed=5"]),
    # BASELINE config 3/4 shape (2-D, 64 bins, [128,128]) on the reference's
    # own bp::environment / bp::agent at 64 bins (ref_harness_bp64)
    "ppo_b64d2": ("learn", ["algo=ppo", "B=64", "D=2", "widths=128,128",
                            "N=4", "T=4", "iters=2", "seed=11"]),
    # the config-3 shape with enough envs for several 64-row groups per train
    # workgroup (640 groups per epoch): the device's multi-group dW
    # accumulation pinned by the reference itself, not only by the oracle
    "ppo_b64d2_n160": ("learn", ["algo=ppo", "B=64", "D=2", "widths=128,128",
                                 "N=160", "T=4", "iters=2", "seed=31"]),
    # ppo2_training.cc: KL-regulated PPO, conv 4->128->64->1 + softmax,
    # policy sgd(1e-4, wd 1e-5), 16 workers x 8 steps; beta carries over
    "klppo_b8d2": ("learn", ["algo=klppo", "B=8", "D=2", "widths=128,64",
                             "N=16", "T=8", "iters=4", "wd_pi=1e-5",
                             "seed=21"]),
    # ac_training.cc shapes: conv 4->64->32->1 + softmax-xent, 16x8
    "ac_b8d2": ("learn", ["algo=ac", "B=8", "D=2", "widths=64,32", "N=16",
                          "T=8", "iters=4", "seed=3"]),
    # BASELINE config 5 shape (3-D, 128 bins, [128,128], actor-critic)
    "ac_b128d3": ("learn", ["algo=ac", "B=128", "D=3", "widths=128,128",
                            "N=2", "T=8", "iters=2", "seed=13"]),
    # deep_agent.cc's first round as its main runs it (engine seeded 1
    # before the model's He init draws; 10000 episodes)
    "deep_w20_main": ("deep", ["seed=1", "episodes=10000", "main=1",
                               "weights=%s/apps/bin_packing/weights.20" % REF]),
    # ppo_training.cc / ac_training.cc prologue seeded: initial parameters
    # and engine state after the workers' envs (pins include/xylo_compat)
    "driver_ppo_s7": ("driver", ["algo=ppo", "seed=7"]),
    "driver_ac_s7": ("driver", ["algo=ac", "seed=7"]),
    "driver_ppo2_s7": ("driver", ["algo=ppo", "seed=7", "workers=16"]),
    # random_agent.cc's loop seeded: 3 rounds x 100 episodes
    "random_s5": ("random", ["seed=5", "rounds=3", "episodes=100"]),
    # the reference's own heuristic agents (firstfit/bestfit/minwaste_agent.cc
    # policies, random_agent.cc's random_policy), seeded: 2 rounds x 1000
    "heur_firstfit": ("heuristic", ["policy=firstfit", "seed=3", "rounds=2",
                                    "episodes=1000"]),
    "heur_bestfit": ("heuristic", ["policy=bestfit", "seed=3", "rounds=2",
                                   "episodes=1000"]),
    "heur_minwaste": ("heuristic", ["policy=minwaste", "seed=3", "rounds=2",
                                    "episodes=1000"]),
    "heur_random": ("heuristic", ["policy=random", "seed=3", "rounds=2",
                                  "episodes=1000"]),
    # the reference's other optimizers (nn.h:630-698) in the learners: PPO
    # with adam on the policy and momentum on the value net, AC the other
    # way round; state (moments, velocity, adam's t) carries across learn()
    "ppo_adam_b8d2": ("learn", ["algo=ppo", "B=8", "D=2", "widths=128,64",
                                "N=8", "T=8", "iters=3", "seed=23",
                                "opt_pi=adam", "opt_v=momentum"]),
    "ac_mom_b8d2": ("learn", ["algo=ac", "B=8", "D=2", "widths=64,32",
                              "N=16", "T=8", "iters=3", "seed=29",
                              "opt_pi=momentum", "opt_v=adam"]),
    # the config-5 shape with 768 row groups per epoch (3 per train workgroup
    # at 256 CUs) and the config-2 shape with 1536 two-env groups (3 per
    # workgroup at 2 x 256): the multi-group gradient accumulation of the
    # 128-row and the [64,64] train kernels pinned by the reference itself.
    # Learner row matrices dropped (the GPU tests do not read them).
    "ac_b128d3_n96": ("learn", ["algo=ac", "B=128", "D=3", "widths=128,128",
                                "N=96", "T=8", "iters=1", "seed=37"], ("_rows",)),
    "ppo_b32d1_n768": ("learn", ["algo=ppo", "B=32", "D=1", "widths=64,64",
                                 "N=768", "T=4", "iters=1", "seed=41"], ("_rows",)),
    # BASELINE config 1 (REINFORCE, 1-D, 8 bins, 1 env, full MLP[32])
    "pg_b8d1": ("learn", ["algo=pg", "B=8", "D=1", "widths=32", "N=1",
                          "episodes=4", "iters=3", "seed=17"]),
    # pg_training.cc's network (full 32->256->128->8, softmax-xent) with one
    # worker playing 4 episodes per iteration (one engine stream)
    "pg_b8d2": ("learn", ["algo=pg", "B=8", "D=2", "widths=256,128", "N=1",
                          "episodes=4", "iters=3", "seed=19"]),
}


def main(names):
    if not (os.path.exists(HARNESS) and os.path.exists(HARNESS_BP64)):
        sys.exit("build the harnesses first: make -C oracle ref")
    names = names or list(FIXTURES)
    for name in names:
        mode, args = FIXTURES[name][:2]
        drop = FIXTURES[name][2] if len(FIXTURES[name]) > 2 else ()
        with tempfile.TemporaryDirectory() as td:
            rec = os.path.join(td, "out.rec")
            harness = HARNESS_BP64 if name in BP64 else HARNESS
            subprocess.run([harness, mode, "out=" + rec] + args, check=True,
                           cwd=td)
            arrs = read_records(rec)
            arrs = {k: v for k, v in arrs.items()
                    if not any(k.endswith(d) for d in drop)}
        meta = {"mode": mode, "args": " ".join(args)}
        if "env_is_reference" in arrs:
            # which environment the reference learner drove (ref_harness.cc)
            kv = dict(a.split("=", 1) for a in args)
            meta["env"] = ("bp::environment (apps/bin_packing/bin_packing.h%s)"
                           % (", num_bins = 64" if name in BP64 else "")
                           if arrs["env_is_reference"][0] else
                           "gen_env<%s,%s> (ref_harness.cc)" % (kv["B"], kv["D"]))
        for k, v in meta.items():
            arrs["meta_" + k] = np.array(v)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **arrs)
        print("%-10s %8d bytes  %d arrays" % (name, os.path.getsize(path),
                                                len(arrs)))


if __name__ == "__main__":
    main(sys.argv[1:])
