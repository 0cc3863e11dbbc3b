#!/usr/bin/env python3
"""Benchmark: PPO env-steps/s on vectorised 64-bin x 2-D bin packing.

BASELINE.json metric "env-steps/sec (whole node) PPO bin-packing 64-bin";
workload = BASELINE config 3 per GPU (32768 envs, 64 bins, D=2, per-bin
policy [128,128], value [256,64,32], T=4, k=4 PPO epochs), weak-scaled over
N GPUs (config 4 at N=8).  A "step" is one training iteration: T env steps
of every env + learn() (value step, GAE, 4 policy epochs), i.e. N*T env-steps.

    python bench.py [--gpus N --steps K --warmup W] [--config 2|3|5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Prints ONE JSON line (rank 0).  The timed region starts with all state
resident in HBM; rank 0 additionally times the reference CPU path
(oracle/_ref, single thread) on a bounded sample: `cpu_baseline`.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# BASELINE.json configs that run on the device (config 1 is the CPU-only
# REINFORCE plumbing case; config 4 = config 3 per GPU at N=8).  The default
# and headline is config 3; --config 2 / 5 measure the other shapes.
CONFIGS = {
    2: dict(algo="ppo", B=32, D=1, N=4096, T=4, H=(64, 64), epochs=4,
            ref_iters=100,
            name="PPO, 1-D bin packing 32 bins, %d envs/GPU, per-bin policy "
                 "[64,64], value [64,64,32], T=4, k=4"),
    3: dict(algo="ppo", B=64, D=2, N=32768, T=4, H=(128, 128), epochs=4,
            ref_iters=60,
            name="PPO, 2-D bin packing 64 bins, %d envs/GPU, per-bin policy "
                 "[128,128], value [256,64,32], T=4, k=4"),
    5: dict(algo="ac", B=128, D=3, N=16384, T=8, H=(128, 128), epochs=1,
            ref_iters=20,
            name="online actor-critic, 3-D bin packing 128 bins, %d envs/GPU, "
                 "per-bin policy [128,128], value [768,64,32], T=8"),
}
B, D, T, H1, H2, V1, V2 = 64, 2, 4, 128, 128, 64, 32
F0 = 2 * D
ALGO, EPOCHS, REF_ITERS = "ppo", 4, 60


def select_config(c):
    global B, D, T, H1, H2, F0, ALGO, EPOCHS, REF_ITERS
    k = CONFIGS[c]
    B, D, T, (H1, H2) = k["B"], k["D"], k["T"], k["H"]
    F0, ALGO, EPOCHS, REF_ITERS = 2 * D, k["algo"], k["epochs"], k["ref_iters"]
    return k
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32 MFMA (= f32 vector) peak
# Which kernels ran, and the MFMA peak of their arithmetic, come from the
# library itself (xh_trainer_kernel_info): the 64- and 128-bin train kernels
# run layer 2 on f16 pairs (three f16 products per f32 product), dH1 on f16
# pairs against the exact mask (two) and dW2 on the exact bf16 split (three):
# eight products per three f32 products, peak = dense 2500 / (8/3); the
# split rollouts' layer 2 on f16 pairs: dense 2500 / 3.
# Diagnostic variables that steer kernel selection (the bench refuses them
# unless --allow-kernel-override is given):
KERNEL_OVERRIDES = ("XH_TRAIN_KERNEL", "XH_ROLLOUT_KERNEL", "XH_VALUE_KERNEL",
                    "XH_W0_FUSE")
HBM_PEAK_GBS = 8000.0
# the line's dtype names the arithmetic the train kernel ran (its `math`
# from xh_trainer_kernel_info): f32 values on 16-bit matrix cores, exactly
# split, f32 accumulation
TRAIN_DTYPE = {
    "f32_mfma": "f32",
    "f16_pair_bf16_split": "f32 via f16-pair (layer 2, dH1) / 3-part bf16 "
                           "split (dW2) MFMA, f32 accumulate",
    "bf16_split": "f32 via 3-part bf16 split MFMA, f32 accumulate",
}
PHASE_ITERS = 3  # the phase-breakdown pass after the timed region


def kernel_roofline(k, flops_per_launch, avg_ms):
    """Roofline of one kernel from what the library says ran (an entry of
    xh_trainer_kernel_info): its name, arithmetic and that arithmetic's MFMA
    peak.  Nothing here re-derives the kernel selection."""
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    return {"kernel": k["kernel"], "bound": "mfma", "math": k["math"],
            "bf16_products_per_f32_product": k["bf16_products_per_f32_product"],
            "products_per_f32_product": k.get("products_per_f32_product"),
            "math_source": "xh_trainer_kernel_info",
            "achieved": round(achieved, 2), "peak": round(k["peak_tflops"], 1),
            "unit": "TFLOP/s", "frac": round(achieved / k["peak_tflops"], 4),
            "frac_of_f32_mfma_peak": round(achieved / FP32_PEAK_TFLOPS, 4)}


def policy_fwd_flops_per_env_step():
    # 2*B*(F0*H1 + H1*H2 + H2): per-bin Dense chain
    return 2 * B * (F0 * H1 + H1 * H2 + H2)


def value_fwd_flops_per_row():
    fin = B * F0
    return 2 * (fin * V1 + V1 * V2 + V2)


def _harness_cmd(harness, n_env, iters, seed):
    return [harness, "bench", "algo=%s" % ALGO, "B=%d" % B, "D=%d" % D,
            "widths=%d,%d" % (H1, H2), "N=%d" % n_env, "T=%d" % T,
            "iters=%d" % iters, "seed=%d" % seed]


def host_cores():
    """CPU cores this process may use, capped at the GPU box's per-GPU share
    (16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline():
    """Time the reference's single-threaded CPU path (oracle/_ref/ref_harness
    = the reference's own ppo_learner / actor_critic_learner and agents,
    compiled from its sources) on a bounded sample of the same workload:
    first one process alone (the single-core rate), then one independent
    seeded process per usable core at once (the whole-host rate, SURVEY
    8(d): the reference path is single-threaded, so a whole host runs it as
    that many independent processes).  About 2 x 8 s."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    # config 3 (64 bins, 2-D): the harness built against the reference's own
    # bin_packing.h with num_bins = 64, i.e. bp::environment / bp::agent
    # themselves (oracle/Makefile); the other shapes run gen_env<B,D>
    bp64 = os.path.join(REPO, "oracle", "_ref", "ref_harness_bp64")
    env_src = "gen_env<%d,%d>" % (B, D)
    if B == 64 and D == 2 and os.path.exists(bp64):
        harness, env_src = bp64, "bp::environment (bin_packing.h, num_bins = 64)"
    n_env, iters = 16, max(1, REF_ITERS // 3)
    learner = {"ppo": "ppo_learner", "klppo": "kl_ppo_learner (ppo2_training.cc)",
               "ac": "actor_critic_learner"}[ALGO]
    sample = ("reference %s on %s, %d envs x T=%d x %d iterations per "
              "process, B=%d D=%d [%d,%d], single-threaded processes" % (
                  learner, env_src, n_env, T, iters, B, D, H1, H2))
    if os.path.exists(harness):
        try:
            out = subprocess.run(_harness_cmd(harness, n_env, iters, 1),
                                 capture_output=True, text=True, timeout=600,
                                 check=True)
            single = json.loads(out.stdout.strip().splitlines()[-1])
            cores = host_cores()
            procs = [subprocess.Popen(_harness_cmd(harness, n_env, iters, 1 + k),
                                      stdout=subprocess.PIPE, text=True)
                     for k in range(cores)]
            rates = []
            for p in procs:
                o, _ = p.communicate(timeout=600)
                if p.returncode != 0:
                    raise RuntimeError("harness rc %d" % p.returncode)
                rates.append(json.loads(o.strip().splitlines()[-1])["env_steps_per_s"])
            return {"value": round(sum(rates), 3), "unit": "env-steps/s",
                    "cores": cores, "kind": "reference",
                    "sample": sample + "; value = sum over %d concurrent "
                              "processes" % cores,
                    "single_core": round(single["env_steps_per_s"], 3),
                    "per_process_min": round(min(rates), 3)}
        except Exception as e:  # fall through to the port
            print("cpu_baseline: reference harness failed: %s" % e,
                  file=sys.stderr)
    # the reference harness is built from /root/reference in the build
    # container; without it, the oracle port (the reference's loop structure
    # restated in C) is timed instead and `kind` says so
    from oracle import pyoracle as po
    from dependence_free_rl_amd.trainer import init_policy, init_value
    n_env, iters = 8, 3
    pol = po.perbin_model(F0, [H1, H2],
                          po.OR_SOFTMAX_XENT if ALGO == "ac" else po.OR_SOFTMAX)
    val = po.full_model(B * F0, [V1, V2], 1)
    tr = po.Trainer({"ppo": po.OR_PPO, "klppo": po.OR_KLPPO, "ac": po.OR_AC}[ALGO],
                    B, D, n_env, T,
                    pol, init_policy(D, H1, H2),
                    val, init_value(B, D), x0=1)
    t0 = time.perf_counter()
    for _ in range(iters):
        tr.rollout()
        tr.learn()
    dt = time.perf_counter() - t0
    return {"value": round(n_env * T * iters / dt, 3), "unit": "env-steps/s",
            "cores": 1, "kind": "port",
            "sample": "oracle port (%s), %d envs x T=%d x %d iterations" % (ALGO,
                n_env, T, iters)}


def library_sha256():
    """sha256 of the libxylo_hip.so this process loaded (the build the PMC
    summaries must have profiled to be cited)."""
    import hashlib
    from dependence_free_rl_amd import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def pmc_traffic(kernel="policy_train", any_shape=False, lib_sha=None,
                meta_match=None, envs=None):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 FETCH_SIZE /
    WRITE_SIZE summary (separate --pmc passes; tools/pmc_summary.py):
    2 x FETCH_SIZE + WRITE_SIZE, the gfx950 read correction measured for 1- to
    16-byte lanes by tools/probes/fetch_probe.hip.

    Only a summary of THIS library build is cited: its "_meta".library_sha256
    must equal `lib_sha` (the sha256 of the loaded libxylo_hip.so; a summary
    of another build -- older kernels -- gives None).  Among matching
    summaries the newest by its recorded creation time wins, and only a
    summary of this very shape counts (PShape<B, D, H1, H2> for the f32
    kernels; the split kernels have one shape each)."""
    import glob
    shape = "PShape<%d, %d, %d, %d>" % (B, D, H1, H2)
    best = None
    for path in glob.glob(os.path.join(REPO, "profiles", "*_pmc_summary.json")):
        with open(path) as f:
            summ = json.load(f)
        meta = summ.get("_meta", {})
        if lib_sha is None or meta.get("library_sha256") != lib_sha:
            continue
        if meta_match and any(meta.get(k) != v for k, v in meta_match.items()):
            continue
        # a summary that records its run's env count (tools/gpu_profile_env.sh)
        # counts only for that count: bytes per launch scale with it
        if envs is not None and meta.get("envs", envs) != envs:
            continue
        # keys are short kernel names (policy_train_kernel, policy_train8_kernel)
        s = next((v for k, v in sorted(summ.items())
                  if k.startswith(kernel) and (any_shape or shape in v.get("kernel", ""))
                  and "hbm_bytes" in v), None)
        if s and (best is None or meta.get("created", "") > best[0]):
            best = (meta.get("created", ""), s["hbm_bytes"],
                    os.path.relpath(path, REPO), s)
    if best is None:
        return None, None, None
    return best[1], best[2], best[3]


# bytes one venv step moves per env (venv_kernels.hip venv_step_kernel, mode
# 1): the bins read and written (B*D int8 each), the action read (4), the
# item record read and written (4 + 4), the engine state read and written
# (4 + 4), the reward (4) and done (1) written
def venv_bytes_per_env_step():
    return 2 * B * D + 4 + 8 + 8 + 4 + 1


def env_only(args, cfg, ctx, rank, world, rdzv):
    """--env-only: the env half of the path alone:
    xh_venv_step -- agent::step minus react for every env in ONE kernel
    (bin_packing.h:53-70, rl.h:325-349) -- over the config's env batch, each
    env replaying a fixed bin choice (uploaded once; an env overflows its
    bin within a few steps and resets, so apply, the item draws and reset
    all run), streams in reference order with a sampling policy's 2 draws
    skipped per step.  HBM-bound: `roofline` is HBM GB/s of venv_step_kernel
    (algorithmic bytes / HIP-event launch time) against 8 TB/s.  Beside it,
    the reference's first-fit heuristic agent (firstfit_agent.cc:10-28) on
    the device evaluator, whole episodes with the state in registers."""
    from dependence_free_rl_amd.trainer import heuristic_evaluate
    from dependence_free_rl_amd.venv import VecEnv
    n = args.envs or cfg["N"]
    env = VecEnv(ctx, n, bins=B, dims=D, rng_state=20241008, env_offset=n * rank,
                 num_envs_global=n * world, policy_draws=2)
    env.set_actions(np.random.default_rng(1234 + rank).integers(0, B, n))
    for _ in range(args.warmup):
        env.step(fetch=False)
    env.synchronize()
    if rdzv:
        rdzv.barrier()
    # the timed region carries no events; the per-launch HIP-event average
    # comes from a second pass of the same launches after it
    t0 = time.perf_counter()
    for _ in range(args.steps):
        env.step(fetch=False)
    env.synchronize()
    if rdzv:
        rdzv.barrier()
    dt = time.perf_counter() - t0
    if rdzv:
        dt = rdzv.allreduce_max(dt)
    env.set_timing(True)
    for _ in range(args.steps):
        env.step(fetch=False)
    env.synchronize()
    ms, launches = env.kernel_time()
    env.set_timing(False)
    avg_ms = ms / max(launches, 1)
    reward, done = env.get(_venv_reward()), env.get(_venv_done())
    env.close()
    value = n * world * args.steps / dt
    bytes_launch = n * venv_bytes_per_env_step()
    achieved = bytes_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    # a summary of this library's env-only run at this env count and shape
    # (tools/gpu_profile_env.sh records them in its _meta)
    traffic, traffic_src, pmc = pmc_traffic(
        "venv_step_kernel", any_shape=True, lib_sha=library_sha256(),
        meta_match={"workload": "env_only", "envs": n, "bins": B, "dims": D})
    # the first-fit agent: 4 episodes of every env on the device evaluator
    # (its own kernel, whole episodes with the env state in registers)
    ff = heuristic_evaluate(ctx, "firstfit", B, D, n, 4, 20241008 + rank)
    ff_steps = int(ff["steps"].sum())
    line = {
        "metric": "env-steps/sec (whole node) bin-packing env step, %d-bin "
                  "%d-D, env only" % (B, D),
        "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic (fixed-size bin-packing instances; every env "
                "replays a fixed random bin choice)",
        "config": {"workload": "env only (xh_venv_step) on the env batch of "
                               "BASELINE config %d: %d envs/GPU, %d bins, %d-D"
                               % (args.config, n, B, D),
                   "envs_per_gpu": n, "bins": B, "dims": D,
                   "parallelism": "dp%d" % world},
        "roofline": {"kernel": "venv_step_kernel<%d, %d>" % (B, D),
                     "bound": "hbm", "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "traffic_over_algorithmic": (round(traffic / bytes_launch, 3)
                                                  if traffic else None),
                     "occupancy": pmc and pmc.get("occupancy"),
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "bytes_per_env_step": venv_bytes_per_env_step(),
                     "avg_launch_ms": round(avg_ms, 5)},
        "health": {"done_rate": float(done.mean()),
                   "reward_mean": float(reward.mean())},
        "firstfit_agent": {
            "env_steps_per_s": round(ff_steps / (ff["elapsed_ms"] * 1e-3), 1)
            if ff["elapsed_ms"] > 0 else None,
            "env_steps": ff_steps, "episodes": 4 * n,
            "mean_episode_reward": float(ff["totals"].sum() / (4 * n)),
            "device_ms": round(ff["elapsed_ms"], 3),
            "source": "xh_heuristic_evaluate (firstfit_agent.cc:10-28), "
                      "HIP events around its launch"},
    }
    if rank == 0:
        print(json.dumps(line), flush=True)


def _venv_reward():
    from dependence_free_rl_amd._lib import VENV_REWARD
    return VENV_REWARD


def _venv_done():
    from dependence_free_rl_amd._lib import VENV_DONE
    return VENV_DONE


_VISIBLE_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                 "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")


def visible_devices_no_hip():
    """GPUs this process could open, counted WITHOUT initialising HIP (the
    launcher parent must never touch the device: a process that has
    initialised HIP may not start the ranks by exec, and the ranks must be
    the first HIP users of their devices).  A GPU is a KFD topology node with
    SIMDs whose DRM render node this process may open; a non-empty
    *_VISIBLE_DEVICES list caps the count at its length."""
    import glob
    n = 0
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        kv = {}
        try:
            with open(props) as f:
                for line in f:
                    p = line.split()
                    if len(p) == 2:
                        kv[p[0]] = p[1]
        except OSError:
            continue
        if int(kv.get("simd_count", "0")) <= 0:
            continue  # a CPU node
        minor = kv.get("drm_render_minor")
        if minor is not None and not os.access("/dev/dri/renderD%s" % minor,
                                               os.R_OK | os.W_OK):
            continue  # not passed into this container / cgroup
        n += 1
    for var in _VISIBLE_VARS:
        v = os.environ.get(var, "").strip()
        if v:
            n = min(n, len([e for e in v.split(",") if e.strip()]))
    return n


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: start the N
    rank processes here (one per GPU, the same contract torch.distributed.run
    gives them: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, and
    XH_RDZV_PORT for the torch-free rendezvous), relay rank 0's JSON line
    (the children inherit stdout; only rank 0 prints) and exit with the worst
    child status.  This process never initialises HIP and never execs."""
    import signal
    n = args.gpus
    if not args.dry_run_ranks:
        have = visible_devices_no_hip()
        if have < n:
            print("bench.py: --gpus %d needs %d devices, %d visible (KFD "
                  "topology nodes with an accessible render node); not "
                  "starting the ranks" % (n, n, have), file=sys.stderr)
            return 3
    port = _free_port()
    base = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                XH_RDZV_PORT=str(port))
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)]
                                      + argv, env=env))
    rcs = [None] * n
    failed = False
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] not in (None, 0) and not failed:
                    failed = True
                    print("bench.py: rank %d exited with %d; stopping the "
                          "others" % (i, rcs[i]), file=sys.stderr)
                    for q in procs:
                        if q.poll() is None:
                            q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    worst = 0
    for rc in rcs:
        code = rc if rc >= 0 else 128 - rc
        worst = max(worst, code)
    return worst


def dry_run_rank(rank, world, local):
    """--dry-run-ranks: a rank's plumbing without the device -- its env, the
    rendezvous (an id broadcast, barriers, the max-over-ranks of its wall
    time) and rank 0's one line; stops before any HIP call."""
    print("bench.py rank env: %s" % json.dumps(
        {"RANK": rank, "LOCAL_RANK": local, "WORLD_SIZE": world,
         "MASTER_ADDR": os.environ.get("MASTER_ADDR"),
         "XH_RDZV_PORT": os.environ.get("XH_RDZV_PORT"), "pid": os.getpid()}),
        file=sys.stderr, flush=True)
    ranks = [{"rank": rank, "local_rank": local, "pid": os.getpid()}]
    dt = 0.001 * (rank + 1)
    if world > 1:
        # the module file alone: the package's __init__ loads libxylo_hip.so
        import importlib.util
        spec = importlib.util.spec_from_file_location(
            "xh_rendezvous", os.path.join(REPO, "dependence_free_rl_amd",
                                          "rendezvous.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        rdzv = mod.Rendezvous(rank, world)
        uid = rdzv.broadcast(bytes(range(128)) if rank == 0 else None)
        assert uid == bytes(range(128))
        rdzv.barrier()
        got = rdzv.gather(json.dumps(ranks[0]).encode())
        dt = rdzv.allreduce_max(dt)
        rdzv.barrier()
        rdzv.close()
        if rank == 0:
            ranks = [json.loads(g) for g in got]
    if rank == 0:
        print(json.dumps({"metric": "dry run (rank plumbing only, no device)",
                          "value": None, "n_gpus": world, "dry_run": True,
                          "max_rank_time_s": dt, "ranks": ranks}), flush=True)
    assert "dependence_free_rl_amd._lib" not in sys.modules  # no HIP loaded
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks = GPUs of this node (default: WORLD_SIZE, else "
                         "1).  Without WORLD_SIZE in the environment, N > 1 "
                         "starts the N rank processes itself")
    ap.add_argument("--dry-run-ranks", action="store_true",
                    help="start / join the ranks and their rendezvous, print "
                         "rank 0's line, and stop before any HIP call")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS),
                    help="BASELINE.json config (3 = the headline)")
    ap.add_argument("--envs", type=int, default=None,
                    help="envs per GPU (default: the config's)")
    ap.add_argument("--rollout-steps", type=int, default=None,
                    help="T, env steps per env per iteration (default: the "
                         "config's; SURVEY 8(d)'s larger-T throughput point)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--allow-kernel-override", action="store_true",
                    help="run even if XH_TRAIN_KERNEL / XH_ROLLOUT_KERNEL / XH_VALUE_KERNEL / "
                         "XH_W0_FUSE are "
                         "set (A/B measurements; the line records them)")
    ap.add_argument("--algo", choices=("ppo", "klppo", "ac"), default=None,
                    help="learner on the config's shape (default: the "
                         "config's; klppo = kl_ppo_learner, a side line, not "
                         "the headline)")
    ap.add_argument("--env-only", action="store_true",
                    help="the env step alone (xh_venv_step over the config's "
                         "env batch, HBM roofline) instead of training")
    ap.add_argument("--reference-lr", action="store_true",
                    help="raw lr on row sums as the reference (diverges at "
                         "this batch size; default: lr_scale_rows)")
    argv = sys.argv[1:]
    args = ap.parse_args(argv)
    set_over = {k: os.environ[k] for k in KERNEL_OVERRIDES if k in os.environ}
    if set_over and not args.allow_kernel_override:
        print("bench.py: kernel-selection override(s) set %s; unset them or "
              "pass --allow-kernel-override" % set_over, file=sys.stderr)
        sys.exit(2)
    cfg = select_config(args.config)
    if args.algo:
        global ALGO
        ALGO = args.algo
    if args.rollout_steps:
        global T
        T = args.rollout_steps

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if args.gpus is not None and args.gpus != int(env_world):
            print("bench.py: --gpus %d disagrees with WORLD_SIZE=%s" % (
                args.gpus, env_world), file=sys.stderr)
            sys.exit(2)
    elif (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args, argv))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run_ranks:
        sys.exit(dry_run_rank(rank, world, local))
    rdzv = None
    uid = None
    device = local
    if world > 1:
        # one node by the bench contract: RCCL's bootstrap stays on loopback
        # (the container hostname may not resolve).  No torch in this process
        # (its bundled HIP / RCCL would shadow /opt/rocm's under the same
        # sonames): the unique id, the barriers and the max-time reduce go
        # over a plain TCP star (dependence_free_rl_amd/rendezvous.py).
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        from dependence_free_rl_amd import Context, device_count
        from dependence_free_rl_amd.rendezvous import Rendezvous
        ndev = device_count()
        if local >= ndev:
            narrowed = [v for v in _VISIBLE_VARS
                        if len([e for e in os.environ.get(v, "").split(",")
                                if e.strip()]) == 1]
            if ndev == 1 and narrowed:  # a launcher gave each rank one device
                device = 0
            else:  # two ranks on one device: RCCL refuses them; fail first
                print("bench.py: rank %d (LOCAL_RANK %d) of %d needs device %d;"
                      " %d visible" % (rank, local, world, local, ndev),
                      file=sys.stderr)
                sys.exit(3)
        rdzv = Rendezvous(rank, world)
        uid = rdzv.broadcast(Context.unique_id() if rank == 0 else None)

    from dependence_free_rl_amd import (POLICY, VALUE, Context, Trainer,
                                        init_policy, init_value, runtime_info)
    ctx = Context(device=device, rank=rank, world=world, uid=uid)
    if args.env_only:
        env_only(args, cfg, ctx, rank, world, rdzv)
        ctx.close()
        if rdzv:
            rdzv.close()
        return
    n = args.envs or cfg["N"]
    # lr_scale_rows: the reference applies its raw lr to row SUMS (nn.h:
    # 94-98, 624); at this batch (N*T*B rows per epoch) that diverges to
    # non-finite probabilities within ~25 iterations (test_gpu_scale.py), so
    # the bench runs the documented opt-in lr / rows (same work, same kernels;
    # off in every parity test)
    tr = Trainer(ctx, algo=ALGO, bins=B, dims=D, num_envs=n, steps=T,
                 widths=(H1, H2), value_widths=(V1, V2), rng_state=20241008,
                 num_envs_global=n * world, env_offset=n * rank,
                 lr_scale_rows=not args.reference_lr)
    # random-init weights of the reference architecture (same on every rank)
    tr.set_params(POLICY, init_policy(D, H1, H2, seed=0))
    tr.set_params(VALUE, init_value(B, D, V1, V2, seed=1))

    if args.warmup:
        tr.iterate(args.warmup)
    tr.synchronize()
    if rdzv:
        rdzv.barrier()
    # inside the timed region only the policy train launches carry HIP events
    # (the dominant kernel's average duration); per-launch events on every
    # launch cost ~2 us each (config 2: 0.40 -> 0.47 ms per iteration), so the
    # phase breakdown comes from a separate pass after the timed region
    tr.set_timing("train")
    tr.reset_timing()
    t0 = time.perf_counter()
    tr.iterate(args.steps)
    tr.synchronize()
    if rdzv:
        rdzv.barrier()
    dt = time.perf_counter() - t0
    if rdzv:
        dt = rdzv.allreduce_max(dt)

    ms_pt, n_pt = tr.kernel_time("policy_train")
    # KL-PPO trains every row of kl_ppo_learner's state matrix: the N T
    # transitions, N open end rows and the n_end terminal end rows of the
    # batch -- read from the done flags of the LAST TIMED iteration, before
    # the phase pass below overwrites them (the other timed iterations' counts
    # are not kept; they differ by a fraction of a percent)
    n_end = None
    if ALGO == "klppo":
        from dependence_free_rl_amd.trainer import BUF_DONE
        n_end = int(np.asarray(tr.buffer(BUF_DONE)).astype(np.int64).sum())
    # the phase pass also records the last step's probabilities (diagnostics,
    # off inside the timed region) for the health check after it
    # the phase breakdown: PHASE_ITERS more iterations (every rank), every
    # launch timed
    tr.set_timing(True)
    tr.set_record_last_step(True)
    tr.iterate(1)  # (the events' own first use)
    tr.reset_timing()
    tr.iterate(PHASE_ITERS)
    tr.synchronize()
    ph = {k: tr.kernel_time(k)[0] / PHASE_ITERS
          for k in ("rollout_step", "policy_train", "value", "reduce_sgd",
                    "allreduce")}
    tr.set_timing(False)
    # numerical health (after the timed region): finite parameters and
    # last-step probabilities, done rate and mean episode length
    health = tr.health()
    env_steps = n * world * T * args.steps
    value = env_steps / dt
    # dominant kernel: policy_train (one PPO epoch over N*T env-steps);
    # algorithmic FLOPs = fwd + bwd(2x fwd) of the per-bin policy per env-step
    # (KL-PPO trains every row of kl_ppo_learner's state matrix: the N T
    # transitions, N open end rows and the last iteration's n_end terminal
    # end rows -- their count read from its done flags)
    rows_epoch = n * T
    if ALGO == "klppo":
        rows_epoch += n + n_end
    flops_epoch = 3.0 * policy_fwd_flops_per_env_step() * rows_epoch
    avg_ms = ms_pt / max(n_pt, 1)
    # what ran, and the peak of its arithmetic: from the library
    kinfo = tr.kernel_info()
    if kinfo.get("train_grid_cap"):  # test-only depth control (xh_config)
        print("bench.py: the trainer ran with train_grid_cap %d; the bench "
              "measures the library's own grid only" % kinfo["train_grid_cap"],
              file=sys.stderr)
        sys.exit(2)
    kt, kr = kinfo["policy_train"], kinfo["rollout_step"]
    split = kt["math"] != "f32_mfma"
    # the split kernels have one shape each: their summaries are keyed by
    # name; the f32 kernels by their PShape<B, D, H1, H2> instantiation
    lib_sha = library_sha256()
    traffic, traffic_src, pmc = (
        pmc_traffic(kt["kernel"], any_shape=True, lib_sha=lib_sha, envs=n) if split
        else pmc_traffic(lib_sha=lib_sha, envs=n))
    if args.rollout_steps and args.rollout_steps != cfg["T"]:
        # the PMC passes profile the config's own T: their bytes per launch
        # are not this launch's
        traffic, traffic_src = None, None
    train_peak = kt["peak_tflops"]
    # compulsory bytes of one epoch: per env-step state (B*D + 4 B) + action,
    # p_old, advantage (12 B); per workgroup of the train grid (the library
    # reports it: 256 at configs 3 / 5, 512 at config 2) one f32 gradient slab
    from dependence_free_rl_amd.trainer import policy_param_count
    # (KL-PPO rows also read their old distribution, B floats)
    alg_bytes = (rows_epoch * (B * D + 4 + 12 + (4 * B if ALGO == "klppo" else 0)) +
                 kinfo["train_grid"] * policy_param_count(D, H1, H2) * 4)
    roofline = kernel_roofline(kt, flops_epoch, avg_ms)
    # whole-iteration HBM roofline (BASELINE metric: "fraction of the HBM
    # roofline"): compulsory bytes per env-step, SURVEY §8d -- env state
    # read + write (2*B*D int8) and one trajectory record (B*D state + D item
    # + action, p_old, reward, V (4 B each) + done (1 B)) written once and read
    # 3 + k times; params and slabs excluded.
    rec = B * D + D + 4 * 4 + 1
    hbm_bytes_per_step = 2 * B * D + rec * (1 + 3 + EPOCHS)
    hbm_gbs = value * hbm_bytes_per_step / 1e9
    # whole-iteration compute roofline: (1 + 3k) Fp + 5 Fv
    # algorithmic FLOPs per env-step -- the rollout forward, k epochs of
    # forward + backward, and the value net's evaluations and step
    it_flops = ((1 + 3 * EPOCHS) * policy_fwd_flops_per_env_step() +
                5 * value_fwd_flops_per_row())
    it_tflops = value * it_flops / 1e12
    # roofline time of one env-step: the rollout forward at its kernel's
    # peak (bf16-split at 64 bins), the value net at the f32 MFMA peak, the k
    # train epochs at the train kernel's peak; frac = that time x the
    # measured env-steps/s
    roll_peak = kr["peak_tflops"]
    it_ideal_s = (policy_fwd_flops_per_env_step() / (roll_peak * 1e12) +
                  5 * value_fwd_flops_per_row() / (FP32_PEAK_TFLOPS * 1e12) +
                  3 * EPOCHS * policy_fwd_flops_per_env_step() / (train_peak * 1e12))
    if args.config == 3 and ALGO == "ppo":
        metric = "env-steps/sec (whole node) PPO bin-packing 64-bin"
        workload = "BASELINE config %d: " % (3 if world == 1 else 4)
    elif ALGO != cfg["algo"]:
        metric = "env-steps/sec (whole node) %s bin-packing %d-bin %d-D" % (
            {"ppo": "PPO", "klppo": "KL-PPO", "ac": "actor-critic"}[ALGO], B, D)
        workload = "side line, %s on the shape of BASELINE config %d: " % (
            ALGO, args.config)
    else:
        metric = "env-steps/sec (whole node) %s bin-packing %d-bin %d-D" % (
            "PPO" if ALGO == "ppo" else "actor-critic", B, D)
        workload = "BASELINE config %d: " % args.config
    line = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": TRAIN_DTYPE.get(kt["math"], "f32 (%s)" % kt["math"]),
        "data": "synthetic (fixed-size bin-packing instances, random-init "
                "weights of the reference architecture)",
        "config": {"workload": workload + cfg["name"] % n + (
                       "; larger-T point: T=%d" % T if args.rollout_steps
                       else ""),
                   "learner": ALGO,
                   "envs_per_gpu": n, "bins": B, "dims": D, "T": T,
                   "epochs": EPOCHS, "parallelism": "dp%d" % world,
                   "lr_scale_rows": not args.reference_lr},
        "roofline": dict(roofline, **{
                     "traffic": traffic,
                     "traffic_source": traffic_src,
                     "library_sha256": lib_sha,
                     "mfma_busy_frac": pmc and pmc.get("mfma_busy_frac"),
                     "clock_ghz_profiled": pmc and pmc.get("clock_ghz"),
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "avg_launch_ms": round(avg_ms, 4),
                     "flops_per_launch": flops_epoch,
                     "rows_per_launch": rows_epoch}),
        "iteration_roofline": {"flops_per_env_step": it_flops,
                               "achieved": round(it_tflops, 2),
                               "unit": "TFLOP/s",
                               "roofline_s_per_env_step": it_ideal_s,
                               "frac": round(value / world * it_ideal_s, 4)},
        "hbm_roofline": {"bytes_per_env_step": hbm_bytes_per_step,
                         "achieved": round(hbm_gbs, 2),
                         "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                         "frac": round(hbm_gbs / (HBM_PEAK_GBS * world), 6)},
        "health": health,
        "kernels": kinfo,
        "runtime": runtime_info(),
        "phase_ms_per_step": {
            "rollout": round(ph["rollout_step"], 3),
            "policy_train": round(ph["policy_train"], 3),
            "value": round(ph["value"], 3),
            "reduce_sgd": round(ph["reduce_sgd"], 3),
            "allreduce": round(ph["allreduce"], 3),
            "source": "%d iterations after the timed region, HIP events on "
                      "every launch" % PHASE_ITERS},
    }
    # the CPU baseline is timed on rank 0 of the N=1 run only
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(line), flush=True)
    tr.close()
    ctx.close()
    if rdzv:
        rdzv.close()


if __name__ == "__main__":
    main()
