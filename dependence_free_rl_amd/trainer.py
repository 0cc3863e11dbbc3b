"""Python host wrapper over the C ABI: one process per GPU.

Mirrors the reference's learner vocabulary (xylo/policy_gradient.h,
apps/bin_packing/bin_packing.h) for the vectorised path:

    ctx = Context(device=0)
    tr = Trainer(ctx, algo="ppo", bins=64, dims=2, num_envs=32768, steps=4,
                 widths=(128, 128))
    tr.set_params(POLICY, w); tr.set_params(VALUE, v)
    tr.iterate(10)           # 10 x (agents.play_steps(T); learner.step())

All arrays crossing this wrapper are numpy host copies; the hot loop never
leaves the device.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import (BUF_ACTION, BUF_ADV, BUF_BINS, BUF_DONE, BUF_ITEMS,
                   BUF_KL, BUF_LEN, BUF_LOGITS, BUF_POLD, BUF_POLICY_GRADS, BUF_PROBS,
                   BUF_QOLD, BUF_RNG, BUF_TARGETS, BUF_V_STATE, BUF_V_STATE0,
                   BUF_V_TERM, BUF_VALUE_GRAD, XH_AC, XH_KLPPO, XH_PG,
                   XH_POLICY, XH_PPO, XH_VALUE, check)

POLICY, VALUE = XH_POLICY, XH_VALUE
ALGOS = {"ppo": XH_PPO, "ac": XH_AC, "klppo": XH_KLPPO, "pg": XH_PG}


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class Context:
    """xh_ctx: a device, its stream and (world > 1) an RCCL communicator."""

    def __init__(self, device=0, rank=0, world=1, uid=None):
        self.h = C.c_void_p()
        buf = None
        if uid is not None:
            buf = (C.c_char * 128).from_buffer_copy(bytes(uid))
        check(_lib.lib.xh_ctx_create(device, rank, world,
                                     C.cast(buf, C.c_void_p) if buf else None,
                                     C.byref(self.h)))
        self.device, self.rank, self.world = device, rank, world

    @staticmethod
    def unique_id():
        out = (C.c_char * 128)()
        check(_lib.lib.xh_comm_unique_id(out))
        return bytes(out)

    def synchronize(self):
        check(_lib.lib.xh_ctx_synchronize(self.h))

    def allreduce_host(self, arr):
        a = np.ascontiguousarray(arr, np.float32).copy()
        check(_lib.lib.xh_ctx_allreduce_host(self.h, _ptr(a), a.size))
        return a

    def inject_fault(self, kind=1):
        """Test hook (xh_ctx_inject_fault): kind 1 makes the next gradient
        all-reduce pass RCCL an invalid argument; 0 clears it."""
        check(_lib.lib.xh_ctx_inject_fault(self.h, kind))

    def close(self):
        if self.h:
            check(_lib.lib.xh_ctx_destroy(self.h))
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _eval_struct(n_envs, episodes, rng_state, D, init_items, trace_cap,
                 argmax_probs=False):
    out = {"totals": np.zeros(n_envs, np.float64),
           "steps": np.zeros(n_envs, np.int64),
           "final_items": np.zeros((n_envs, D), np.int32),
           "rng": np.zeros(n_envs, np.uint32),
           "trace": np.zeros(max(trace_cap, 1), np.int32)}
    e = _lib.Eval()
    e.n_envs, e.episodes = n_envs, episodes
    e.argmax_probs, e.rng_state = 1 if argmax_probs else 0, rng_state
    keep = []
    if init_items is not None:
        init = np.ascontiguousarray(init_items, np.int32).reshape(n_envs, D)
        keep.append(init)
        e.init_items = init.ctypes.data
    e.final_items = out["final_items"].ctypes.data
    e.rng_out = out["rng"].ctypes.data
    e.totals = out["totals"].ctypes.data
    e.steps = out["steps"].ctypes.data
    if trace_cap > 0:
        e.trace, e.trace_cap = out["trace"].ctypes.data, trace_cap
    return e, out, keep


def _eval_result(e, out, trace_cap):
    if trace_cap <= 0:
        del out["trace"]
    out["elapsed_ms"] = e.elapsed_ms
    return out


def heuristic_evaluate(ctx, kind, bins, dims, n_envs, episodes, rng_state,
                       init_items=None, trace_cap=0):
    """The reference's heuristic agents (firstfit / bestfit / minwaste /
    random) on the device: n_envs independent envs (multiple of 64/bins),
    `episodes` episodes each; env 0 reproduces a single-env reference run
    seeded at rng_state.  Returns totals, steps, final_items, rng, trace,
    elapsed_ms (device time)."""
    e, out, keep = _eval_struct(n_envs, episodes, rng_state, dims, init_items,
                                trace_cap)
    check(_lib.lib.xh_heuristic_evaluate(ctx.h, _lib.HEURISTICS[kind], bins,
                                         dims, C.byref(e)))
    del keep
    return _eval_result(e, out, trace_cap)


def model_eval(ctx, layers, params, x):
    """xylo::model::eval on the device (xh_model_eval).  layers: sequence of
    (kind, in, out) with kind in "full" | "conv1d_1" | "relu" | "softmax" |
    "softmax_xent" (in / out ignored for the activations); x: [rows][cols]."""
    kinds = {"full": _lib.LAYER_FULL, "conv1d_1": _lib.LAYER_CONV1D_1,
             "relu": _lib.LAYER_RELU, "softmax": _lib.LAYER_SOFTMAX,
             "softmax_xent": _lib.LAYER_SOFTMAX_XENT}
    arr = (_lib.Layer * len(layers))()
    for i, (k, a, b) in enumerate(layers):
        arr[i].kind, arr[i].inp, arr[i].out = kinds[k], a, b
    x = np.ascontiguousarray(x, np.float32)
    p = np.ascontiguousarray(params, np.float32)
    rows, cols = x.shape
    widest = max([cols] + [b * (cols // a if k == "conv1d_1" else 1)
                           for k, a, b in layers if k in ("full", "conv1d_1")])
    out = np.zeros(rows * widest, np.float32)
    oc = C.c_int()
    check(_lib.lib.xh_model_eval(ctx.h, arr, len(layers), _ptr(p), p.size,
                                 _ptr(x), rows, cols, _ptr(out), out.size,
                                 C.byref(oc)))
    return out[:rows * oc.value].reshape(rows, oc.value).copy()


_LAYER_KINDS = {"full": _lib.LAYER_FULL, "conv1d_1": _lib.LAYER_CONV1D_1,
                "relu": _lib.LAYER_RELU, "softmax": _lib.LAYER_SOFTMAX,
                "softmax_xent": _lib.LAYER_SOFTMAX_XENT}


def _layers(layers):
    arr = (_lib.Layer * len(layers))()
    for i, (k, a, b) in enumerate(layers):
        arr[i].kind, arr[i].inp, arr[i].out = _LAYER_KINDS[k], a, b
    return arr


def _widths(layers, cols):
    w = [cols]
    for k, a, b in layers:
        w.append(b if k == "full" else w[-1] // a * b if k == "conv1d_1"
                 else w[-1])
    return w


def model_forward(ctx, layers, params, x):
    """xylo::model::forward on the device (xh_model_forward): the input and
    every layer's output, as a list of [rows][width] arrays."""
    x = np.ascontiguousarray(x, np.float32)
    p = np.ascontiguousarray(params, np.float32)
    rows, cols = x.shape
    w = _widths(layers, cols)
    acts = np.zeros(rows * sum(w), np.float32)
    got = (C.c_int * (len(layers) + 1))()
    check(_lib.lib.xh_model_forward(ctx.h, _layers(layers), len(layers),
                                    _ptr(p), p.size, _ptr(x), rows, cols,
                                    _ptr(acts), acts.size, got))
    out, off = [], 0
    for k in range(len(layers) + 1):
        assert got[k] == w[k]
        out.append(acts[off:off + rows * w[k]].reshape(rows, w[k]).copy())
        off += rows * w[k]
    return out


def model_gradient(ctx, layers, params, inputs, target):
    """xylo::model::gradient on the device (xh_model_gradient): inputs = the
    first len(layers) arrays of model_forward, target = dL/d(output)."""
    p = np.ascontiguousarray(params, np.float32)
    rows, cols = inputs[0].shape
    flat = np.ascontiguousarray(np.concatenate([np.ravel(a) for a in
                                                inputs[:len(layers)]]),
                                np.float32)
    t = np.ascontiguousarray(target, np.float32)
    g = np.zeros(p.size, np.float32)
    check(_lib.lib.xh_model_gradient(ctx.h, _layers(layers), len(layers),
                                     _ptr(p), p.size, _ptr(flat), rows, cols,
                                     _ptr(t), t.shape[1], _ptr(g)))
    return g


def layer_backward(ctx, layer, params, x, backprop):
    """layer::backward of one layer on the device (xh_layer_backward)."""
    x = np.ascontiguousarray(x, np.float32)
    bp = np.ascontiguousarray(backprop, np.float32)
    p = np.ascontiguousarray(params, np.float32)
    out = np.zeros_like(x)
    check(_lib.lib.xh_layer_backward(ctx.h, _layers([layer]), _ptr(p), p.size,
                                     _ptr(x), x.shape[0], x.shape[1], _ptr(bp),
                                     bp.shape[1], _ptr(out)))
    return out


def layer_gradient(ctx, layer, x, backprop):
    """layer::gradient of one layer on the device (xh_layer_gradient)."""
    x = np.ascontiguousarray(x, np.float32)
    bp = np.ascontiguousarray(backprop, np.float32)
    k, a, b = layer
    n = a * b + b if k in ("full", "conv1d_1") else 0
    g = np.zeros(max(n, 1), np.float32)
    check(_lib.lib.xh_layer_gradient(ctx.h, _layers([layer]), _ptr(x),
                                     x.shape[0], x.shape[1], _ptr(bp),
                                     bp.shape[1], _ptr(g), n))
    return g[:n]


LOSSES = {"gradient_log": _lib.LOSS_GRADIENT_LOG,
          "policy_loss": _lib.LOSS_SOFTMAX_GRADIENT_LOG,
          "surrogate_loss": _lib.LOSS_CLIPPED,
          "kl_regulated": _lib.LOSS_KL_REGULATED}


def action_loss_grad(ctx, kind, choice, advantage, probs, distrib=None,
                     param=0.2):
    """The discrete-action loss gradients of a batch (xh_action_loss_grad):
    kind in LOSSES; probs [rows][range] (the model's output), distrib the
    actions' sampling distributions (all kinds but policy_loss)."""
    probs = np.ascontiguousarray(probs, np.float32)
    rows, rng = probs.shape
    ch = np.ascontiguousarray(choice, np.int32)
    adv = np.ascontiguousarray(advantage, np.float32)
    q = None if distrib is None else np.ascontiguousarray(distrib, np.float32)
    out = np.zeros_like(probs)
    check(_lib.lib.xh_action_loss_grad(ctx.h, LOSSES[kind], rows, rng, _ptr(ch),
                                       None if q is None else _ptr(q), _ptr(adv),
                                       _ptr(probs), param, _ptr(out)))
    return out


def optimizer_apply(ctx, kind, params, grad, lr, weight_decay=0.0, beta1=0.9,
                    beta2=0.999, t=1.0, m=None, v=None):
    """optimizer::next_parameters on the device (xh_optimizer_apply); returns
    (params, m, v), the state arrays updated in place as well."""
    p = np.ascontiguousarray(params, np.float32).copy()
    g = np.ascontiguousarray(grad, np.float32)
    m = np.zeros_like(p) if m is None else m
    v = np.zeros_like(p) if v is None else v
    check(_lib.lib.xh_optimizer_apply(ctx.h, _lib.OPTIMIZERS[kind], lr,
                                      weight_decay, beta1, beta2, t, _ptr(p),
                                      _ptr(g), _ptr(m), _ptr(v), p.size))
    return p, m, v


def policy_param_count(dims, h1, h2):
    f0 = 2 * dims
    return h1 * f0 + h1 + h2 * h1 + h2 + h2 + 1


def value_param_count(bins, dims, v1=64, v2=32):
    fin = bins * 2 * dims
    return v1 * fin + v1 + v2 * v1 + v2 + v2 + 1


def init_policy(dims, h1, h2, seed=0):
    """Reference initialisation scheme for conv1d_1 layers: weights
    N(0, sqrt(2/fan_in)) (he_initialize, nn.h:16-18,123), biases 0.  Drawn
    with numpy (distribution-equal, not stream-equal to the reference)."""
    rng = np.random.default_rng(seed)
    f0 = 2 * dims
    parts = []
    for fi, fo in ((f0, h1), (h1, h2), (h2, 1)):
        parts.append(rng.normal(0.0, np.sqrt(2.0 / fi), fo * fi))
        parts.append(np.zeros(fo))
    return np.concatenate(parts).astype(np.float32)


def init_full_policy(bins, dims, widths, seed=0):
    """REINFORCE's full-layer policy 4B -> widths... -> B, full_layer init
    N(0, 0.01) (nn.h:12-14,68), biases 0."""
    rng = np.random.default_rng(seed)
    sizes = [bins * 2 * dims] + [w for w in widths if w] + [bins]
    parts = []
    for fi, fo in zip(sizes[:-1], sizes[1:]):
        parts.append(rng.normal(0.0, 0.01, fo * fi))
        parts.append(np.zeros(fo))
    return np.concatenate(parts).astype(np.float32)


def init_value(bins, dims, v1=64, v2=32, seed=1):
    """full_layer init N(0, 0.01) (normal_initialize, nn.h:12-14,68)."""
    rng = np.random.default_rng(seed)
    fin = bins * 2 * dims
    parts = []
    for fi, fo in ((fin, v1), (v1, v2), (v2, 1)):
        parts.append(rng.normal(0.0, 0.01, fo * fi))
        parts.append(np.zeros(fo))
    return np.concatenate(parts).astype(np.float32)


class Trainer:
    """xh_trainer: N vectorised bin-packing envs + per-bin policy + value net +
    PPO (ppo_learner), KL-PPO (kl_ppo_learner) or actor-critic
    (actor_critic_learner) learner."""

    def __init__(self, ctx, algo="ppo", bins=64, dims=2, num_envs=4096, steps=4,
                 widths=(128, 128), value_widths=(64, 32), epochs=None,
                 lr_policy=None, lr_value=None, wd_policy=None, wd_value=None,
                 gamma=0.99, lam=0.95, clip_eps=0.2, rng_state=1,
                 num_envs_global=None, env_offset=0, adv_normalize=False,
                 lr_scale_rows=False, train_grid_cap=0, record_distrib=False,
                 record_last_step=False):
        cfg = _lib.Config()
        a = ALGOS[algo]
        _lib.lib.xh_config_default(C.byref(cfg), a, bins, dims, num_envs, steps)
        cfg.num_envs_global = num_envs_global or num_envs
        cfg.env_offset = env_offset
        cfg.policy_h1, cfg.policy_h2 = widths
        cfg.value_h1, cfg.value_h2 = value_widths
        if epochs is not None:
            cfg.epochs = epochs
        if lr_policy is not None:
            cfg.lr_policy = lr_policy
        if lr_value is not None:
            cfg.lr_value = lr_value
        if wd_policy is not None:
            cfg.wd_policy = wd_policy
        if wd_value is not None:
            cfg.wd_value = wd_value
        cfg.gamma, cfg.lambda_, cfg.clip_eps = gamma, lam, clip_eps
        cfg.rng_state = rng_state
        # opt-in, off in the reference configuration (xh_config)
        cfg.adv_normalize = int(bool(adv_normalize))
        cfg.lr_scale_rows = int(bool(lr_scale_rows))
        # test-only: cap on the train workgroups (accumulation depth tests)
        cfg.train_grid_cap = int(train_grid_cap)
        cfg.record_distrib = int(bool(record_distrib))
        # diagnostics: the last slot's logits / probabilities (BUF_LOGITS,
        # BUF_PROBS); off in the product path
        cfg.record_last_step = int(bool(record_last_step))
        self.cfg = cfg
        self.ctx = ctx
        self.B, self.D, self.N, self.T = bins, dims, num_envs, steps
        self.epochs = cfg.epochs
        self.h = C.c_void_p()
        check(_lib.lib.xh_trainer_create(ctx.h, C.byref(cfg), C.byref(self.h)))
        self.np_ = _lib.lib.xh_trainer_num_params(self.h, POLICY)
        self.nv = _lib.lib.xh_trainer_num_params(self.h, VALUE)
        if algo == "pg":  # steps = episodes per env; the batch has a step bound
            self.episodes = steps
            self.T = _lib.lib.xh_trainer_buffer_bytes(self.h, BUF_ACTION) // (
                4 * num_envs)

    # ------------------------------------------------------------ params --
    def num_params(self, which):
        return self.np_ if which == POLICY else self.nv

    def set_params(self, which, p):
        p = np.ascontiguousarray(p, np.float32)
        check(_lib.lib.xh_trainer_set_params(self.h, which, _ptr(p), p.size))

    def params(self, which):
        out = np.zeros(self.num_params(which), np.float32)
        check(_lib.lib.xh_trainer_get_params(self.h, which, _ptr(out), out.size))
        return out

    def set_optimizer(self, which, kind, lr, weight_decay=0.0, beta1=0.9,
                      beta2=0.999):
        """kind: "sgd" | "momentum" | "adam" (nn.h:616-698); fresh state."""
        check(_lib.lib.xh_trainer_set_optimizer(
            self.h, which, _lib.OPTIMIZERS[kind], lr, weight_decay, beta1,
            beta2))

    def set_learning_rate(self, which, lr):
        """optimizer::set_rate (nn.h:591); the optimizer state is kept."""
        check(_lib.lib.xh_trainer_set_learning_rate(self.h, which, lr))

    # -------------------------------------------------------------- loop --
    def set_record_last_step(self, on):
        """Record the last rollout step's logits / probabilities (BUF_LOGITS,
        BUF_PROBS) from the next rollout on (xh_trainer_set_record_last_step)."""
        check(_lib.lib.xh_trainer_set_record_last_step(self.h, int(bool(on))))
        self.cfg.record_last_step = int(bool(on))

    def rollout(self):
        check(_lib.lib.xh_trainer_rollout(self.h))

    def learn(self):
        check(_lib.lib.xh_trainer_learn(self.h))

    def iterate(self, n=1):
        check(_lib.lib.xh_trainer_iterate(self.h, n))

    def synchronize(self):
        self.ctx.synchronize()

    def forget(self):
        """replay_buffer::forget() without learn() (xh_trainer_forget)."""
        check(_lib.lib.xh_trainer_forget(self.h))

    def set_forced_actions(self, actions):
        if actions is None:
            check(_lib.lib.xh_trainer_set_forced_actions(self.h, None))
            return
        a = np.ascontiguousarray(actions, np.int32).reshape(self.T, self.N)
        check(_lib.lib.xh_trainer_set_forced_actions(self.h, _ptr(a)))

    # ----------------------------------------------------------- buffers --
    def _spec(self, which):
        T, N, B, D = self.T, self.N, self.B, self.D
        return {
            BUF_BINS: (np.int8, (T + 1, N, B, D)),
            BUF_ITEMS: (np.int8, (T + 1, N, 4)),
            BUF_ACTION: (np.int32, (T, N)),
            BUF_POLD: (np.float32, (T, N)),
            BUF_DONE: (np.uint8, (T, N)),
            BUF_RNG: (np.uint32, (N,)),
            BUF_V_STATE: (np.float32, (T + 1, N)),
            BUF_V_STATE0: (np.float32, (T + 1, N)),
            BUF_V_TERM: (np.float32, (T, N)),
            BUF_TARGETS: (np.float32, (T, N)),
            BUF_ADV: (np.float32, (T, N)),
            BUF_VALUE_GRAD: (np.float32, (self.nv,)),
            BUF_POLICY_GRADS: (np.float32, (self.epochs, self.np_)),
            BUF_LOGITS: (np.float32, (N, B)),
            BUF_PROBS: (np.float32, (N, B)),
            BUF_QOLD: (np.float32, (T, N, B)),
            BUF_KL: (np.float32, (self.epochs, 3)),
            BUF_LEN: (np.int32, (N,)),
        }[which]

    def buffer(self, which):
        dt, shape = self._spec(which)
        out = np.zeros(shape, dt)
        check(_lib.lib.xh_trainer_get_buffer(self.h, which, _ptr(out), out.nbytes))
        return out

    def set_buffer(self, which, arr):
        dt, shape = self._spec(which)
        a = np.ascontiguousarray(arr, dt).reshape(shape)
        check(_lib.lib.xh_trainer_set_buffer(self.h, which, _ptr(a), a.nbytes))

    def env_state(self, first=0, count=None):
        """(bins [count][B][D], items [count][D]) int8: the states the next
        rollout starts from (xh_trainer_get_env_state)."""
        count = self.N - first if count is None else count
        bins = np.zeros((count, self.B, self.D), np.int8)
        items = np.zeros((count, self.D), np.int8)
        check(_lib.lib.xh_trainer_get_env_state(self.h, first, count,
                                                _ptr(bins), _ptr(items)))
        return bins, items

    def set_env_state(self, first, bins, items):
        """Replace envs [first, first + len) for the next rollout
        (xh_trainer_set_env_state)."""
        bins = np.ascontiguousarray(bins, np.int8)
        items = np.ascontiguousarray(items, np.int8)
        count = bins.shape[0]
        assert bins.shape == (count, self.B, self.D)
        assert items.shape == (count, self.D)
        check(_lib.lib.xh_trainer_set_env_state(self.h, first, count,
                                                _ptr(bins), _ptr(items)))

    def health(self):
        """Numerical health of the training state (host copies, call outside
        any timed region): finite parameters and last-step probabilities
        (when a rollout recorded them: record_last_step), and the last
        batch's done rate / mean episode length (every episode ends on
        exactly one done step)."""
        pp, pv = self.params(POLICY), self.params(VALUE)
        out = {"finite": bool(np.isfinite(pp).all() and np.isfinite(pv).all())}
        if self.cfg.algo != XH_PG:
            done = self.buffer(BUF_DONE)
            try:
                probs = self.buffer(BUF_PROBS)
            except _lib.XhError:
                probs = None  # no rollout recorded its last step
            if probs is not None:
                out["finite"] = out["finite"] and bool(np.isfinite(probs).all())
                out["max_prob"] = float(probs.max())
            rate = float(done.mean())
            out["done_rate"] = rate
            out["mean_episode_len"] = (1.0 / rate) if rate > 0 else None
        return out

    def evaluate(self, n_envs, episodes, rng_state, argmax_probs=False,
                 init_items=None, trace_cap=0):
        """Argmax evaluation (deep_agent.cc / the drivers' periodic eval).
        Returns a dict: totals, steps, final_items, rng (per env), env 0's
        first trace_cap actions (trace_cap > 0), elapsed_ms."""
        e, out, keep = _eval_struct(n_envs, episodes, rng_state, self.D,
                                    init_items, trace_cap, argmax_probs)
        check(_lib.lib.xh_trainer_evaluate(self.h, C.byref(e)))
        del keep
        return _eval_result(e, out, trace_cap)

    def seed_streams(self, x):
        """Re-base the env streams on global engine state x (reference order:
        env g steps from x advanced 4*T*g draws)."""
        check(_lib.lib.xh_trainer_seed_streams(self.h, x))

    # ------------------------------------------------------------ timing --
    def set_timing(self, on):
        """on: False / True (every launch) / "train" (the policy train
        launches only: XH_TIMING_TRAIN)."""
        mode = 2 if on == "train" else (1 if on else 0)
        check(_lib.lib.xh_trainer_set_timing(self.h, mode))

    def reset_timing(self):
        check(_lib.lib.xh_trainer_reset_timing(self.h))

    def kernel_time(self, name):
        ms, n = C.c_double(), C.c_long()
        check(_lib.lib.xh_trainer_kernel_time(self.h, name.encode(), C.byref(ms),
                                              C.byref(n)))
        return ms.value, n.value

    def kernel_info(self):
        """The kernels the last rollout step / policy epoch launched and their
        arithmetic (xh_trainer_kernel_info): {"rollout_step": {...},
        "policy_train": {...}, "overrides": {...}}."""
        import json
        buf = C.create_string_buffer(2048)
        check(_lib.lib.xh_trainer_kernel_info(self.h, buf, len(buf)))
        return json.loads(buf.value.decode())

    def close(self):
        if self.h:
            check(_lib.lib.xh_trainer_destroy(self.h))
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
