"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker / baseline, never as the thing measured or shipped.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

OR_FULL, OR_POINT, OR_RELU, OR_SOFTMAX, OR_SOFTMAX_XENT = range(5)
OR_PPO, OR_AC, OR_PG, OR_KLPPO = range(4)
OPT_SGD, OPT_MOMENTUM, OPT_ADAM = range(3)
(BUF_STEP_BINS, BUF_STEP_ITEM, BUF_STEP_CHOICE, BUF_STEP_DONE, BUF_STEP_PCHOICE,
 BUF_ROWS, BUF_ROW_ENV, BUF_ROW_STEP, BUF_ROW_IS_END, BUF_VALUES, BUF_TARGETS,
 BUF_VALUE_GRAD, BUF_ADVANTAGES, BUF_POLICY_GRADS, BUF_FINAL_BINS,
 BUF_FINAL_ITEM, BUF_ROW_CHOICE, BUF_ROW_POLD, BUF_KL, BUF_POLICY_GRADS_MAG,
 BUF_VALUE_GRAD_MAG) = range(21)
_INT_BUFS = {BUF_STEP_BINS, BUF_STEP_ITEM, BUF_STEP_CHOICE, BUF_STEP_DONE,
             BUF_ROW_ENV, BUF_ROW_STEP, BUF_ROW_IS_END, BUF_FINAL_BINS,
             BUF_FINAL_ITEM, BUF_ROW_CHOICE}


class EnvCfg(C.Structure):
    _fields_ = [("B", C.c_int), ("D", C.c_int), ("cap", C.c_int),
                ("item_a", C.c_int * 3), ("item_b", C.c_int * 3),
                ("p_a", C.c_double)]


class Model(C.Structure):
    _fields_ = [("nl", C.c_int), ("type", C.c_int * 16), ("inp", C.c_int * 16),
                ("out", C.c_int * 16)]


def build():
    """Compile liboracle.so (gcc, no GPU)."""
    subprocess.run(["make", "-s", "-C", HERE, "port"], check=True)


def lib():
    if not hasattr(lib, "_l"):
        if not os.path.exists(LIB):
            build()
        l = C.CDLL(LIB)
        u32p = C.POINTER(C.c_uint32)
        l.or_minstd_seed.restype = C.c_uint32
        l.or_minstd_seed.argtypes = [C.c_uint64]
        l.or_minstd_next.restype = C.c_uint32
        l.or_minstd_next.argtypes = [u32p]
        l.or_minstd_jump.restype = C.c_uint32
        l.or_minstd_jump.argtypes = [C.c_uint32, C.c_uint64]
        l.or_canonical.restype = C.c_double
        l.or_canonical.argtypes = [u32p]
        l.or_bernoulli.argtypes = [u32p, C.c_double]
        l.or_discrete.argtypes = [u32p, C.c_void_p, C.c_int]
        l.or_env_default.argtypes = [C.POINTER(EnvCfg), C.c_int, C.c_int]
        for f in ("or_env_construct", "or_env_reset"):
            getattr(l, f).argtypes = [C.POINTER(EnvCfg), C.c_void_p, C.c_void_p, u32p]
        l.or_env_apply.argtypes = [C.POINTER(EnvCfg), C.c_void_p, C.c_void_p,
                                   C.c_int, u32p]
        l.or_obs.argtypes = [C.POINTER(EnvCfg), C.c_void_p, C.c_void_p, C.c_void_p]
        l.or_model_nparams.restype = C.c_size_t
        l.or_model_nparams.argtypes = [C.POINTER(Model)]
        l.or_model_eval.argtypes = [C.POINTER(Model), C.c_void_p, C.c_void_p,
                                    C.c_int, C.c_int, C.c_void_p]
        l.or_trainer_create.restype = C.c_void_p
        l.or_trainer_create.argtypes = [
            C.c_int, C.POINTER(EnvCfg), C.c_int, C.c_int, C.c_int,
            C.POINTER(Model), C.c_void_p, C.POINTER(Model), C.c_void_p,
            C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, C.c_uint32]
        l.or_trainer_destroy.argtypes = [C.c_void_p]
        l.or_trainer_rollout.argtypes = [C.c_void_p, C.c_void_p]
        l.or_trainer_learn.argtypes = [C.c_void_p]
        l.or_trainer_rng.restype = C.c_uint32
        l.or_trainer_rng.argtypes = [C.c_void_p]
        l.or_trainer_get_params.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        l.or_trainer_set_params.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        l.or_trainer_buf.restype = C.c_void_p
        l.or_trainer_buf.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_size_t)]
        l.or_policy_grad_rows.argtypes = [C.POINTER(Model), C.c_void_p, C.c_void_p,
                                          C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_int, C.c_void_p]
        l.or_value_grad_rows.argtypes = [C.POINTER(Model), C.c_void_p, C.c_void_p,
                                         C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        l.or_policy_grad_rows_mag.argtypes = [C.POINTER(Model), C.c_void_p,
                                              C.c_void_p, C.c_int, C.c_int,
                                              C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.c_int, C.c_void_p, C.c_void_p]
        l.or_value_grad_rows_mag.argtypes = [C.POINTER(Model), C.c_void_p,
                                             C.c_void_p, C.c_int, C.c_int,
                                             C.c_void_p, C.c_void_p, C.c_void_p]
        l.or_eval_argmax.restype = C.c_double
        l.or_eval_argmax.argtypes = [C.POINTER(EnvCfg), C.POINTER(Model),
                                     C.c_void_p, C.c_long, u32p]
        l.or_trainer_set_options.argtypes = [C.c_void_p, C.c_int, C.c_int]
        l.or_venv_run.restype = C.c_uint32
        l.or_venv_run.argtypes = [C.POINTER(EnvCfg), C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.c_uint32, C.c_int, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_void_p]
        lib._l = l
    return lib._l


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def env_cfg(B, D):
    c = EnvCfg()
    lib().or_env_default(C.byref(c), B, D)
    return c


def perbin_model(f0, widths, head):
    """conv1d_1 chain f0 -> widths... -> 1 (+ head), relu between."""
    layers = []
    prev = f0
    for w in widths:
        layers += [(OR_POINT, prev, w), (OR_RELU, 0, 0)]
        prev = w
    layers.append((OR_POINT, prev, 1))
    if head is not None:
        layers.append((head, 0, 0))
    return _model(layers)


def full_model(inp, widths, out, head=None):
    layers = []
    prev = inp
    for w in widths:
        layers += [(OR_FULL, prev, w), (OR_RELU, 0, 0)]
        prev = w
    layers.append((OR_FULL, prev, out))
    if head is not None:
        layers.append((head, 0, 0))
    return _model(layers)


def _model(layers):
    m = Model()
    m.nl = len(layers)
    for i, (t, a, b) in enumerate(layers):
        m.type[i], m.inp[i], m.out[i] = t, a, b
    return m


def nparams(m):
    return lib().or_model_nparams(C.byref(m))


def model_eval(m, params, x):
    x = np.ascontiguousarray(x, np.float32)
    params = np.ascontiguousarray(params, np.float32)
    rows, cols = x.shape
    out = np.zeros(rows * max(cols, 4096), np.float32)
    oc = lib().or_model_eval(C.byref(m), _ptr(params), _ptr(x), rows, cols,
                             _ptr(out))
    return out[:rows * oc].reshape(rows, oc).copy()


class Rng:
    """std::minstd_rand0 + libstdc++ distributions."""

    def __init__(self, state):
        self.x = C.c_uint32(state)

    @staticmethod
    def seeded(seed):
        return Rng(lib().or_minstd_seed(seed))

    def next(self):
        return lib().or_minstd_next(C.byref(self.x))

    def canonical(self):
        return lib().or_canonical(C.byref(self.x))

    def bernoulli(self, p=0.4):
        return lib().or_bernoulli(C.byref(self.x), p)

    def discrete(self, p):
        p = np.ascontiguousarray(p, np.float32)
        return lib().or_discrete(C.byref(self.x), _ptr(p), len(p))

    @property
    def state(self):
        return self.x.value


def minstd_jump(x, k):
    return lib().or_minstd_jump(x, k)


class Env:
    """One env (bins int32 [B][D], item int32 [D]) with a shared Rng."""

    def __init__(self, cfg, rng):
        self.cfg, self.rng = cfg, rng
        self.bins = np.zeros((cfg.B, cfg.D), np.int32)
        self.item = np.zeros(3, np.int32)
        lib().or_env_construct(C.byref(cfg), _ptr(self.bins), _ptr(self.item),
                               C.byref(rng.x))

    def apply(self, choice):
        return lib().or_env_apply(C.byref(self.cfg), _ptr(self.bins),
                                  _ptr(self.item), int(choice), C.byref(self.rng.x))

    def reset(self):
        lib().or_env_reset(C.byref(self.cfg), _ptr(self.bins), _ptr(self.item),
                           C.byref(self.rng.x))

    def obs(self):
        out = np.zeros(self.cfg.B * 2 * self.cfg.D, np.float32)
        lib().or_obs(C.byref(self.cfg), _ptr(self.bins), _ptr(self.item), _ptr(out))
        return out


def venv_run(B, D, N, x0, actions, policy_draws=2, n_global=None, offset=0):
    """or_venv_run: Ng agents stepped once per step in env order on one
    engine seeded at state x0; actions [S][N] for envs [offset, offset + N).
    Returns dict bins [S+1][N][B][D], item [S+1][N][D], reward / done [S][N],
    x_end."""
    actions = np.ascontiguousarray(actions, np.int32)
    S = actions.shape[0]
    cfg = env_cfg(B, D)
    out = {"bins": np.zeros((S + 1, N, B, D), np.int32),
           "item": np.zeros((S + 1, N, D), np.int32),
           "reward": np.zeros((S, N), np.float32),
           "done": np.zeros((S, N), np.uint8)}
    out["x_end"] = lib().or_venv_run(
        C.byref(cfg), N, n_global or N, offset, policy_draws, x0, S,
        _ptr(actions), _ptr(out["bins"]), _ptr(out["item"]),
        _ptr(out["reward"]), _ptr(out["done"]))
    return out


class Trainer:
    """Sequential reference-order trainer (PPO / AC / PG) on the oracle."""

    def __init__(self, algo, B, D, N, T, pol_model, pol_params, val_model=None,
                 val_params=None, lr_pi=1e-4, lr_v=1e-5, wd_pi=0.0, wd_v=0.0,
                 gamma=0.99, x0=1, episodes=1):
        self.cfg = env_cfg(B, D)
        self.B, self.D, self.N, self.T = B, D, N, T
        self.pm, self.vm = pol_model, val_model
        pp = np.ascontiguousarray(pol_params, np.float32)
        vp = (np.ascontiguousarray(val_params, np.float32)
              if val_params is not None else np.zeros(1, np.float32))
        self.np_, self.nv = nparams(pol_model), (nparams(val_model) if val_model else 0)
        assert pp.size == self.np_, (pp.size, self.np_)
        self.h = lib().or_trainer_create(
            algo, C.byref(self.cfg), N, T, episodes, C.byref(pol_model), _ptr(pp),
            C.byref(val_model) if val_model else None, _ptr(vp), lr_pi, lr_v,
            wd_pi, wd_v, gamma, x0)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_trainer_destroy(self.h)
            self.h = None

    def set_optimizer(self, which, kind, lr, wd=0.0, beta1=0.9, beta2=0.999):
        """kind: OPT_SGD / OPT_MOMENTUM / OPT_ADAM (nn.h:616-698)."""
        l = lib()
        l.or_trainer_set_optimizer.argtypes = [C.c_void_p, C.c_int, C.c_int,
                                               C.c_float, C.c_float, C.c_float,
                                               C.c_float]
        l.or_trainer_set_optimizer(self.h, which, kind, lr, wd, beta1, beta2)

    def set_options(self, adv_normalize=False, lr_scale_rows=False):
        lib().or_trainer_set_options(self.h, int(adv_normalize),
                                     int(lr_scale_rows))

    def set_env_streams(self, stride=1 << 26, reconstruct=True):
        """Env i on its own stream: x0 advanced by i * stride (reconstructing
        the envs), or the current engine advanced by i * stride (keeping
        them)."""
        l = lib()
        l.or_trainer_set_env_streams.argtypes = [C.c_void_p, C.c_uint64, C.c_int]
        l.or_trainer_set_env_streams(self.h, stride, 1 if reconstruct else 0)

    def set_stream_states(self, xs):
        """Env i draws from stream state xs[i] from the next rollout on (the
        envs are kept): a sample of a larger reference-order job."""
        xs = np.ascontiguousarray(xs, np.uint32)
        assert xs.size == self.N
        l = lib()
        l.or_trainer_set_stream_states.argtypes = [C.c_void_p, C.c_void_p]
        l.or_trainer_set_stream_states(self.h, _ptr(xs))

    def env_streams(self):
        l = lib()
        l.or_trainer_env_streams.restype = C.POINTER(C.c_uint32)
        l.or_trainer_env_streams.argtypes = [C.c_void_p]
        p = l.or_trainer_env_streams(self.h)
        return np.array([p[i] for i in range(self.N)], np.uint32)

    def rollout(self, forced=None):
        if forced is not None:
            forced = np.ascontiguousarray(forced, np.int32)
            lib().or_trainer_rollout(self.h, _ptr(forced))
        else:
            lib().or_trainer_rollout(self.h, None)

    def learn(self):
        lib().or_trainer_learn(self.h)

    @property
    def rng(self):
        return lib().or_trainer_rng(self.h)

    def params(self, which=0):
        out = np.zeros(self.np_ if which == 0 else self.nv, np.float32)
        lib().or_trainer_get_params(self.h, which, _ptr(out))
        return out

    def set_params(self, which, p):
        p = np.ascontiguousarray(p, np.float32)
        lib().or_trainer_set_params(self.h, which, _ptr(p))

    def buf(self, which):
        n = C.c_size_t()
        p = lib().or_trainer_buf(self.h, which, C.byref(n))
        dt = np.int32 if which in _INT_BUFS else np.float32
        if not p or n.value == 0:
            return np.zeros(0, dt)
        arr = (C.c_int32 if dt == np.int32 else C.c_float) * n.value
        return np.frombuffer(arr.from_address(p), dt).copy()


class Opt(C.Structure):
    """or_opt: an optimizer with its state (nn.h:616-698)."""
    _fields_ = [("kind", C.c_int), ("lr", C.c_float), ("wd", C.c_float),
                ("b1", C.c_float), ("b2", C.c_float), ("t", C.c_float),
                ("m", C.c_void_p), ("v", C.c_void_p)]

    def __init__(self, kind, lr, wd=0.0, beta1=0.9, beta2=0.999):
        super().__init__(kind, lr, wd, beta1, beta2, 1.0, None, None)

    def step(self, params, grad):
        """In place on the float32 array `params`."""
        grad = np.ascontiguousarray(grad, np.float32)
        l = lib()
        l.or_opt_step.argtypes = [C.POINTER(Opt), C.c_void_p, C.c_void_p,
                                  C.c_size_t]
        l.or_opt_step(C.byref(self), _ptr(params), _ptr(grad), params.size)

    def __del__(self):
        l = lib()
        l.or_opt_free.argtypes = [C.POINTER(Opt)]
        l.or_opt_free(C.byref(self))


def policy_grad_rows(model, params, x, choice, pold, adv, algo):
    x = np.ascontiguousarray(x, np.float32)
    params = np.ascontiguousarray(params, np.float32)
    ch = np.ascontiguousarray(choice, np.int32)
    pold = np.ascontiguousarray(pold, np.float32)
    adv = np.ascontiguousarray(adv, np.float32)
    g = np.zeros(nparams(model), np.float32)
    lib().or_policy_grad_rows(C.byref(model), _ptr(params), _ptr(x), x.shape[0],
                              x.shape[1], _ptr(ch), _ptr(pold), _ptr(adv), algo,
                              _ptr(g))
    return g


def value_grad_rows(model, params, x, targets):
    x = np.ascontiguousarray(x, np.float32)
    params = np.ascontiguousarray(params, np.float32)
    tg = np.ascontiguousarray(targets, np.float32)
    g = np.zeros(nparams(model), np.float32)
    lib().or_value_grad_rows(C.byref(model), _ptr(params), _ptr(x), x.shape[0],
                             x.shape[1], _ptr(tg), _ptr(g))
    return g


def policy_grad_rows_mag(model, params, x, choice, pold, adv, algo):
    """(gradient, per-entry sum of |terms|) of the policy loss over rows."""
    x = np.ascontiguousarray(x, np.float32)
    params = np.ascontiguousarray(params, np.float32)
    ch = np.ascontiguousarray(choice, np.int32)
    pold = np.ascontiguousarray(pold, np.float32)
    adv = np.ascontiguousarray(adv, np.float32)
    g = np.zeros(nparams(model), np.float32)
    mag = np.zeros(nparams(model), np.float32)
    lib().or_policy_grad_rows_mag(C.byref(model), _ptr(params), _ptr(x),
                                  x.shape[0], x.shape[1], _ptr(ch), _ptr(pold),
                                  _ptr(adv), algo, _ptr(g), _ptr(mag))
    return g, mag


def value_grad_rows_mag(model, params, x, targets):
    """(gradient, per-entry sum of |terms|) of the square loss over rows."""
    x = np.ascontiguousarray(x, np.float32)
    params = np.ascontiguousarray(params, np.float32)
    tg = np.ascontiguousarray(targets, np.float32)
    g = np.zeros(nparams(model), np.float32)
    mag = np.zeros(nparams(model), np.float32)
    lib().or_value_grad_rows_mag(C.byref(model), _ptr(params), _ptr(x),
                                 x.shape[0], x.shape[1], _ptr(tg), _ptr(g),
                                 _ptr(mag))
    return g, mag


OR_HEUR = {"random": 0, "firstfit": 1, "bestfit": 2, "minwaste": 3}


def heuristic_eval(B, D, kind, episodes, x0):
    """The reference's heuristic agents on one env seeded at x0: (total
    reward, per-episode lengths, engine state after)."""
    cfg = env_cfg(B, D)
    x = C.c_uint32(x0)
    lens = np.zeros(max(episodes, 1), np.int32)
    l = lib()
    l.or_heuristic_eval.restype = C.c_double
    l.or_heuristic_eval.argtypes = [C.c_void_p, C.c_int, C.c_long,
                                    C.POINTER(C.c_uint32), C.c_void_p]
    total = l.or_heuristic_eval(C.byref(cfg), OR_HEUR[kind], episodes,
                                C.byref(x), _ptr(lens))
    return total, lens[:episodes], x.value


def eval_argmax(B, D, model, params, episodes, x0):
    cfg = env_cfg(B, D)
    x = C.c_uint32(x0)
    params = np.ascontiguousarray(params, np.float32)
    total = lib().or_eval_argmax(C.byref(cfg), C.byref(model), _ptr(params),
                                 episodes, C.byref(x))
    return total, x.value
