"""ctypes binding of the C ABI in include/xylo_hip.h (libxylo_hip.so).

The library is the product: there is no CPU fallback.  If the in-tree
``libxylo_hip.so`` is missing, importing this module raises immediately.
"""
import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# XH_LIB_PATH: diagnostic builds only (`make diag`, tools/ablate.sh)
LIB_PATH = os.environ.get("XH_LIB_PATH") or os.path.join(HERE, "libxylo_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "xylo_hip.h")

XH_OK, XH_ERR_INVALID, XH_ERR_HIP, XH_ERR_RCCL, XH_ERR_STATE = range(5)
XH_PPO, XH_AC, XH_KLPPO, XH_PG = 0, 1, 2, 3
HEURISTICS = {"random": 0, "firstfit": 1, "bestfit": 2, "minwaste": 3}
XH_POLICY, XH_VALUE = 0, 1
OPTIMIZERS = {"sgd": 0, "momentum": 1, "adam": 2}
(VENV_ACTIONS, VENV_REWARD, VENV_DONE, VENV_BINS, VENV_ITEMS, VENV_RNG,
 VENV_OBS, VENV_MASK) = range(8)
(BUF_BINS, BUF_ITEMS, BUF_ACTION, BUF_POLD, BUF_DONE, BUF_RNG, BUF_V_STATE,
 BUF_V_TERM, BUF_TARGETS, BUF_ADV, BUF_VALUE_GRAD, BUF_POLICY_GRADS,
 BUF_LOGITS, BUF_PROBS, BUF_V_STATE0, BUF_QOLD, BUF_KL, BUF_LEN) = range(18)


class XhError(RuntimeError):
    """A non-zero status from the C ABI (message from xh_last_error())."""


class Config(C.Structure):
    """Mirror of xh_config."""
    _fields_ = [
        ("algo", C.c_int), ("num_envs", C.c_int), ("num_envs_global", C.c_int),
        ("env_offset", C.c_int), ("bins", C.c_int), ("dims", C.c_int),
        ("steps", C.c_int), ("epochs", C.c_int), ("policy_h1", C.c_int),
        ("policy_h2", C.c_int), ("value_h1", C.c_int), ("value_h2", C.c_int),
        ("lr_policy", C.c_float), ("lr_value", C.c_float),
        ("wd_policy", C.c_float), ("wd_value", C.c_float), ("gamma", C.c_float),
        ("lambda_", C.c_float), ("clip_eps", C.c_float),
        ("rng_state", C.c_uint32), ("kl_beta", C.c_float),
        ("kl_target", C.c_float), ("adv_normalize", C.c_int),
        ("lr_scale_rows", C.c_int), ("train_grid_cap", C.c_int),
        ("record_distrib", C.c_int), ("record_last_step", C.c_int)]


class Eval(C.Structure):
    """Mirror of xh_eval."""
    _fields_ = [
        ("n_envs", C.c_int), ("episodes", C.c_int), ("argmax_probs", C.c_int),
        ("rng_state", C.c_uint32), ("init_items", C.c_void_p),
        ("final_items", C.c_void_p), ("rng_out", C.c_void_p),
        ("totals", C.c_void_p), ("steps", C.c_void_p), ("trace", C.c_void_p),
        ("trace_cap", C.c_long), ("elapsed_ms", C.c_double)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libxylo_hip.so not built (%s); run `make lib` or "
            "__graft_entry__.build() -- there is no CPU fallback" % LIB_PATH)
    lib = C.CDLL(LIB_PATH)
    vp, i, sz = C.c_void_p, C.c_int, C.c_size_t
    sig = {
        "xh_last_error": (C.c_char_p, []),
        "xh_version": (C.c_char_p, []),
        "xh_struct_size": (sz, [C.c_char_p]),
        "xh_device_count": (i, [C.POINTER(C.c_int)]),
        "xh_runtime_info": (i, [C.c_char_p, sz]),
        "xh_comm_unique_id": (i, [vp]),
        "xh_ctx_create": (i, [i, i, i, vp, C.POINTER(vp)]),
        "xh_ctx_destroy": (i, [vp]),
        "xh_ctx_synchronize": (i, [vp]),
        "xh_ctx_allreduce_host": (i, [vp, vp, sz]),
        "xh_config_default": (None, [C.POINTER(Config), i, i, i, i, i]),
        "xh_trainer_create": (i, [vp, C.POINTER(Config), C.POINTER(vp)]),
        "xh_trainer_destroy": (i, [vp]),
        "xh_trainer_num_params": (sz, [vp, i]),
        "xh_trainer_set_params": (i, [vp, i, vp, sz]),
        "xh_trainer_get_params": (i, [vp, i, vp, sz]),
        "xh_trainer_set_optimizer": (i, [vp, i, i, C.c_float, C.c_float,
                                         C.c_float, C.c_float]),
        "xh_trainer_set_learning_rate": (i, [vp, i, C.c_float]),
        "xh_trainer_rollout": (i, [vp]),
        "xh_trainer_learn": (i, [vp]),
        "xh_trainer_iterate": (i, [vp, i]),
        "xh_trainer_set_forced_actions": (i, [vp, vp]),
        "xh_trainer_buffer_bytes": (sz, [vp, i]),
        "xh_trainer_get_buffer": (i, [vp, i, vp, sz]),
        "xh_trainer_set_buffer": (i, [vp, i, vp, sz]),
        "xh_trainer_evaluate": (i, [vp, C.POINTER(Eval)]),
        "xh_trainer_seed_streams": (i, [vp, C.c_uint32]),
        "xh_heuristic_evaluate": (i, [vp, i, i, i, C.POINTER(Eval)]),
        "xh_trainer_set_timing": (i, [vp, i]),
        "xh_trainer_kernel_time": (i, [vp, C.c_char_p, C.POINTER(C.c_double),
                                       C.POINTER(C.c_long)]),
        "xh_trainer_reset_timing": (i, [vp]),
        "xh_trainer_kernel_info": (i, [vp, C.c_char_p, sz]),
        "xh_ctx_inject_fault": (i, [vp, i]),
        "xh_trainer_get_env_state": (i, [vp, i, i, vp, vp]),
        "xh_trainer_set_env_state": (i, [vp, i, i, vp, vp]),
        "xh_venv_create": (i, [vp, i, i, i, C.c_uint32, i, i, i,
                               C.POINTER(vp)]),
        "xh_venv_destroy": (i, [vp]),
        "xh_venv_bytes": (sz, [vp, i]),
        "xh_venv_device_ptr": (vp, [vp, i]),
        "xh_venv_get": (i, [vp, i, vp, sz]),
        "xh_venv_set": (i, [vp, i, vp, sz]),
        "xh_venv_step": (i, [vp, i]),
        "xh_venv_apply": (i, [vp, i]),
        "xh_venv_reset": (i, [vp, i]),
        "xh_venv_observe": (i, [vp]),
        "xh_venv_synchronize": (i, [vp]),
        "xh_venv_set_timing": (i, [vp, i]),
        "xh_venv_kernel_time": (i, [vp, C.POINTER(C.c_double),
                                    C.POINTER(C.c_long)]),
        "xh_model_eval": (i, [vp, vp, i, vp, sz, vp, i, i, vp, sz,
                              C.POINTER(C.c_int)]),
        "xh_model_forward": (i, [vp, vp, i, vp, sz, vp, i, i, vp, sz,
                                 C.POINTER(C.c_int)]),
        "xh_model_gradient": (i, [vp, vp, i, vp, sz, vp, i, i, vp, i, vp]),
        "xh_layer_backward": (i, [vp, vp, vp, sz, vp, i, i, vp, i, vp]),
        "xh_layer_gradient": (i, [vp, vp, vp, i, i, vp, i, vp, sz]),
        "xh_action_loss_grad": (i, [vp, i, i, i, vp, vp, vp, vp, C.c_float,
                                    vp]),
        "xh_optimizer_apply": (i, [vp, i, C.c_float, C.c_float, C.c_float,
                                   C.c_float, C.c_float, vp, vp, vp, vp, sz]),
        "xh_trainer_forget": (i, [vp]),
        "xh_trainer_set_record_last_step": (i, [vp, i]),
        "xh_tensor_reduce": (i, [vp, i, vp, vp, C.c_float, sz, i,
                                 C.POINTER(C.c_double),
                                 C.POINTER(C.c_int64)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


class Layer(C.Structure):
    """Mirror of xh_layer."""
    _fields_ = [("kind", C.c_int), ("inp", C.c_int), ("out", C.c_int)]


LAYER_FULL, LAYER_CONV1D_1, LAYER_RELU, LAYER_SOFTMAX, LAYER_SOFTMAX_XENT = range(5)
(LOSS_GRADIENT_LOG, LOSS_SOFTMAX_GRADIENT_LOG, LOSS_CLIPPED,
 LOSS_KL_REGULATED) = range(4)

lib = _load()
for _name, _mirror in (("xh_config", Config), ("xh_eval", Eval),
                       ("xh_layer", Layer)):
    if lib.xh_struct_size(_name.encode()) != C.sizeof(_mirror):
        raise ImportError("ctypes mirror of %s is out of date (%d vs %d bytes)"
                          % (_name, C.sizeof(_mirror),
                             lib.xh_struct_size(_name.encode())))


def check(status):
    if status != XH_OK:
        raise XhError("xylo-hip status %d: %s" % (
            status, lib.xh_last_error().decode(errors="replace")))
    return status


def runtime_info():
    """The HIP / RCCL shared objects this process bound (xh_runtime_info)."""
    import json
    buf = C.create_string_buffer(4096)
    check(lib.xh_runtime_info(buf, len(buf)))
    return json.loads(buf.value.decode())


def device_count():
    n = C.c_int()
    check(lib.xh_device_count(C.byref(n)))
    return n.value


def header_symbols():
    """Function names declared by include/xylo_hip.h (for the ABI test)."""
    with open(HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(xh_[a-z0-9_]+)\s*\(", text)))
