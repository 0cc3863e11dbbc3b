"""dependence_free_rl_amd -- MI355X-native PPO / actor-critic rollout-and-update
path for vectorised bin packing (drop-in for beehover/dependence_free_rl's
xylo::rl / xylo::policy_gradient hot path).  See DESIGN.md."""
from ._lib import (XhError, device_count, lib,  # noqa: F401  (fails loudly
                   runtime_info)                 # if not built)
from .trainer import (ALGOS, POLICY, VALUE, Context, Trainer,  # noqa: F401
                      heuristic_evaluate, init_full_policy, init_policy,
                      init_value,
                      policy_param_count, value_param_count)
from .venv import VecEnv  # noqa: F401

__all__ = ["Context", "Trainer", "POLICY", "VALUE", "init_policy", "init_value",
           "init_full_policy",
           "heuristic_evaluate", "XhError", "runtime_info", "device_count", "VecEnv"]
