"""Vectorised bin-packing environments for a caller's own policy (xh_venv_*).

    env = VecEnv(ctx, num_envs=32768, bins=64, dims=2, rng_state=7,
                 policy_draws=2)
    obs = env.observe()                 # [N][B][2D] float32
    env.set_actions(actions)            # int32 [N]
    reward, done = env.step()           # agent::step minus react, all envs

Mirrors xylo::environment<A,S>::apply / view / reset (rl.h:163-170) with the
id ranging over the batch, bp::environment (bin_packing.h:46-85) and
xylo::agent::step (rl.h:325-349).  State lives in HBM; numpy arrays here are
host copies.  `device_ptr(which)` exposes the device buffers for a policy
kernel of the caller's own on the same device.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import (VENV_ACTIONS, VENV_BINS, VENV_DONE, VENV_ITEMS, VENV_MASK,
                   VENV_OBS, VENV_REWARD, VENV_RNG, check)


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class VecEnv:
    """xh_venv: N envs of B bins x D dims stepped by one kernel per call."""

    def __init__(self, ctx, num_envs, bins=64, dims=2, rng_state=1,
                 env_offset=0, num_envs_global=None, policy_draws=2):
        self.ctx = ctx
        self.N, self.B, self.D = num_envs, bins, dims
        self.h = C.c_void_p()
        check(_lib.lib.xh_venv_create(ctx.h, num_envs, bins, dims, rng_state,
                                      env_offset, num_envs_global or num_envs,
                                      policy_draws, C.byref(self.h)))

    def _spec(self, which):
        N, B, D = self.N, self.B, self.D
        return {VENV_ACTIONS: (np.int32, (N,)), VENV_REWARD: (np.float32, (N,)),
                VENV_DONE: (np.uint8, (N,)), VENV_BINS: (np.int8, (N, B, D)),
                VENV_ITEMS: (np.int8, (N, 4)), VENV_RNG: (np.uint32, (N,)),
                VENV_OBS: (np.float32, (N, B, 2 * D)),
                VENV_MASK: (np.uint8, (N,))}[which]

    def get(self, which):
        dt, shape = self._spec(which)
        out = np.zeros(shape, dt)
        check(_lib.lib.xh_venv_get(self.h, which, _ptr(out), out.nbytes))
        return out

    def set(self, which, arr):
        dt, shape = self._spec(which)
        a = np.ascontiguousarray(arr, dt).reshape(shape)
        check(_lib.lib.xh_venv_set(self.h, which, _ptr(a), a.nbytes))

    def device_ptr(self, which):
        return _lib.lib.xh_venv_device_ptr(self.h, which)

    # ---- environment<A,S> / agent<A,S> ---------------------------------
    def set_actions(self, actions):
        self.set(VENV_ACTIONS, actions)

    def step(self, write_obs=False, fetch=True):
        """agent::step minus react for every env; (reward, done) if fetch."""
        check(_lib.lib.xh_venv_step(self.h, 1 if write_obs else 0))
        if fetch:
            return self.get(VENV_REWARD), self.get(VENV_DONE)
        return None

    def apply(self, mask=None):
        """environment::apply(actions[e], e) for the masked envs (no reset);
        returns game_over per env ([N] uint8; 0 for the envs not applied)."""
        if mask is not None:
            self.set(VENV_MASK, np.asarray(mask, np.uint8))
        check(_lib.lib.xh_venv_apply(self.h, 0 if mask is None else 1))
        return self.get(VENV_DONE)

    def reset(self, mask=None):
        """environment::reset(e) for the masked envs (all if mask is None)."""
        if mask is not None:
            self.set(VENV_MASK, np.asarray(mask, np.uint8))
        check(_lib.lib.xh_venv_reset(self.h, 0 if mask is None else 1))

    def observe(self):
        """observation::to_vector of every env: [N][B][2D] float32."""
        check(_lib.lib.xh_venv_observe(self.h))
        return self.get(VENV_OBS)

    def view(self):
        """(bins [N][B][D] int8, items [N][D] int8): environment::view."""
        return self.get(VENV_BINS), self.get(VENV_ITEMS)[:, :self.D]

    def synchronize(self):
        check(_lib.lib.xh_venv_synchronize(self.h))

    def set_timing(self, on):
        """HIP events around every later launch (xh_venv_set_timing); drops
        the events recorded so far."""
        check(_lib.lib.xh_venv_set_timing(self.h, 1 if on else 0))

    def kernel_time(self):
        """(milliseconds, launches) of the timed launches."""
        ms, n = C.c_double(), C.c_long()
        check(_lib.lib.xh_venv_kernel_time(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def close(self):
        if self.h:
            check(_lib.lib.xh_venv_destroy(self.h))
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
