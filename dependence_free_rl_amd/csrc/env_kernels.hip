// env_kernels.hip -- vectorised bin-packing environment construction.
//
// Reference order of the engine draws: the N_global envs are
// constructed one after another (2 draws each: environment() -> get_item,
// bin_packing.h:50-52,76-81), then every iteration steps worker 0 for T steps,
// worker 1 for T steps, ... (ppo_training.cc:53-62 run sequentially), 4 draws
// per step.  Env g therefore starts its iteration-0 steps at stream position
// 2*N_global + 4*T*g; each env holds its own minstd state and jumps ahead
// instead of sharing one racy engine (tensor.cc:71-75).
#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {

__global__ void env_init_kernel(EnvDesc E, Batch b, uint32_t x0,
                                int env_offset, int n_global) {
  const int BD = E.B * E.D;
  for (int env = blockIdx.x * blockDim.x + threadIdx.x; env < b.N;
       env += gridDim.x * blockDim.x) {
    const uint64_t g = (uint64_t)env_offset + env;
    uint32_t x = mstd_jump(x0, 2 * g);  // this env's construction draws
    const bool first = canonical(x) < E.p_a;
    int8_t *bp = b.bins + (size_t)env * BD;  // slot 0
    for (int i = 0; i < BD; ++i) bp[i] = (int8_t)kCapacity;
    int8_t *ip = b.items + (size_t)env * 4;
    for (int d = 0; d < 4; ++d)
      ip[d] = d < E.D ? (int8_t)(first ? E.item_a[d] : E.item_b[d]) : 0;
    // position after construction: 2g + 2 -> first step: 2 Ng + 4 T g
    const uint64_t target = 2ull * n_global + 4ull * b.T * g;
    b.rng[env] = mstd_jump(x, target - (2 * g + 2));
  }
}

hipError_t launch_env_init(const EnvDesc &env, Batch b, uint32_t x0,
                           int env_offset, int n_global, hipStream_t s) {
  const int blocks = (b.N + 255) / 256;
  hipLaunchKernelGGL(env_init_kernel, dim3(blocks), dim3(256), 0, s, env, b,
                     x0, env_offset, n_global);
  return hipGetLastError();
}

// xh_trainer_seed_streams: window-start stream of env g = x advanced 4*T*g.
__global__ void env_seed_kernel(Batch b, uint32_t x, int env_offset) {
  for (int env = blockIdx.x * blockDim.x + threadIdx.x; env < b.N;
       env += gridDim.x * blockDim.x)
    b.rng[env] = mstd_jump(x, 4ull * b.T * ((uint64_t)env_offset + env));
}

hipError_t launch_env_seed(Batch b, uint32_t x, int env_offset,
                           hipStream_t s) {
  const int blocks = (b.N + 255) / 256;
  hipLaunchKernelGGL(env_seed_kernel, dim3(blocks), dim3(256), 0, s, b, x,
                     env_offset);
  return hipGetLastError();
}

}  // namespace xh
