// pg_kernels.hip -- REINFORCE (policy_gradient_learner, policy_gradient.h:
// 88-147; bp::pg_learner, bin_packing.h:109-116; pg_training.cc) on the
// device: whole-episode rollouts of a full-MLP softmax policy, the reversed
// discounted rewards-to-go with the mean-return baseline, and the
// softmax-log loss gradient.  The Dense layers run through dense_kernels.hip.
//
// Per iteration every env plays `episodes` whole episodes
// (agent::play_one_episode, rl.h:351-354).  Step t of the iteration is slot t
// of the Batch for every env; an env that has finished its episodes carries
// its (post-reset) state forward, so after the last step slot S holds every
// env's current state.  Learn rows are the envs' transitions in the
// reference's replay-buffer order: env 0's episodes, then env 1's, ...
#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {

// One env per thread: softmax_cross_entropy_layer::forward (nn.h:382-392, no
// max shift) of its logits, discrete_distribution sample (tensor.cc:467-470,
// sequential libstdc++ order), bp::environment::apply / get_reward / reset
// (bin_packing.h:53-106), 4 engine draws per step.
__global__ void pg_step_kernel(PgStepArgs a) {
#pragma clang fp contract(off)
  const EnvDesc &E = a.env;
  const int B = E.B, D = E.D, BD = B * D, N = a.b.N, t = a.t;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < N;
       e += gridDim.x * blockDim.x) {
    const int8_t *sb = a.b.bins + ((size_t)t * N + e) * BD;
    const int8_t *si = a.b.items + ((size_t)t * N + e) * 4;
    int8_t *ob = a.b.bins + ((size_t)(t + 1) * N + e) * BD;
    int8_t *oi = a.b.items + ((size_t)(t + 1) * N + e) * 4;
    const size_t q = (size_t)t * N + e;
    int eps = a.ep_done[e];
    if (eps >= a.episodes) {  // finished: carry the state
      for (int i = 0; i < BD; ++i) ob[i] = sb[i];
      for (int d = 0; d < 4; ++d) oi[d] = si[d];
      a.b.action[q] = -1;
      a.b.done[q] = 0;
      continue;
    }
    const float *z = a.logits + (size_t)e * B;
    float p[128];
    float sum = 0.0f;
    for (int j = 0; j < B; ++j) {
      p[j] = expf(z[j]);
      sum += p[j];
    }
    for (int j = 0; j < B; ++j) p[j] = p[j] / sum;
    uint32_t x = a.b.rng[e];
    // discrete_distribution: p -> double, / std::accumulate, partial sums,
    // last forced to 1, lower_bound(u)
    const double u = canonical(x);
    double s = 0.0;
    for (int j = 0; j < B; ++j) s += (double)p[j];
    int choice = B - 1;
    double acc = 0.0;
    for (int j = 0; j < B; ++j) {
      acc = j == 0 ? (double)p[j] / s : acc + (double)p[j] / s;
      const double cp = j == B - 1 ? 1.0 : acc;
      if (!(cp < u)) {
        choice = j;
        break;
      }
    }
    if (a.forced) choice = a.forced[q];
    int over = 0;
    for (int i = 0; i < BD; ++i) {
      int v = sb[i];
      if (i / D == choice) v -= si[i % D];
      over |= v < 0;
      ob[i] = (int8_t)v;
    }
    // get_item after the apply, or reset() -> get_item: 2 draws either way
    const bool first = canonical(x) < E.p_a;
    if (over)
      for (int i = 0; i < BD; ++i) ob[i] = (int8_t)kCapacity;
    for (int d = 0; d < 4; ++d)
      oi[d] = d < D ? (int8_t)(first ? E.item_a[d] : E.item_b[d]) : 0;
    a.b.action[q] = choice;
    a.b.pold[q] = p[choice];
    a.b.done[q] = (uint8_t)over;
    a.b.rng[e] = x;
    if (over) {
      ++eps;
      a.ep_done[e] = eps;
      if (eps == a.episodes) {
        a.len[e] = t + 1;
        atomicSub(a.active, 1);
      }
    }
  }
}

hipError_t launch_pg_step(const PgStepArgs &a, hipStream_t s) {
  if (a.env.B > 128) return hipErrorInvalidValue;
  const int blocks = (a.b.N + 255) / 256;
  hipLaunchKernelGGL(pg_step_kernel, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

// Env g (global index) on its own stream: x0 advanced by g * stride, then
// constructed (environment() -> get_item, 2 draws, bin_packing.h:50-52) into
// slot 0.  Env 0 is the single-env reference run on the global engine.
__global__ void pg_env_init_kernel(EnvDesc E, Batch b, uint32_t x0,
                                   int env_offset, uint64_t stride) {
  const int BD = E.B * E.D;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < b.N;
       e += gridDim.x * blockDim.x) {
    uint32_t x = mstd_jump(x0, ((uint64_t)env_offset + e) * stride);
    const bool first = canonical(x) < E.p_a;
    for (int i = 0; i < BD; ++i) b.bins[(size_t)e * BD + i] = (int8_t)kCapacity;
    for (int d = 0; d < 4; ++d)
      b.items[(size_t)e * 4 + d] =
          d < E.D ? (int8_t)(first ? E.item_a[d] : E.item_b[d]) : 0;
    b.rng[e] = x;
  }
}

hipError_t launch_pg_env_init(const EnvDesc &env, Batch b, uint32_t x0,
                              int env_offset, uint64_t stride, hipStream_t s) {
  hipLaunchKernelGGL(pg_env_init_kernel, dim3((b.N + 255) / 256), dim3(256), 0,
                     s, env, b, x0, env_offset, stride);
  return hipGetLastError();
}

// xh_trainer_seed_streams for REINFORCE: env g <- x advanced by g * stride.
__global__ void pg_seed_kernel(Batch b, uint32_t x, int env_offset,
                               uint64_t stride) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < b.N;
       e += gridDim.x * blockDim.x)
    b.rng[e] = mstd_jump(x, ((uint64_t)env_offset + e) * stride);
}

hipError_t launch_pg_seed(Batch b, uint32_t x, int env_offset, uint64_t stride,
                          hipStream_t s) {
  hipLaunchKernelGGL(pg_seed_kernel, dim3((b.N + 255) / 256), dim3(256), 0, s,
                     b, x, env_offset, stride);
  return hipGetLastError();
}

// Iteration start: every env active, no steps, no episodes.
__global__ void pg_begin_kernel(int N, int *active, int *ep_done, int *len) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < N;
       e += gridDim.x * blockDim.x) {
    ep_done[e] = 0;
    len[e] = 0;
    if (e == 0) *active = N;
  }
}

hipError_t launch_pg_begin(int N, int *active, int *ep_done, int *len,
                           hipStream_t s) {
  hipLaunchKernelGGL(pg_begin_kernel, dim3((N + 255) / 256), dim3(256), 0, s,
                     N, active, ep_done, len);
  return hipGetLastError();
}

// Row list in replay-buffer order (env-major, steps ascending) and each
// env's first row: one 1024-thread workgroup, chunked exclusive scan.
__global__ __launch_bounds__(1024) void pg_rows_kernel(PgLearnArgs a) {
  __shared__ int part[1024];
  __shared__ int carry;
  const int N = a.N, tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < N; base += 1024) {
    const int e = base + tid;
    const int l = e < N ? a.len[e] : 0;
    part[tid] = l;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
      const int v = tid >= o ? part[tid - o] : 0;
      __syncthreads();
      part[tid] += v;
      __syncthreads();
    }
    const int off = carry + part[tid] - l;
    if (e < N) {
      a.row_off[e] = off;
      for (int t = 0; t < l; ++t) a.list[off + t] = t * N + e;
    }
    __syncthreads();
    if (tid == 1023) carry += part[1023];
    __syncthreads();
  }
  if (tid == 0) *a.nrows = carry;
}

// policy_gradient_learner::get_advantages (policy_gradient.h:125-147): per
// trajectory, reward <- r_j + gamma * reward over the transitions in order,
// written to the slots from the END backwards (the reference's reversed
// rewards-to-go); the trajectory's slot-0 value adds to the baseline sum.
__global__ void pg_adv_kernel(PgLearnArgs a) {
#pragma clang fp contract(off)
  const int N = a.N;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < N;
       e += gridDim.x * blockDim.x) {
    const int l = a.len[e], off = a.row_off[e];
    int s = 0;
    float part = 0.0f;
    while (s < l) {
      int L = 1;
      while (s + L - 1 < l && !a.done[(size_t)(s + L - 1) * N + e]) ++L;
      if (s + L > l) L = l - s;  // (cannot happen: episodes end on done)
      float reward = 0.0f;
      for (int j = 0; j < L; ++j) {
        const float r = a.done[(size_t)(s + j) * N + e] ? 0.0f : 1.0f;
        reward = r + a.gamma * reward;
        a.rtg[off + s + L - 1 - j] = reward;
      }
      part += a.rtg[off + s];
      s += L;
    }
    a.ep_part[e] = (double)part;
  }
}

// Baseline sum over all trajectories (deterministic, one workgroup) ->
// stats[0] = sum of slot-0 returns, stats[1] = number of trajectories.
__global__ __launch_bounds__(256) void pg_sum_kernel(PgLearnArgs a) {
  __shared__ double red[256];
  double s = 0.0;
  for (int e = threadIdx.x; e < a.N; e += 256) s += a.ep_part[e];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.stats[0] = red[0];
    a.stats[1] = (double)a.N * a.episodes;
  }
}

// policy_loss -> discrete_action::softmax_gradient_log (rl.h:45-52): with
// A = rtg - mean (policy_gradient.h:146), dL/dz = A p, then -A at the chosen
// action; the softmax_cross_entropy_layer passes it through (nn.h:428-430).
__global__ void pg_loss_kernel(PgLearnArgs a) {
#pragma clang fp contract(off)
  const int R = *a.nrows, B = a.B;
  const float avg = (float)a.stats[0] / (float)a.stats[1];
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < R;
       r += gridDim.x * blockDim.x) {
    const float *z = a.logits + (size_t)r * B;
    float *g = a.dlogits + (size_t)r * B;
    float sum = 0.0f;
    for (int j = 0; j < B; ++j) sum += expf(z[j]);
    const int idx = a.list[r];
    const int c = a.action[idx];
    const float A = a.rtg[r] - avg;
    a.adv_grid[idx] = A;
    for (int j = 0; j < B; ++j) {
      const float p = expf(z[j]) / sum;
      float v = A * p;
      if (j == c) v = v - A;
      g[j] = v;
    }
  }
}

hipError_t launch_pg_rows(const PgLearnArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(pg_rows_kernel, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_pg_adv(const PgLearnArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(pg_adv_kernel, dim3((a.N + 255) / 256), dim3(256), 0, s,
                     a);
  if (hipGetLastError() != hipSuccess) return hipGetLastError();
  hipLaunchKernelGGL(pg_sum_kernel, dim3(1), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_pg_loss(const PgLearnArgs &a, int max_rows, hipStream_t s) {
  int blocks = (max_rows + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pg_loss_kernel, dim3(blocks < 1 ? 1 : blocks), dim3(256),
                     0, s, a);
  return hipGetLastError();
}

}  // namespace xh
