// value_kernels.hip -- around the value MLP (full_layer B*2D -> V1 -> V2 -> 1,
// ppo_training.cc:19-26, which runs on the Dense MFMA GEMMs of
// dense_kernels.hip): TD targets, GAE, gradient slab reduction and the
// optimizers.
#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {

// TD(0) targets (policy_gradient.h:205-215): r + gamma * V(next row); the
// next row of a terminal transition is its (un-zeroed) terminal state.
__global__ void value_targets_kernel(ValueArgs a, float gamma, float *targets) {
#pragma clang fp contract(off)
  const int N = a.b.N, T = a.b.T;
  const long n = (long)N * T;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
       q += (long)gridDim.x * blockDim.x) {
    const int done = a.b.done[q];
    const float reward = done ? 0.0f : 1.0f;
    const float vn = done ? a.v_term[q] : a.v_state[q + N];
    targets[q] = reward + gamma * vn;
    // square_loss_grad (nn.h:548-550) of the value step's transition rows
    if (a.row_g) a.row_g[q] = a.v_state[q] - targets[q];
  }
}

// calculate_advantage (policy_gradient.h:220-281) on post-update values:
// V(terminal end row) = 0, delta_t = r + gamma V' - V, A_t = sum_i
// delta_i (lambda gamma)^(i-t) within the segment.  The reference's O(T^2)
// forward sum is evaluated as the equivalent reverse recurrence A_t = delta_t
// + lambda gamma A_{t+1} (A_t = delta_t on the terminal step), one env per
// lane and no per-step arrays, so T is not bounded by registers (SURVEY
// App. A.6: a reverse scan is allowed within tolerance).
// part != nullptr (advantage normalisation, opt-in): the block's sum and sum
// of squares of its advantages in double, reduced across the wave with
// shuffles and across the block's waves in LDS, written to part[block][2].
__global__ __launch_bounds__(256) void gae_kernel(ValueArgs a, float gamma,
                                                  float lambda, float *adv,
                                                  double *part) {
#pragma clang fp contract(off)
  const int N = a.b.N, T = a.b.T;
  const float lg = lambda * gamma;
  double s1 = 0.0, s2 = 0.0;
  // T in chunks of up to 8 steps, latest first: every load of a chunk (its
  // done bytes and the 9 values V(S_t0-7) .. V(S_t0+1)) issued before the
  // chunk's arithmetic and unconditionally (the terminal step's V(S_t+1) is
  // loaded and then not used), so one HBM round trip per chunk instead of
  // two dependent ones per step; the arithmetic is unchanged (bit-identical)
  constexpr int C = 8;
  for (int env = blockIdx.x * blockDim.x + threadIdx.x; env < N;
       env += gridDim.x * blockDim.x) {
    float A = 0.0f;
    for (int hi = T - 1; hi >= 0; hi -= C) {
      int dn[C];
      float v[C + 1];
#pragma unroll
      for (int k = 0; k < C; ++k) {
        const int t = hi - k;
        dn[k] = t >= 0 ? a.b.done[(size_t)t * N + env] : 0;
      }
#pragma unroll
      for (int k = 0; k <= C; ++k) {
        const int t = hi + 1 - k;  // v[k] = V(S_t), t = hi + 1 .. hi - 7
        v[k] = t >= 0 ? a.v_state[(size_t)t * N + env] : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < C; ++k) {
        const int t = hi - k;
        if (t < 0) break;
        const int done = dn[k];
        const float reward = done ? 0.0f : 1.0f;
        const float vn = done ? 0.0f : v[k];
        const float delta = reward + gamma * vn - v[k + 1];
        A = done ? delta : delta + lg * A;
        adv[(size_t)t * N + env] = A;
        s1 += (double)A;
        s2 += (double)A * (double)A;
      }
    }
  }
  if (!part) return;
  __shared__ double red[2][4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, kWave);
    s2 += __shfl_xor(s2, o, kWave);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    part[2 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

// Block partials -> stats[0..1] = (sum, sum of squares), a fixed-order
// reduction in one wave (deterministic); all-reduced over ranks next.
__global__ __launch_bounds__(64) void adv_stats_kernel(const double *part,
                                                       int nparts,
                                                       double *stats) {
  double s1 = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 64) {
    s1 += part[2 * i];
    s2 += part[2 * i + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, kWave);
    s2 += __shfl_xor(s2, o, kWave);
  }
  if (threadIdx.x == 0) {
    stats[0] = s1;
    stats[1] = s2;
  }
}

// A <- (A - mean) / (std + 1e-8) over the job's `count` transition rows
// (population variance), evaluated in double and rounded once.
__global__ void adv_normalize_kernel(float *adv, long n, const double *stats,
                                     double count) {
  const double mean = stats[0] / count;
  double var = stats[1] / count - mean * mean;
  var = var > 0.0 ? var : 0.0;
  const double inv = 1.0 / (sqrt(var) + 1e-8);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    adv[i] = (float)(((double)adv[i] - mean) * inv);
}

// Deterministic slab reduction: the sum over slabs in a fixed order.
// A 256-thread block takes 64 consecutive entries x 4 slab ranges (each
// wave reads 256-byte rows, enough blocks to cover the chip); the 4 range
// sums combine in LDS as (s0 + s1) + (s2 + s3).  Returned to wave 0's lanes.
// slab index whose sums entry i takes (SlabAlias: the bin-0 item column)
__device__ __forceinline__ int slab_src(int i, const SlabAlias &al) {
  if (al.B > 0 && i < al.rows * al.in) {
    const int col = i % al.in, b = col / (2 * al.D);
    if (b > 0 && col - b * 2 * al.D >= al.D) return i - b * 2 * al.D;
  }
  return i;
}
// kSlabRows partial sums per parameter (wave r sums slabs r, r + kSlabRows,
// ...: the loads of one step are kSlabRows rows apart, and every wave's
// serial chain is nslab / kSlabRows long), then a fixed-order pairwise tree:
// deterministic, the same bits run to run
constexpr int kSlabRows = 16;
__device__ __forceinline__ float slab_sum(const float *slab, int nslab,
                                          int stride, int n, int i,
                                          int src) {
  __shared__ float part[kSlabRows][64];
  const int p = threadIdx.x & 63, r = threadIdx.x >> 6;
  float s = 0.0f;
  if (i < n) {
#pragma unroll 8
    for (int k = r; k < nslab; k += kSlabRows) s += slab[(size_t)k * stride + src];
  }
  part[r][p] = s;
  __syncthreads();
  float t[kSlabRows];
#pragma unroll
  for (int q = 0; q < kSlabRows; ++q) t[q] = part[q][p];
#pragma unroll
  for (int w = kSlabRows / 2; w >= 1; w >>= 1)
#pragma unroll
    for (int q = 0; q < w; ++q) t[q] = t[q] + t[q + w];
  return t[0];
}

__global__ __launch_bounds__(64 * kSlabRows) void slab_reduce_kernel(const float *slab,
                                                          int nslab, int stride,
                                                          int n, float *out,
                                                          SlabAlias al) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const float g = slab_sum(slab, nslab, stride, n, i, slab_src(i, al));
  if (threadIdx.x < 64 && i < n) out[i] = g;
}

// One parameter's update, the reference's operation order:
//   sgd_optimizer::next_parameters (nn.h:622-625): p * (1 - wd) - g * lr
//   momentum_optimizer::next_parameters (nn.h:637-651): v = rho v + g;
//     p - v * lr
//   adam_optimizer::next_parameters (nn.h:666-691): m, v moments,
//     bias-corrected by c1 = 1 - beta1^t, c2 = 1 - beta2^t;
//     p - m^ lr / (sqrt(v^) + 1e-7)
__device__ __forceinline__ void opt_update(float *p, float *m, float *v, int i,
                                           float gi, const OptStep &o) {
#pragma clang fp contract(off)
  if (o.kind == 0) {
    p[i] = p[i] * (1.0f - o.wd) - gi * o.lr;
  } else if (o.kind == 1) {
    const float vel = 0.9f * m[i] + gi;
    m[i] = vel;
    p[i] = p[i] - vel * o.lr;
  } else {
    const float m1 = m[i] * o.beta1 + gi * (1.0f - o.beta1);
    const float m2 = v[i] * o.beta2 + gi * gi * (1.0f - o.beta2);
    m[i] = m1;
    v[i] = m2;
    const float mu = m1 / o.c1, vu = m2 / o.c2;
    p[i] = p[i] - mu * o.lr / (sqrtf(vu) + 1e-7f);
  }
}

// sgd_optimizer::next_parameters (nn.h:622-625): p * (1 - wd) - g * lr
__global__ void sgd_kernel(float *p, const float *g, int n, float lr,
                           float wd) {
#pragma clang fp contract(off)
  const float keep = 1.0f - wd;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += gridDim.x * blockDim.x)
    p[i] = p[i] * keep - g[i] * lr;
}

// momentum / adam steps (opt_update), one element per lane
__global__ void opt_kernel(float *p, const float *g, float *m, float *v, int n,
                           OptStep o) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += gridDim.x * blockDim.x)
    opt_update(p, m, v, i, g[i], o);
}

// Single rank: the slab reduce and the optimizer step in one launch (the
// reduced gradient is still written out for introspection).
__global__ __launch_bounds__(64 * kSlabRows) void slab_reduce_opt_kernel(
    const float *slab, int nslab, int stride, int n, float *out, float *p,
    float *m, float *v, OptStep o, SlabAlias al) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const float g = slab_sum(slab, nslab, stride, n, i, slab_src(i, al));
  if (threadIdx.x < 64 && i < n) {
    out[i] = g;
    opt_update(p, m, v, i, g, o);
  }
}

// ----------------------------------------------------------- launchers ----
bool value_shape_supported(int V1, int V2) {
  return V1 >= 1 && V1 <= 1024 && V2 >= 1 && V2 <= 1024;
}

static int blocks_for(long n, int per = 256, int cap = 4096) {
  long b = (n + per - 1) / per;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

hipError_t launch_value_targets(const ValueArgs &a, float gamma, float *targets,
                                hipStream_t s) {
  hipLaunchKernelGGL(value_targets_kernel, dim3(blocks_for((long)a.b.N * a.b.T)),
                     dim3(256), 0, s, a, gamma, targets);
  return hipGetLastError();
}

// one env per thread up to 2^20 envs (the scan's loads are latency-bound:
// every env's chain in flight at once)
int gae_grid(int N) { return blocks_for(N, 256, 4096); }

hipError_t launch_gae(const ValueArgs &a, float gamma, float lambda, float *adv,
                      double *part, hipStream_t s) {
  hipLaunchKernelGGL(gae_kernel, dim3(gae_grid(a.b.N)), dim3(256), 0, s, a,
                     gamma, lambda, adv, part);
  return hipGetLastError();
}

hipError_t launch_adv_stats(const double *part, int nparts, double *stats,
                            hipStream_t s) {
  hipLaunchKernelGGL(adv_stats_kernel, dim3(1), dim3(64), 0, s, part, nparts,
                     stats);
  return hipGetLastError();
}

hipError_t launch_adv_normalize(float *adv, long n, const double *stats,
                                double count, hipStream_t s) {
  hipLaunchKernelGGL(adv_normalize_kernel, dim3(blocks_for(n)), dim3(256), 0, s,
                     adv, n, stats, count);
  return hipGetLastError();
}

hipError_t launch_slab_reduce(const float *slab, int nslab, int stride, int n,
                              float *out, hipStream_t s, SlabAlias al) {
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((n + 63) / 64), dim3(64 * kSlabRows), 0, s,
                     slab, nslab, stride, n, out, al);
  return hipGetLastError();
}

hipError_t launch_slab_reduce_opt(const float *slab, int nslab, int stride,
                                  int n, float *out, float *params, float *m,
                                  float *v, OptStep o, hipStream_t s,
                                  SlabAlias al) {
  hipLaunchKernelGGL(slab_reduce_opt_kernel, dim3((n + 63) / 64), dim3(64 * kSlabRows), 0,
                     s, slab, nslab, stride, n, out, params, m, v, o, al);
  return hipGetLastError();
}

hipError_t launch_sgd(float *params, const float *grad, int n, float lr,
                      float wd, hipStream_t s) {
  hipLaunchKernelGGL(sgd_kernel, dim3(blocks_for(n)), dim3(256), 0, s, params,
                     grad, n, lr, wd);
  return hipGetLastError();
}

hipError_t launch_opt(float *params, const float *grad, float *m, float *v,
                      int n, OptStep o, hipStream_t s) {
  hipLaunchKernelGGL(opt_kernel, dim3(blocks_for(n)), dim3(256), 0, s, params,
                     grad, m, v, n, o);
  return hipGetLastError();
}

}  // namespace xh
