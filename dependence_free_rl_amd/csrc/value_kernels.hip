// value_kernels.hip -- the value MLP (full_layer B*2D -> V1 -> V2 -> 1,
// ppo_training.cc:19-26), TD targets, GAE, gradient slab reduction and SGD.
//
// The value net is ~1% of the iteration's FLOPs, so it runs on the f32 VALU
// (whose peak equals the f32 MFMA peak on gfx950): one lane per row for the
// forward / per-row backward, and a split-K "one thread per weight column"
// kernel for the weight gradients (weights and per-row deltas are read with
// wave-uniform scalar loads).
#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {

// Row feature k of S_slot[env] (observation::to_vector, bin_packing.h:31-40);
// `term_choice` >= 0 yields the terminal view E_t (bins[c] -= item, item kept).
__device__ __forceinline__ void row_bins(const EnvDesc &E, const Batch &b,
                                         int slot, int env, const int8_t *&bp,
                                         int (&iv)[3]) {
  const int BD = E.B * E.D;
  bp = b.bins + ((size_t)slot * b.N + env) * BD;
  const int8_t *ip = b.items + ((size_t)slot * b.N + env) * 4;
  iv[0] = ip[0];
  iv[1] = ip[1];
  iv[2] = ip[2];
}

template <int V1, int V2>
__device__ __forceinline__ float value_forward(const ValueArgs &a, int slot,
                                               int env, int term_choice,
                                               float (&h1)[V1], float (&h2)[V2],
                                               float (&p1)[V1],
                                               float (&p2)[V2]) {
  const EnvDesc &E = a.env;
  const ValueLayout L{E.B * 2 * E.D, V1, V2};
  const float *__restrict__ P = a.params;
  const int8_t *bp;
  int iv[3];
  row_bins(E, a.b, slot, env, bp, iv);
  float acc[V1];
#pragma unroll
  for (int o = 0; o < V1; ++o) acc[o] = 0.0f;
  const float inv = 1.0f / (float)kCapacity;  // exact (power of two)
  for (int bin = 0; bin < E.B; ++bin) {
    for (int c = 0; c < 2 * E.D; ++c) {
      int v;
      if (c < E.D) {
        v = bp[bin * E.D + c];
        if (bin == term_choice) v -= iv[c];
      } else {
        v = iv[c - E.D];
      }
      const float x = (float)v * inv;
      const float *__restrict__ wk = a.w1t + (size_t)(bin * 2 * E.D + c) * V1;
#pragma unroll
      for (int o = 0; o < V1; ++o) acc[o] += x * wk[o];
    }
  }
#pragma unroll
  for (int o = 0; o < V1; ++o) {
    p1[o] = acc[o] + P[L.ob1() + o];
    h1[o] = p1[o] > 0.0f ? p1[o] : 0.0f;
  }
#pragma unroll
  for (int o = 0; o < V2; ++o) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < V1; ++i) s += h1[i] * P[L.oW2() + o * V1 + i];
    p2[o] = s + P[L.ob2() + o];
    h2[o] = p2[o] > 0.0f ? p2[o] : 0.0f;
  }
  float v = 0.0f;
#pragma unroll
  for (int o = 0; o < V2; ++o) v += h2[o] * P[L.ow3() + o];
  return v + P[L.ob3()];
}

// model::eval (nn.h:473-479) over S_0..S_T and the terminal views E_0..E_{T-1}.
template <int V1, int V2>
__global__ __launch_bounds__(256) void value_eval_kernel(ValueArgs a) {
  const int N = a.b.N, T = a.b.T;
  const long rows = (long)N * (T + 1) + (a.with_term ? (long)N * T : 0);
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < rows;
       r += (long)gridDim.x * blockDim.x) {
    float h1[V1], h2[V2], p1[V1], p2[V2];
    if (r < (long)N * (T + 1)) {
      const int slot = (int)(r / N), env = (int)(r % N);
      a.v_state[r] = value_forward<V1, V2>(a, slot, env, -1, h1, h2, p1, p2);
    } else {
      const long q = r - (long)N * (T + 1);
      const int t = (int)(q / N), env = (int)(q % N);
      const int c = a.b.action[q];
      a.v_term[q] = value_forward<V1, V2>(a, t, env, c, h1, h2, p1, p2);
    }
  }
}

// Value step rows (update_value_model, policy_gradient.h:196-218): forward,
// square_loss_grad (nn.h:548-550) g = V - target, per-row backward through
// the two relu layers (nn.h:81-100, 364-376).  End rows are skipped: their
// target is their own value, so their gradient is exactly zero.
template <int V1, int V2>
__global__ __launch_bounds__(256) void value_rows_kernel(ValueArgs a) {
  const int N = a.b.N, T = a.b.T;
  const ValueLayout L{a.env.B * 2 * a.env.D, V1, V2};
  const float *__restrict__ P = a.params;
  const long rows = (long)N * T;
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < rows;
       r += (long)gridDim.x * blockDim.x) {
    const int t = (int)(r / N), env = (int)(r % N);
    float h1[V1], h2[V2], p1[V1], p2[V2];
    const float v = value_forward<V1, V2>(a, t, env, -1, h1, h2, p1, p2);
    const float g = v - a.targets[r];
    a.row_g[r] = g;
    float d2[V2];
#pragma unroll
    for (int o = 0; o < V2; ++o) {
      const float dh = g * P[L.ow3() + o];
      d2[o] = p2[o] > 0.0f ? dh : 0.0f;
      a.row_h2[r * V2 + o] = h2[o];
      a.row_d2[r * V2 + o] = d2[o];
    }
#pragma unroll
    for (int i = 0; i < V1; ++i) {
      float s = 0.0f;
#pragma unroll
      for (int o = 0; o < V2; ++o) s += d2[o] * P[L.oW2() + o * V1 + i];
      a.row_h1[r * V1 + i] = h1[i];
      a.row_d1[r * V1 + i] = p1[i] > 0.0f ? s : 0.0f;
    }
  }
}

// Split-K weight gradients of the value net: workgroup w sums a contiguous
// chunk of rows into its slab (flat model::parameters() layout).
//   dW1[o][k] = sum_r d1[r][o] x[r][k]   thread -> feature column k
//   dW2[o][i] = sum_r d2[r][o] h1[r][i]  thread -> (i, 8 o's)
//   db1, db2, dw3, db3                   thread -> one entry
template <int V1, int V2, int KPT>
__global__ __launch_bounds__(256) void value_wgrad_kernel(ValueArgs a,
                                                          float *slab,
                                                          int stride) {
  static_assert(V1 * V2 <= 2048 && 256 % V1 == 0, "dW2 mapping");
  const EnvDesc &E = a.env;
  const int Fin = E.B * 2 * E.D;
  const ValueLayout L{Fin, V1, V2};
  const int N = a.b.N, T = a.b.T;
  const long rows = (long)N * T;
  const long per = (rows + gridDim.x - 1) / gridDim.x;
  const long r0 = blockIdx.x * per, r1 = min(rows, r0 + per);
  const int tid = threadIdx.x;
  // KPT feature columns per thread (Fin <= 256 * KPT)
  float aw1[KPT][V1];
#pragma unroll
  for (int m = 0; m < KPT; ++m)
#pragma unroll
    for (int o = 0; o < V1; ++o) aw1[m][o] = 0.0f;
  constexpr int OPT = (V1 * V2 + 255) / 256;  // dW2 entries per thread
  float aw2[OPT];
#pragma unroll
  for (int q = 0; q < OPT; ++q) aw2[q] = 0.0f;
  float ab1 = 0.0f, ab2 = 0.0f, aw3 = 0.0f, ab3 = 0.0f;
  const int i2 = tid % V1, o2base = (tid / V1) * OPT;

  for (long r = r0; r < r1; ++r) {
    const int t = (int)(r / N), env = (int)(r % N);
    const float *__restrict__ d1 = a.row_d1 + r * V1;
    const float *__restrict__ d2 = a.row_d2 + r * V2;
    const int8_t *bp;
    int iv[3];
    row_bins(E, a.b, t, env, bp, iv);
#pragma unroll
    for (int m = 0; m < KPT; ++m) {
      const int k = tid + m * 256;
      if (k < Fin) {
        const int bin = k / (2 * E.D), c = k - bin * 2 * E.D;
        const int v = c < E.D ? bp[bin * E.D + c] : iv[c - E.D];
        const float x = (float)v / (float)kCapacity;
#pragma unroll
        for (int o = 0; o < V1; ++o) aw1[m][o] += d1[o] * x;
      }
    }
    const float hv = a.row_h1[r * V1 + i2];
#pragma unroll
    for (int q = 0; q < OPT; ++q)
      if (o2base + q < V2) aw2[q] += d2[o2base + q] * hv;
    if (tid < V1) ab1 += d1[tid];
    if (tid < V2) {
      ab2 += d2[tid];
      aw3 += a.row_g[r] * a.row_h2[r * V2 + tid];
    }
    if (tid == 0) ab3 += a.row_g[r];
  }
  float *s = slab + (size_t)blockIdx.x * stride;
#pragma unroll
  for (int m = 0; m < KPT; ++m) {
    const int k = tid + m * 256;
    if (k < Fin)
#pragma unroll
      for (int o = 0; o < V1; ++o) s[L.oW1() + o * Fin + k] = aw1[m][o];
  }
#pragma unroll
  for (int q = 0; q < OPT; ++q)
    if (o2base + q < V2 && tid / V1 * OPT < V2)
      s[L.oW2() + (o2base + q) * V1 + i2] = aw2[q];
  if (tid < V1) s[L.ob1() + tid] = ab1;
  if (tid < V2) {
    s[L.ob2() + tid] = ab2;
    s[L.ow3() + tid] = aw3;
  }
  if (tid == 0) s[L.ob3()] = ab3;
}

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
  }
}

// calculate_advantage (policy_gradient.h:220-281) on post-update values:
// V(terminal end row) = 0, delta_t = r + gamma V' - V, A_t = sum_i
// delta_i (lambda gamma)^(i-t) within the segment (forward sum, coefficient by
// repeated multiplication, as the reference).
__global__ void gae_kernel(ValueArgs a, float gamma, float lambda, float *adv) {
#pragma clang fp contract(off)
  const int N = a.b.N, T = a.b.T;
  for (int env = blockIdx.x * blockDim.x + threadIdx.x; env < N;
       env += gridDim.x * blockDim.x) {
    float delta[64];
    int done[64];
    for (int t = 0; t < T; ++t) {
      const size_t q = (size_t)t * N + env;
      done[t] = a.b.done[q];
      const float reward = done[t] ? 0.0f : 1.0f;
      const float vn = done[t] ? 0.0f : a.v_state[q + N];
      delta[t] = reward + gamma * vn - a.v_state[q];
    }
    const float lg = lambda * gamma;
    for (int t = 0; t < T; ++t) {
      float A = 0.0f, coef = 1.0f;
      for (int i = t; i < T; ++i) {
        A += delta[i] * coef;
        coef *= lg;
        if (done[i]) break;
      }
      adv[(size_t)t * N + env] = A;
    }
  }
}

__global__ void transpose_kernel(const float *src, float *dst, int rows,
                                 int cols) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
       i < (long)rows * cols; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    dst[(size_t)c * rows + r] = src[i];
  }
}

// Deterministic slab reduction: out[i] = sum over slabs in a fixed order.
// A 256-thread block takes 64 consecutive entries x 4 slab ranges (each
// wave reads 256-byte rows, enough blocks to cover the chip); the 4 range
// sums combine in LDS as (s0 + s1) + (s2 + s3).
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float *slab,
                                                          int nslab, int stride,
                                                          int n, float *out) {
  __shared__ float part[4][64];
  const int p = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + p;
  const int per = (nslab + 3) / 4, k0 = r * per,
            k1 = k0 + per < nslab ? k0 + per : nslab;
  float s = 0.0f;
  if (i < n) {
#pragma unroll 8
    for (int k = k0; k < k1; ++k) s += slab[(size_t)k * stride + i];
  }
  part[r][p] = s;
  __syncthreads();
  if (r == 0 && i < n)
    out[i] = (part[0][p] + part[1][p]) + (part[2][p] + part[3][p]);
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

// momentum_optimizer::next_parameters (nn.h:637-651): v = rho v + g;
// p - v * lr.  adam_optimizer::next_parameters (nn.h:666-691): m, v moments,
// bias-corrected by c1 = 1 - beta1^t, c2 = 1 - beta2^t; p - m^ lr /
// (sqrt(v^) + 1e-7).  One element per lane, the reference's operation order.
__global__ void opt_kernel(float *p, const float *g, float *m, float *v, int n,
                           OptStep o) {
#pragma clang fp contract(off)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += gridDim.x * blockDim.x) {
    const float gi = g[i];
    if (o.kind == 1) {
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
}

// ----------------------------------------------------------- launchers ----
bool value_shape_supported(int V1, int V2) {
  return (V1 == 64 && V2 == 32) || (V1 == 32 && V2 == 32);
}

#define XH_VALUE_SHAPES(X) X(64, 32) X(32, 32)

static int blocks_for(long n, int per = 256, int cap = 4096) {
  long b = (n + per - 1) / per;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

hipError_t launch_value_eval(const ValueArgs &a, int V1, int V2,
                             hipStream_t s) {
  const long rows =
      (long)a.b.N * (a.b.T + 1) + (a.with_term ? (long)a.b.N * a.b.T : 0);
#define X(v1, v2)                                                         \
  if (V1 == v1 && V2 == v2) {                                             \
    hipLaunchKernelGGL((value_eval_kernel<v1, v2>), dim3(blocks_for(rows)), \
                       dim3(256), 0, s, a);                               \
    return hipGetLastError();                                             \
  }
  XH_VALUE_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_value_rows(const ValueArgs &a, int V1, int V2,
                             hipStream_t s) {
  const long rows = (long)a.b.N * a.b.T;
#define X(v1, v2)                                                         \
  if (V1 == v1 && V2 == v2) {                                             \
    hipLaunchKernelGGL((value_rows_kernel<v1, v2>), dim3(blocks_for(rows)), \
                       dim3(256), 0, s, a);                               \
    return hipGetLastError();                                             \
  }
  XH_VALUE_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_value_wgrad(const ValueArgs &a, int V1, int V2, float *slab,
                              int stride, int grid, hipStream_t s) {
  const int Fin = a.env.B * 2 * a.env.D;
  if (Fin > 768) return hipErrorInvalidValue;
#define X(v1, v2)                                                            \
  if (V1 == v1 && V2 == v2) {                                                \
    if (Fin <= 256)                                                          \
      hipLaunchKernelGGL((value_wgrad_kernel<v1, v2, 1>), dim3(grid),        \
                         dim3(256), 0, s, a, slab, stride);                  \
    else                                                                     \
      hipLaunchKernelGGL((value_wgrad_kernel<v1, v2, 3>), dim3(grid),        \
                         dim3(256), 0, s, a, slab, stride);                  \
    return hipGetLastError();                                                \
  }
  XH_VALUE_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_value_targets(const ValueArgs &a, float gamma, float *targets,
                                hipStream_t s) {
  hipLaunchKernelGGL(value_targets_kernel, dim3(blocks_for((long)a.b.N * a.b.T)),
                     dim3(256), 0, s, a, gamma, targets);
  return hipGetLastError();
}

hipError_t launch_gae(const ValueArgs &a, float gamma, float lambda, float *adv,
                      hipStream_t s) {
  hipLaunchKernelGGL(gae_kernel, dim3(blocks_for(a.b.N)), dim3(256), 0, s, a,
                     gamma, lambda, adv);
  return hipGetLastError();
}

hipError_t launch_transpose(const float *src, float *dst, int rows, int cols,
                            hipStream_t s) {
  hipLaunchKernelGGL(transpose_kernel, dim3(blocks_for((long)rows * cols)),
                     dim3(256), 0, s, src, dst, rows, cols);
  return hipGetLastError();
}

hipError_t launch_slab_reduce(const float *slab, int nslab, int stride, int n,
                              float *out, hipStream_t s) {
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((n + 63) / 64), dim3(256), 0, s,
                     slab, nslab, stride, n, out);
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
