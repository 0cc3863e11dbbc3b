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

hipError_t launch_gae(const ValueArgs &a, float gamma, float lambda, float *adv,
                      hipStream_t s) {
  hipLaunchKernelGGL(gae_kernel, dim3(blocks_for(a.b.N)), dim3(256), 0, s, a,
                     gamma, lambda, adv);
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
