// heuristic_kernels.hip -- the reference's heuristic agents as device
// policies: firstfit (firstfit_agent.cc:10-28), bestfit
// (bestfit_agent.cc:10-30), minwaste (minwaste_agent.cc:10-39) and the
// uniform random_policy (rl.h:305-316), each playing whole episodes of the
// bin-packing env (bin_packing.h:46-107) on independent envs.
//
// Layout: one wave runs G = 64/B envs, lane = (env, bin); an env's state
// (its bins, the item, the engine) lives in registers for the whole run, so
// the kernel never touches HBM inside the step loop: it is bound by VALU /
// cross-lane latency, not by memory.  No LDS, no barriers: every wave runs
// its own envs to completion.
#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {

template <int B, int D, int KIND>
__global__ __launch_bounds__(256) void heuristic_kernel(HeuristicArgs a) {
  static_assert(B <= 64, "one segment per env");
  constexpr int G = 64 / B;
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * (blockDim.x / 64);
  const int ngroups = a.n_envs / G;
  const int e = lane / B, bin = lane % B;
  for (int grp = wave; grp < ngroups; grp += nwaves) {
    const int env = grp * G + e;
    uint32_t x = mstd_jump(a.x0, (uint64_t)env * a.stream_stride);
    int item[D], bv[D];
    {
      bool first = false;
      if (!a.init_items) first = canonical(x) < a.env.p_a;  // environment()
#pragma unroll
      for (int d = 0; d < D; ++d) {
        item[d] = a.init_items ? a.init_items[env * D + d]
                               : (first ? a.env.item_a[d] : a.env.item_b[d]);
        bv[d] = kCapacity;
      }
    }
    int left = a.episodes;
    double reward = 0.0;
    long steps = 0;
    for (long it = 0; it < a.max_steps; ++it) {
      const bool active = left > 0;
      if (!__any(active)) break;
      // ---- react: the policy's scores, then from_vector_deterministic
      bool fits = true;
#pragma unroll
      for (int d = 0; d < D; ++d) fits = fits && item[d] <= bv[d];
      int choice;
      if constexpr (KIND == kHeurRandom) {
        // v = 1.0 / N (a float vector), discrete_distribution: 2 draws
        const float p = (float)(1.0 / B);
        const double u = active ? canonical(x) : 0.0;
        choice = sample_discrete<B>(p, lane, u);
      } else {
        float sc;
        if constexpr (KIND == kHeurFirstfit) {
          sc = fits ? 1.0f : 0.0f;  // the first fitting bin scores 1
        } else if constexpr (KIND == kHeurBestfit) {
          sc = -1.0f;
          if (fits) {
            sc = (float)item[0] / (float)bv[0];
#pragma unroll
            for (int d = 1; d < D; ++d) sc = sc + (float)item[d] / (float)bv[d];
          }
        } else {  // minwaste: 0 when the residual is (cap/2, 0) or (0, cap/2)
          sc = -1.0f;
          if (fits) {
            int half = 0, zero = 0;
#pragma unroll
            for (int d = 0; d < D; ++d) {
              const int r = bv[d] - item[d];
              half += r == kCapacity / 2;
              zero += r == 0;
            }
            sc = (half == 1 && zero == D - 1) ? 0.0f : 1.0f;
          }
        }
        choice = seg_argmax_first<B>(sc, bin);
      }
      // ---- apply (bin_packing.h:53-64); overflow -> reset; get_item
      int nb[D];
      int neg = 0;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        nb[d] = bin == choice ? bv[d] - item[d] : bv[d];
        neg |= nb[d] < 0;
      }
      const int done = __shfl(neg, e * B + choice, kWave);
      if (active) {
        const bool first = canonical(x) < a.env.p_a;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          bv[d] = done ? kCapacity : nb[d];
          item[d] = first ? a.env.item_a[d] : a.env.item_b[d];
        }
        if (a.trace && env == 0 && bin == 0 && steps < a.trace_cap)
          a.trace[steps] = choice;
        reward += done ? 0.0 : 1.0;
        ++steps;
        left -= done;
      }
    }
    if (bin == 0) {
      a.total[env] = reward;
      a.steps[env] = steps;
      a.rng_out[env] = x;
#pragma unroll
      for (int d = 0; d < D; ++d) a.final_items[env * D + d] = item[d];
    }
  }
}

template <int B, int D>
hipError_t launch_heuristic_bd(const HeuristicArgs &a, int kind, int grid,
                               hipStream_t s) {
  switch (kind) {
    case kHeurRandom:
      hipLaunchKernelGGL((heuristic_kernel<B, D, kHeurRandom>), dim3(grid),
                         dim3(256), 0, s, a);
      break;
    case kHeurFirstfit:
      hipLaunchKernelGGL((heuristic_kernel<B, D, kHeurFirstfit>), dim3(grid),
                         dim3(256), 0, s, a);
      break;
    case kHeurBestfit:
      hipLaunchKernelGGL((heuristic_kernel<B, D, kHeurBestfit>), dim3(grid),
                         dim3(256), 0, s, a);
      break;
    case kHeurMinwaste:
      hipLaunchKernelGGL((heuristic_kernel<B, D, kHeurMinwaste>), dim3(grid),
                         dim3(256), 0, s, a);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

bool heuristic_shape_supported(int B, int D) {
  return (B == 8 || B == 16 || B == 32 || B == 64) && D >= 1 && D <= 3;
}

hipError_t launch_heuristic(const HeuristicArgs &a, int kind, hipStream_t s) {
  const int B = a.env.B, D = a.env.D;
  const int groups = a.n_envs / (64 / B);
  const int waves_per_block = 4;
  int grid = (groups + waves_per_block - 1) / waves_per_block;
  if (grid > 65536) grid = 65536;
#define XH_H(XB, XD) \
  if (B == XB && D == XD) return launch_heuristic_bd<XB, XD>(a, kind, grid, s);
  XH_H(8, 1) XH_H(8, 2) XH_H(8, 3) XH_H(16, 1) XH_H(16, 2) XH_H(16, 3)
  XH_H(32, 1) XH_H(32, 2) XH_H(32, 3) XH_H(64, 1) XH_H(64, 2) XH_H(64, 3)
#undef XH_H
  return hipErrorInvalidValue;
}

}  // namespace xh
