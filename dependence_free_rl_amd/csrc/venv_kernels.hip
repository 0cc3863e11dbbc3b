// venv_kernels.hip -- N bp::environment instances stepped by ONE kernel per
// call, for callers that bring their own policy (xh_venv_*, include/
// xylo_hip.h).  Reference: bp::environment::apply/view/reset
// (bin_packing.h:53-70, get_item :76-81), bp::agent::game_over/get_reward
// (:94-106), xylo::agent::step minus the policy's react (rl.h:325-349),
// observation::to_vector (bin_packing.h:31-40); generalised to B bins and D
// dims as the trainer's env (xylo_hip.cpp make_env).
//
// Layout in HBM: bins int8 [N][B][D], items int8 [N][4], rng u32 [N] (one
// minstd_rand0 state per env).  A lane owns one (env, bin) pair (two bins per
// lane at B = 128), so a wave covers 64 / B envs with fully coalesced int8
// row loads; the env's verdicts (game over = any bin negative) are segment
// ballots and the item / RNG / reward record is written by the env's bin-0
// lane.  HBM-bound: 2 * B * D + 4 + 4 + 4 + 1 bytes per env step.
#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {

template <int B, int D>
struct VShape {
  static constexpr int BPL = B > 64 ? B / 64 : 1;  // bins per lane
  static constexpr int LPE = B / BPL;               // lanes per env
  static constexpr int EPW = 64 / LPE;              // envs per wave
  static constexpr int BD = B * D;
};

// The step kernel's layout: XH_VENV_BPL (16) consecutive bins per lane
// (their bytes as aligned 32-bit words: 32 bytes at D = 2), so 64 / (B / 16)
// envs share a wave (16 at 64 bins).  With one lane per (env, bin) the step
// was issue-bound, not HBM-bound: every lane of an env draws the env's item
// (two engine draws and a double-precision canonical, register-only) and
// steps its stream with 64-bit modular multiplies, so the instruction count
// per byte falls with the bins a lane carries.  Round 6, 64 bins, 2-D, 1M
// envs: one env per wave 1.27 TB/s with the traffic at its algorithmic bytes
// (counters: 25% issuing, 40% issue stalls, 35% waiting on memory); 4 / 8 /
// 16 / 32 / 64 bins per lane 2.7 / 3.9 / 4.8 / 5.3 / 4.8 TB/s; at 32768 envs
// (launch-bound) 16 is the fastest (tools/env_ab.sh, profiles/r06j-k_*).
#ifndef XH_VENV_BPL
#define XH_VENV_BPL 16
#endif
template <int B, int D>
struct VStepShape {
  // bins per lane (contiguous; at most B)
  static constexpr int BPL = XH_VENV_BPL < B ? XH_VENV_BPL : B;
  static constexpr int NW = BPL * D / 4;   // 32-bit words per lane
  // the lane's words' alignment (the env row starts at env * B * D)
  static constexpr int LOWBIT = (4 * NW) & -(4 * NW);
  static constexpr int ALIGN = LOWBIT > 16 ? 16 : LOWBIT;
  static constexpr int LPE = B / BPL;      // lanes per env
  static constexpr int EPW = 64 / LPE;     // envs per wave
  static constexpr int BD = B * D;
};

// draw one item (get_item: bernoulli(0.4) over generate_canonical<double>)
__device__ __forceinline__ void venv_item(const EnvDesc &E, uint32_t &x,
                                          int8_t *ip) {
  const bool first = canonical(x) < E.p_a;
#pragma unroll
  for (int d = 0; d < 4; ++d)
    ip[d] = d < E.D ? (int8_t)(first ? E.item_a[d] : E.item_b[d]) : 0;
}

template <int B, int D>
__device__ __forceinline__ void venv_obs_row(const int8_t *bp, const int8_t *ip,
                                             float *o) {
#pragma unroll
  for (int d = 0; d < D; ++d) {
    o[d] = (float)bp[d] / (float)kCapacity;
    o[D + d] = (float)ip[d] / (float)kCapacity;
  }
}

// mode 0: environment::apply for every (masked) env -- bins[a] -= item; a new
// item (2 draws) unless that bin went negative; done[e] = game_over after it.
// mode 1: agent::step minus react -- skip the policy's draws, apply, reward =
// game_over ? 0 : 1, reset (2 draws) on game over, then the env's stream
// jumps over the other envs' draws of this step (reference order).
// Every global load is issued first and unconditionally (an out-of-range
// lane reads env 0's words; a masked or refused env's values are not used),
// so their latencies overlap: one HBM round trip before the arithmetic
// instead of three dependent ones (action -> item / bins -> stream state).
// XCD-aware block order: workgroups are dispatched round-robin over the 8
// XCDs (XCD = block index mod 8), each with its own L2; block b takes the
// env range of block (b mod 8) G / 8 + b / 8, so an XCD steps one contiguous
// run of envs and the 4-byte per-env records sharing a 128-byte line
// (action, item, stream state, reward) are fetched by one L2, not eight
__device__ __forceinline__ int xcd_block() {
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  return (G & 7) == 0 ? (b & 7) * (G >> 3) + (b >> 3) : b;
}

template <int B, int D>
__global__ __launch_bounds__(256) void venv_step_kernel(VenvArgs a) {
  using S = VStepShape<B, D>;
  const int lane = threadIdx.x & 63;
  const int wave = (xcd_block() * (int)blockDim.x + (int)threadIdx.x) >> 6;
  const int el = lane / S::LPE, li = lane % S::LPE;
  const int env = wave * S::EPW + el;
  const int seg0 = el * S::LPE;
  const bool in_range = env < a.N;
  const size_t ec = in_range ? (size_t)env : 0;
  int8_t *bp = a.bins + ec * S::BD;
  int8_t *ip = a.items + ec * 4;
  const int act_raw = a.action[ec];
  const bool masked_in = !a.mask || a.mask[ec];
  const unsigned itw = *reinterpret_cast<const unsigned *>(ip);
  uint32_t x = a.rng[ec];
  // this lane's bins li BPL .. li BPL + BPL - 1: NW words, byte k D + d =
  // bin k, dim d
  const uint32_t *wp = reinterpret_cast<const uint32_t *>(
      __builtin_assume_aligned(bp + li * S::BPL * D, S::ALIGN));
  uint32_t wv[S::NW];
#pragma unroll
  for (int q = 0; q < S::NW; ++q) wv[q] = wp[q];
  int v[S::BPL][D];
#pragma unroll
  for (int k = 0; k < S::BPL; ++k)
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int j = k * D + d;
      v[k][d] = (int)(signed char)((wv[j >> 2] >> (8 * (j & 3))) & 0xff);
    }

  const bool on = in_range && masked_in;
  int act = on ? act_raw : 0;
  if (on && (act < 0 || act >= B)) {  // refuse the env, flag the call
    if (li == 0) atomicOr(a.err, 1);
    act = -1;
  }
  const bool live = on && act >= 0;
  int item[D];
#pragma unroll
  for (int d = 0; d < D; ++d) item[d] = live ? (int)(signed char)((itw >> (8 * d)) & 0xff) : 0;
  int nb[S::BPL][D];
  int neg_any = 0, neg_chosen = 0;
#pragma unroll
  for (int k = 0; k < S::BPL; ++k) {
    const int bin = li * S::BPL + k;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int vv = live ? v[k][d] : 0;
      nb[k][d] = bin == act ? vv - item[d] : vv;
      neg_any |= nb[k][d] < 0;
      if (bin == act) neg_chosen |= nb[k][d] < 0;
    }
  }
  // segment verdicts (every lane of the env gets them)
  unsigned long long segmask = S::LPE == 64 ? ~0ull
                                            : ((1ull << S::LPE) - 1ull) << seg0;
  const bool over = (__ballot(neg_any) & segmask) != 0;
  const bool chosen_over = (__ballot(neg_chosen) & segmask) != 0;
  if (!live) {
    // an env not applied (masked out, or its action refused) reports no game
    // over for this call: DONE holds this call's verdicts only
    if (in_range && li == 0 && a.done) a.done[env] = 0;
    return;
  }
  if (a.mode == 1) x = mstd_mulmod(x, a.skip_mul);  // the policy's draws
  const bool reset = a.mode == 1 && over;
  {
    uint32_t ow[S::NW];
#pragma unroll
    for (int q = 0; q < S::NW; ++q) ow[q] = 0u;
#pragma unroll
    for (int k = 0; k < S::BPL; ++k)
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int j = k * D + d;
        ow[j >> 2] |= (uint32_t)((reset ? kCapacity : nb[k][d]) & 0xff) << (8 * (j & 3));
      }
    uint32_t *op = reinterpret_cast<uint32_t *>(
        __builtin_assume_aligned(bp + li * S::BPL * D, S::ALIGN));
#pragma unroll
    for (int q = 0; q < S::NW; ++q) op[q] = ow[q];
  }
  // every lane of the env draws the same item (redundant, register-only: no
  // cross-lane hand-off of the new item); the bin-0 lane writes the record
  int8_t nit[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) nit[d] = d < D ? (int8_t)item[d] : 0;
  if (!chosen_over) venv_item(a.env, x, nit);  // apply's get_item
  if (reset) venv_item(a.env, x, nit);         // reset's get_item
  if (a.mode == 1) x = mstd_mulmod(x, a.jump_mul);
  if (li == 0) {
    *reinterpret_cast<unsigned *>(ip) = (unsigned)(uint8_t)nit[0] |
                                        ((unsigned)(uint8_t)nit[1] << 8) |
                                        ((unsigned)(uint8_t)nit[2] << 16) |
                                        ((unsigned)(uint8_t)nit[3] << 24);
    if (a.mode == 1 && a.reward) a.reward[env] = over ? 0.0f : 1.0f;
    if (a.done) a.done[env] = (uint8_t)over;
    a.rng[env] = x;
  }
  if (a.obs) {  // observation::to_vector of the resulting state
#pragma unroll
    for (int k = 0; k < S::BPL; ++k) {
      const int bin = li * S::BPL + k;
      float *o = a.obs + ((size_t)env * B + bin) * 2 * D;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        o[d] = (float)(reset ? kCapacity : nb[k][d]) / (float)kCapacity;
        o[D + d] = (float)nit[d] / (float)kCapacity;
      }
    }
  }
}

// environment::reset for every (masked) env: bins at capacity, get_item.
template <int B, int D>
__global__ __launch_bounds__(256) void venv_reset_kernel(VenvArgs a) {
  using S = VShape<B, D>;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int el = lane / S::LPE, li = lane % S::LPE;
  const int env = wave * S::EPW + el;
  if (env >= a.N || (a.mask && !a.mask[env])) return;
  int8_t *bp = a.bins + (size_t)env * S::BD;
#pragma unroll
  for (int k = 0; k < S::BPL; ++k)
#pragma unroll
    for (int d = 0; d < D; ++d) bp[(k * 64 + li) * D + d] = (int8_t)kCapacity;
  if (li == 0) {
    uint32_t x = a.rng[env];
    venv_item(a.env, x, a.items + (size_t)env * 4);
    a.rng[env] = x;
  }
}

// observation::to_vector of every env: obs [N][B][2D] f32.
template <int B, int D>
__global__ __launch_bounds__(256) void venv_observe_kernel(VenvArgs a) {
  using S = VShape<B, D>;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int el = lane / S::LPE, li = lane % S::LPE;
  const int env = wave * S::EPW + el;
  if (env >= a.N) return;
  const int8_t *bp = a.bins + (size_t)env * S::BD;
  const int8_t *ip = a.items + (size_t)env * 4;
#pragma unroll
  for (int k = 0; k < S::BPL; ++k) {
    const int bin = k * 64 + li;
    venv_obs_row<B, D>(bp + bin * D, ip, a.obs + ((size_t)env * B + bin) * 2 * D);
  }
}

// Construction (bin_packing.h:50-52): env g (global) draws its item at engine
// position 2g (envs constructed one after another), then its stream moves to
// its first step position 2 Ng + k g (k = draws per env per step).
__global__ void venv_init_kernel(VenvArgs a, uint32_t x0, int env_offset,
                                 int n_global, int k) {
  const int BD = a.env.B * a.env.D;
  for (int env = blockIdx.x * blockDim.x + threadIdx.x; env < a.N;
       env += gridDim.x * blockDim.x) {
    const uint64_t g = (uint64_t)env_offset + env;
    uint32_t x = mstd_jump(x0, 2 * g);
    for (int i = 0; i < BD; ++i) a.bins[(size_t)env * BD + i] = (int8_t)kCapacity;
    venv_item(a.env, x, a.items + (size_t)env * 4);
    const uint64_t target = 2ull * n_global + (uint64_t)k * g;
    a.rng[env] = mstd_jump(x, target - (2 * g + 2));
  }
}

// ------------------------------------------------------------- launchers --
#define XH_VENV_SHAPES(X) \
  X(8, 1) X(8, 2) X(8, 3) X(16, 1) X(16, 2) X(16, 3) X(32, 1) X(32, 2)      \
  X(32, 3) X(64, 1) X(64, 2) X(64, 3) X(128, 1) X(128, 2) X(128, 3)

bool venv_shape_supported(int B, int D) {
#define X(XB, XD) if (B == XB && D == XD) return true;
  XH_VENV_SHAPES(X)
#undef X
  return false;
}

static dim3 venv_grid(int N, int B) {
  const int epw = B >= 64 ? 1 : 64 / B;
  const long waves = (N + epw - 1) / epw;
  return dim3((unsigned)((waves + 3) / 4));
}
// the step kernel's (VStepShape: 4 bins per lane)
static dim3 venv_step_grid(int N, int B) {
  const int epw = 64 / (B / (XH_VENV_BPL < B ? XH_VENV_BPL : B));
  const long waves = (N + epw - 1) / epw;
  return dim3((unsigned)((waves + 3) / 4));
}

hipError_t launch_venv(const VenvArgs &a, int op, hipStream_t s) {
  const int B = a.env.B, D = a.env.D;
  if (a.N <= 0) return hipSuccess;
#define X(XB, XD)                                                            \
  if (B == XB && D == XD) {                                                  \
    if (op == kVenvStep)                                                     \
      hipLaunchKernelGGL((venv_step_kernel<XB, XD>), venv_step_grid(a.N, B), \
                         dim3(256), 0, s, a);                                \
    else if (op == kVenvReset)                                               \
      hipLaunchKernelGGL((venv_reset_kernel<XB, XD>), venv_grid(a.N, B),     \
                         dim3(256), 0, s, a);                                \
    else                                                                     \
      hipLaunchKernelGGL((venv_observe_kernel<XB, XD>), venv_grid(a.N, B),   \
                         dim3(256), 0, s, a);                                \
    return hipGetLastError();                                                \
  }
  XH_VENV_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_venv_init(const VenvArgs &a, uint32_t x0, int env_offset,
                            int n_global, int k, hipStream_t s) {
  hipLaunchKernelGGL(venv_init_kernel, dim3((a.N + 255) / 256), dim3(256), 0, s,
                     a, x0, env_offset, n_global, k);
  return hipGetLastError();
}

}  // namespace xh
