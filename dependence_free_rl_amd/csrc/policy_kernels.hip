// policy_kernels.hip -- the per-bin policy on CDNA4 (gfx950):
//
//  * rollout_step_kernel: ONE kernel per environment step for all envs:
//      obs encode (from int8 state) -> conv1d_1 F0->H1 -> relu -> H1->H2 ->
//      relu -> H2->1 (MFMA f32 32x32x2) -> candidate-bin scores staged in LDS
//      -> softmax (no max shift, nn.h:382-392) -> categorical sample
//      (std::discrete_distribution over minstd_rand0, bit-exact) -> env apply /
//      reward / reset (bin_packing.h:53-106) -> trajectory record.
//  * policy_train_kernel: one PPO (or actor-critic) epoch over the batch:
//      forward, clipped-surrogate (rl.h:54-74) or softmax-log (rl.h:45-52)
//      loss gradient, softmax Jacobian backward (nn.h:393-417), Dense backward
//      (nn.h:149-186) with dW accumulated on chip; one gradient slab per
//      workgroup (reduced in slab order by reduce_sgd.hip: deterministic).
//
// Tiling (both kernels): a "group" is 64 rows = 64/B envs x B bins. Rows live
// on MFMA lanes (col index), features in accumulator registers, so the
// layer-1 accumulator feeds layer 2 as the B operand with no data movement
// (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand").
// W2 is staged once per workgroup in LDS (row stride H1+4: conflict-free
// ds_read_b128 A-operand reads).  Weight gradients contract over rows, so
// H1 and dL/dA2 go through LDS images (row stride +1) once per group.
#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

#include <cstdlib>

// Diagnostic builds only (make diag): extra XH_ABLATE bits in the 8-wave
// train kernel that drop whole phases (results are wrong by design).
#ifndef XH_DIAG_ABLATE
#define XH_DIAG_ABLATE 0
#endif
// Every ablation test folds to `false` in the product build, so a stray
// XH_ABLATE in the environment cannot change what the shipped kernels compute
// (the host refuses it too: xylo_hip.cpp do_learn).
#define XH_ABL(a, k) (XH_DIAG_ABLATE && ((a).ablate & (k)))
// Phase stamps (trace build, make variant VFLAGS=-DXH_DIAG_TRACE=1, run with
// XH_PHASE_TRACE=1): lane 0 of every wave of the first kTraceBlocks
// workgroups records the cycle counter at the 8-wave train kernel's phase
// boundaries for its first kTraceGroups groups.
#ifndef XH_DIAG_TRACE
#define XH_DIAG_TRACE 0
#endif
#if XH_DIAG_TRACE
#define XH_STAMP(a, gi, w, lane, slot)                                        \
  do {                                                                        \
    if ((a).trace && blockIdx.x < kTraceBlocks && (gi) < kTraceGroups &&      \
        (lane) == 0)                                                          \
      (a).trace[((blockIdx.x * kTraceGroups + (gi)) * 8 + (w)) * kTraceSlots + \
                (slot)] = clock64();                                          \
  } while (0)
#else
#define XH_STAMP(a, gi, w, lane, slot) \
  do {                                 \
  } while (0)
#endif
#define XH_STAMP4(a, gi, w, lane, slot) XH_STAMP(a, gi, w, lane, slot)
// Kernel span over all workgroups (trace build): the earliest start and the
// latest end of any workgroup, on the constant-rate wall clock.
#if XH_DIAG_TRACE
#define XH_SPAN(a, which)                                                     \
  do {                                                                        \
    if ((a).trace && threadIdx.x == 0) {                                      \
      unsigned long long *sp = reinterpret_cast<unsigned long long *>(        \
          (a).trace + kTraceBlocks * kTraceGroups * 8 * kTraceSlots);         \
      const unsigned long long tnow = (unsigned long long)wall_clock64();     \
      if ((which) == 0)                                                       \
        atomicMin(sp, tnow);                                                  \
      else if ((which) == 3)                                                  \
        atomicMax(sp + 1, tnow);                                              \
      if (blockIdx.x < 512) sp[2 + 4 * blockIdx.x + (which)] = tnow;          \
      if ((which) == 0 && blockIdx.x < 512) {                                 \
        unsigned hw, xc;                                                      \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));      \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xc));     \
        sp[2 + 2048 + 2 * blockIdx.x] = hw;                                   \
        sp[2 + 2048 + 2 * blockIdx.x + 1] = xc;                               \
      }                                                                       \
    }                                                                         \
  } while (0)
#else
#define XH_SPAN(a, which) \
  do {                    \
  } while (0)
#endif

namespace xh {
// 1 in the diagnostic builds (make diag / trace variants), 0 in the product
// library.
int diag_build() { return XH_DIAG_ABLATE || XH_DIAG_TRACE; }
}  // namespace xh

namespace xh {

template <int B_, int D_, int H1_, int H2_>
struct PShape {
  static constexpr int B = B_, D = D_, H1 = H1_, H2 = H2_;
  static constexpr int F0 = 2 * D;
  static constexpr int S1 = (F0 + 1) / 2;  // layer-1 MFMA k-steps
  static constexpr int NIT = H1 / 32, NOT = H2 / 32;
  static constexpr int G = B <= 64 ? 64 / B : 1;   // envs per group
  static constexpr int HG = B <= 64 ? 1 : B / 64;  // 64-row half-groups
  static constexpr int R = 64 * HG;                // rows per group
  static constexpr int BD = B * D;
  static constexpr int W2S = H1 + 4;           // LDS W2 image row stride
  static constexpr int HS = H1 + 1;            // LDS H1 image row stride
  static constexpr int AS = H2 + 1;            // LDS dA2 image row stride
  static constexpr int FJ = NOT >= 4 ? 2 : 1;  // fwd r-tiles per wave
  static constexpr int JW = (NOT * NIT + 3) / 4;  // dW2 tiles per wave
  static constexpr int JH = (2 * NIT + 3) / 4;    // dH1 r-tiles per wave
  // 4-wave train kernel: workgroups per CU it is compiled for.  The 1-D
  // [64,64] shape (config 2) fits 256 VGPRs without scratch, so two
  // workgroups share a CU and one's barrier / softmax phases overlap the
  // other's MFMAs; the wider shapes need the full register file (spills
  // measured at 2).
  static constexpr int TOCC = (H1 <= 64 && H2 <= 64 && D == 1) ? 2 : 1;
  static_assert(B == 8 || B == 16 || B == 32 || B == 64 || B == 128, "B");
  static_assert(NIT == 1 || NIT == 2 || NIT == 4, "H1 in {32,64,128}");
  static_assert(NOT == 1 || NOT == 2 || NOT == 4, "H2 in {32,64,128}");
  static_assert(D >= 1 && D <= 3, "D");
  // LDS carve (floats), every region 16-byte aligned.
  static constexpr int r4(int x) { return (x + 3) & ~3; }
  static constexpr int L_W2 = 0;
  static constexpr int L_W1 = L_W2 + H2 * W2S;
  static constexpr int L_B1 = L_W1 + r4(H1 * F0);
  static constexpr int L_B2 = L_B1 + H1;
  static constexpr int L_W3 = L_B2 + H2;
  static constexpr int L_B3 = L_W3 + H2;
  static constexpr int L_Z = L_B3 + 4;
  static constexpr int L_ROLLOUT_END = L_Z + NOT * R;
  static constexpr int L_H1 = L_ROLLOUT_END;
  static constexpr int L_DA2 = L_H1 + r4(64 * HS);
  static constexpr int L_TRAIN_END = L_DA2 + r4(64 * AS);
  // 8-wave kernel: transposed images [feature][row] (row stride 64+4 floats:
  // conflict-free ds_read_b128 along rows)
  static constexpr int TS = 68;
  static constexpr int L_H1T = L_ROLLOUT_END;
  static constexpr int L_DAT = L_H1T + H1 * TS;
  // the layer-1 biases with the item's contribution folded in, for the two
  // item-table entries (8-wave kernel, one env per group)
  static constexpr int L_B1F = L_DAT + H2 * TS;
  static constexpr int L_TRAIN8_END = L_B1F + 2 * H1;
  // end-of-kernel reduction scratch (aliases the H1 / dA2 images)
  static constexpr int RED = H1 * F0 + H1 + 2 * H2 + 1;
  static_assert(4 * RED <= 64 * HS + 64 * AS, "scratch fits");
};

// Stage the small per-bin parameters (all of layer 1/3, biases) and the W2
// image into LDS.
template <class S>
__device__ __forceinline__ void stage_params(const float *__restrict__ P,
                                             float *lds) {
  const PolicyLayout L{S::F0, S::H1, S::H2};
  const int tid = threadIdx.x;
  for (int i = tid; i < S::H2 * S::H1; i += blockDim.x) {
    const int o = i / S::H1, k = i - o * S::H1;
    lds[S::L_W2 + o * S::W2S + k] = P[L.oW2() + i];
  }
  for (int i = tid; i < S::H1 * S::F0; i += blockDim.x)
    lds[S::L_W1 + i] = P[L.oW1() + i];
  for (int i = tid; i < S::H1; i += blockDim.x) lds[S::L_B1 + i] = P[L.ob1() + i];
  for (int i = tid; i < S::H2; i += blockDim.x) {
    lds[S::L_B2 + i] = P[L.ob2() + i];
    lds[S::L_W3 + i] = P[L.ow3() + i];
  }
  if (tid == 0) lds[S::L_B3] = P[L.ob3()];
}

// The raw int8 state of the two rows a lane carries (rows rt*32 + lane&31 of
// a group), fetched one group ahead so the global-load latency overlaps the
// previous group's MFMA work (1 wave per SIMD in the train kernel).
template <class S>
struct RowRaw {
  int bv[2][S::D];
  int iv[2][S::D];
};

template <class S>
__device__ __forceinline__ void fetch_rows(const Batch &b, int slot, int e0,
                                           RowRaw<S> &rr) {
  const int lr = threadIdx.x & 31;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int r = rt * 32 + lr;
    const size_t env = (size_t)slot * b.N + e0 + r / S::B;
    const int8_t *bp = b.bins + env * S::BD + (r % S::B) * S::D;
    const int8_t *ip = b.items + env * 4;
#pragma unroll
    for (int d = 0; d < S::D; ++d) {
      rr.bv[rt][d] = bp[d];
      rr.iv[rt][d] = ip[d];
    }
  }
}

// Observation feature f of a row (observation::to_vector, bin_packing.h:31-40):
// [bin dims / 8, item dims / 8].  f may be runtime (lane-half dependent).
template <class S>
__device__ __forceinline__ float row_feature(const RowRaw<S> &rr, int rt,
                                             int f) {
  int v = 0;
#pragma unroll
  for (int d = 0; d < S::D; ++d) {
    if (f == d) v = rr.bv[rt][d];
    if (f == S::D + d) v = rr.iv[rt][d];
  }
  return f < S::F0 ? (float)v / (float)kCapacity : 0.0f;
}

// relu as max(bits, 0) on the int view: one v_max_i32 (x > 0 ? x : 0 costs a
// NaN-canonicalise + v_max_f32); identical for every non-NaN x, -0 -> +0.
__device__ __forceinline__ float relu(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}

// 4 consecutive LDS floats (16-byte aligned) -> bias / weight values of
// accumulator registers 4q..4q+3 (acc_row = 8q + 4h + {0..3}).
__device__ __forceinline__ float4 lds4(const float *p) {
  return *reinterpret_cast<const float4 *>(p);
}

// Layer 1 (F0 -> H1) + bias + relu for the 64 rows of a group, all H1 tiles.
// h1[it][rt]: col = row rt*32 + (lane&31), acc row = feature it*32+acc_row.
template <class S>
__device__ __forceinline__ void layer1(const RowRaw<S> &rr, const float *lds,
                                       f32x16 (&h1)[S::NIT][2]) {
  const int lane = threadIdx.x & 63, lr = lane & 31, h = lane >> 5;
  float xb[2][S::S1];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int s = 0; s < S::S1; ++s) xb[rt][s] = row_feature<S>(rr, rt, 2 * s + h);
#pragma unroll
  for (int it = 0; it < S::NIT; ++it) {
    float wa[S::S1];
#pragma unroll
    for (int s = 0; s < S::S1; ++s) {
      const int k = 2 * s + h;
      wa[s] = k < S::F0 ? lds[S::L_W1 + (it * 32 + lr) * S::F0 + k] : 0.0f;
    }
    f32x16 acc0 = zero16(), acc1 = zero16();
#pragma unroll
    for (int s = 0; s < S::S1; ++s) {
      acc0 = mfma32(wa[s], xb[0][s], acc0);
      acc1 = mfma32(wa[s], xb[1][s], acc1);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 bb = lds4(lds + S::L_B1 + it * 32 + 8 * q + 4 * h);
      const float bq[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float v0 = acc0[4 * q + u] + bq[u];
        const float v1 = acc1[4 * q + u] + bq[u];
        acc0[4 * q + u] = relu(v0);
        acc1[4 * q + u] = relu(v1);
      }
    }
    h1[it][0] = acc0;
    h1[it][1] = acc1;
  }
}

// Layer 2 pre-activations (+ bias) of output tile o2t for NR r-tiles
// rt0..rt0+NR-1: A = W2 rows from the LDS image (4 k-steps per ds_read_b128,
// shared by the NR independent accumulation chains), B = h1 registers.
template <class S, int NR>
__device__ __forceinline__ void layer2(const float *lds,
                                       const f32x16 (&h1)[S::NIT][2], int o2t,
                                       int rt0, f32x16 (&acc)[NR]) {
  const int lane = threadIdx.x & 63, lr = lane & 31, h = lane >> 5;
  const float *wrow = lds + S::L_W2 + (o2t * 32 + lr) * S::W2S + 4 * h;
#pragma unroll
  for (int r = 0; r < NR; ++r) acc[r] = zero16();
#pragma unroll
  for (int it = 0; it < S::NIT; ++it) {
    f32x16 hb[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r)  // compile-time index when NR == 2
      hb[r] = NR == 2 ? h1[it][r] : (rt0 == 0 ? h1[it][0] : h1[it][1]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 a4 = lds4(wrow + it * 32 + 8 * q);
      const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int r = 0; r < NR; ++r) acc[r] = mfma32(av[u], hb[r][4 * q + u], acc[r]);
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 bb = lds4(lds + S::L_B2 + o2t * 32 + 8 * q + 4 * h);
    const float bq[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[r][4 * q + u] += bq[u];
  }
}

// Partial logit over this tile's 32 H2 units for row rt*32 + (lane&31).
// kSwap: the lane-half exchange as v_permlane32_swap (a volatile asm, which
// the scheduler cannot move MFMAs across: only for the train kernel's
// serial logit phase; inside the rollout's MFMA streams the ds_bpermute
// keeps the schedule, measured 2.44 vs 2.59 ms per iteration).  Both give
// the same bits (zp_lo + zp_hi in either half).
template <class S, bool kSwap = false>
__device__ __forceinline__ float logit_part(const float *lds, const f32x16 &pre,
                                            int o2t) {
  const int h = (threadIdx.x & 63) >> 5;
  float zp = 0.0f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 ww = lds4(lds + S::L_W3 + o2t * 32 + 8 * q + 4 * h);
    const float wq[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float v = relu(pre[4 * q + u]);
      zp += v * wq[u];
    }
  }
  return zp + (kSwap ? half_swap(zp) : __shfl_xor(zp, 32, kWave));
}

// Softmax of the candidate-bin scores z (lane = row = bin of env `env`,
// whose B rows sit in lanes seg0 ..), the categorical sample (or the forced
// action), and the env transition of slot t into slot t+1 (rl.h:325-349,
// bin_packing.h:53-79).  `cur` holds this lane's raw row (rows lr / 32+lr).
// x is the env's minstd state (the same in every lane of the segment; the
// caller loads and stores it), `last` marks the launch's last step (the
// optional logits / probabilities outputs).  Out: nbv = this lane's bin in
// slot t+1, first = the env's next item is item_a.
template <class S>
__device__ __forceinline__ void sample_step_x(const RolloutArgs &a, int t, bool last,
                                              float z, int env, int seg0, int bin,
                                              const RowRaw<S> &cur, uint32_t &x,
                                              int (&nbv)[S::D], bool &first) {
  constexpr int B = S::B;
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int N = a.b.N;
  const float ex = expf(z);
  const float sum = seg_sum<B>(ex);
  const float p = ex / sum;
  if (last && a.logits_out) a.logits_out[(size_t)env * B + bin] = z;
  if (last && a.probs_out) a.probs_out[(size_t)env * B + bin] = p;
  if (a.qold_out) a.qold_out[((size_t)t * N + env) * B + bin] = p;

  int choice;
  if (a.forced) {
    choice = a.forced[(size_t)t * N + env];
    (void)canonical(x);  // the sampler's two engine draws
  } else {
    choice = sample_discrete<B>(p, lane, canonical(x));
  }
  const float pold = wave_shfl(p, seg0 + choice);

  // this lane's row (= lane) is row (h ? 32 : 0) + lr of the prefetch
  int nb[S::D];
  int neg = 0;
#pragma unroll
  for (int d = 0; d < S::D; ++d) {
    const int bv = h ? cur.bv[1][d] : cur.bv[0][d];
    const int iv = h ? cur.iv[1][d] : cur.iv[0][d];
    nb[d] = bin == choice ? bv - iv : bv;
    neg |= nb[d] < 0;
  }
  const int done = __shfl(neg, seg0 + choice, kWave);
  // apply -> get_item, or game over -> reset -> get_item: 2 draws either way
  first = canonical(x) < a.env.p_a;
  int8_t *ob = a.b.bins + ((size_t)(t + 1) * N + env) * S::BD + bin * S::D;
#pragma unroll
  for (int d = 0; d < S::D; ++d) {
    nbv[d] = done ? kCapacity : nb[d];
    ob[d] = (int8_t)nbv[d];
  }
  if (bin == 0) {
    int8_t *oi = a.b.items + ((size_t)(t + 1) * N + env) * 4;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      oi[d] = d < S::D ? (int8_t)(first ? a.env.item_a[d] : a.env.item_b[d]) : 0;
    a.b.action[(size_t)t * N + env] = choice;
    a.b.pold[(size_t)t * N + env] = pold;
    a.b.done[(size_t)t * N + env] = (uint8_t)done;
  }
}

// One step (slot a.t) of env `env`: sample_step_x with the stream state read
// from and written back to a.b.rng (jumped after step T-1).
template <class S>
__device__ __forceinline__ void sample_step(const RolloutArgs &a, float z,
                                            int env, int seg0, int bin,
                                            const RowRaw<S> &cur) {
  uint32_t x = a.b.rng[env];
  int nbv[S::D];
  bool first;
  sample_step_x<S>(a, a.t, true, z, env, seg0, bin, cur, x, nbv, first);
  if (bin == 0) a.b.rng[env] = (a.t == a.b.T - 1) ? mstd_mulmod(x, a.jump_mul) : x;
}

// =========================================================== rollout step ==
template <class S>
__global__ __launch_bounds__(256, 2) void rollout_step_kernel(RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  stage_params<S>(a.params, lds);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 31;
  const int N = a.b.N, t = a.t;
  const int ngroups = N / S::G;
  // forward job of this wave: output tile o2t, r-tiles rt0 .. rt0+FJ-1
  const int o2t = w % S::NOT;
  const int rt0 = S::NOT >= 4 ? 0 : w / S::NOT;
  const bool fwd_active = (w / S::NOT) * S::FJ < 2;

  RowRaw<S> cur, nxt;
  if ((int)blockIdx.x < ngroups) fetch_rows<S>(a.b, t, blockIdx.x * S::G, cur);
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int e0 = g * S::G;
    const int gn = g + gridDim.x;
    if (gn < ngroups) fetch_rows<S>(a.b, t, gn * S::G, nxt);
    {
      f32x16 h1[S::NIT][2];
      layer1<S>(cur, lds, h1);
      if (fwd_active) {
        f32x16 pre[S::FJ];
        layer2<S, S::FJ>(lds, h1, o2t, rt0, pre);
#pragma unroll
        for (int q = 0; q < S::FJ; ++q) {
          const float zp = logit_part<S>(lds, pre[q], o2t);
          if (lane < 32) lds[S::L_Z + o2t * 64 + (rt0 + q) * 32 + lr] = zp;
        }
      }
    }
    __syncthreads();
    if (w == 0) {
      // ---- candidate-bin scores -> softmax -> sample -> env step (lane=row)
      constexpr int B = S::B;
      const int e = lane / B, bin = lane % B, env = e0 + e, seg0 = e * B;
      float zs = 0.0f;
#pragma unroll
      for (int o = 0; o < S::NOT; ++o) zs += lds[S::L_Z + o * 64 + lane];
      const float z = zs + lds[S::L_B3];
      sample_step<S>(a, z, env, seg0, bin, cur);
    }
    __syncthreads();
    cur = nxt;
  }
}

// Partial logits of one 64-row half-group for the wave-per-env rollouts,
// one 32-row r-tile at a time (XH_V_RPASS): the wave keeps all four H2
// tiles' accumulators of the r-tile (four independent MFMA chains) and
// computes each layer-1 tile once per r-tile instead of once per H2 tile
// (config 3: 576 -> 528 MFMAs per env; config 5: 1216 -> 1072).  Every
// sum runs in the order of the tile-major loop (layer 1 over k-steps, + bias,
// relu; layer 2 over it, q, u; + bias; the logit over o2t), so logits are
// bit-identical.  zl[rt]: the partial logit of row rt*32 + (lane & 31).
// Measured (tools/gpu_ab_vars.sh): config 3 rollout 2.44 -> 2.19 ms per
// iteration at 12 waves per workgroup (3 per SIMD; all four tiles' chains
// at 4 per SIMD spill at 128 VGPRs, and without the scheduling barriers the
// operand reads of all four tiles are hoisted: 428 B of spills); config 5
// 5.09 -> 4.83 ms the same way, 4.63 ms in two-tile passes at 4 per SIMD.
#ifndef XH_V_RPASS
#define XH_V_RPASS 1
#endif
// waves per workgroup of the wave-per-env rollouts (one workgroup of 12 per
// CU = 3 waves per SIMD with 168 VGPRs: the r-tile pass keeps four H2 tiles'
// accumulators; 8 = two workgroups per CU, 4 waves per SIMD, 128 VGPRs)
// H2 tiles per pass of the r-tile pass, per kernel: 4 = all four (layer 1
// once per r-tile, 12 waves per workgroup = 3 per SIMD), 2 = two passes
// (layer 1 twice, half the accumulators: 8 waves = 4 per SIMD at 128
// VGPRs).  Measured: 64 bins 2.19 ms (4) vs 2.28 ms (2) per iteration; 128
// bins 4.81 ms (4) vs 4.63 ms (2).
#ifndef XH_V_RTILES64
#define XH_V_RTILES64 4
#endif
#ifndef XH_V_RTILES128
#define XH_V_RTILES128 2
#endif
constexpr int roll_waves(int tiles) { return XH_V_RPASS && tiles == 4 ? 12 : 8; }
constexpr int roll_occ(int waves) { return waves == 8 ? 4 : (waves == 12 ? 3 : 2); }
constexpr int kRollWaves64 = roll_waves(XH_V_RTILES64);
constexpr int kRollWaves128 = roll_waves(XH_V_RTILES128);
#ifndef XH_V_RSB
#define XH_V_RSB 1
#endif
template <class S, int OT>
__device__ __forceinline__ void wave_logits_rpass(const float *lds,
                                                  const RowRaw<S> &cur,
                                                  float (&zl)[2]) {
  const int lane = threadIdx.x & 63, lr = lane & 31, h = lane >> 5;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    float xb[S::S1];
#pragma unroll
    for (int s = 0; s < S::S1; ++s) xb[s] = row_feature<S>(cur, rt, 2 * s + h);
    float z = 0.0f;
#pragma unroll 1
    for (int op = 0; op < 4 / OT; ++op) {
    f32x16 pre[OT];
#pragma unroll
    for (int o = 0; o < OT; ++o) pre[o] = zero16();
#pragma unroll 1
    for (int it = 0; it < 4; ++it) {
      f32x16 t1 = zero16();
#pragma unroll
      for (int s = 0; s < S::S1; ++s) {
        const int k = 2 * s + h;
        const float wa = k < S::F0 ? lds[S::L_W1 + (it * 32 + lr) * S::F0 + k] : 0.0f;
        t1 = mfma32(wa, xb[s], t1);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bb = lds4(lds + S::L_B1 + it * 32 + 8 * q + 4 * h);
        const float bq[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) t1[4 * q + u] = relu(t1[4 * q + u] + bq[u]);
      }
#pragma unroll
      for (int oo = 0; oo < OT; ++oo) {
        const int o = op * OT + oo;
        const float *wrow = lds + S::L_W2 + (o * 32 + lr) * S::W2S + 4 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 a4 = lds4(wrow + it * 32 + 8 * q);
          const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) pre[oo] = mfma32(av[u], t1[4 * q + u], pre[oo]);
        }
        // keep the scheduler from hoisting every tile's operand reads
        if (XH_V_RSB) __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int oo = 0; oo < OT; ++oo) {
      const int o = op * OT + oo;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bb = lds4(lds + S::L_B2 + o * 32 + 8 * q + 4 * h);
        const float bq[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) pre[oo][4 * q + u] += bq[u];
      }
      z += logit_part<S>(lds, pre[oo], o);
    }
    }
    if (rt == 0)
      zl[0] = z;
    else
      zl[1] = z;
  }
}

// ================================================ rollout step, wave per env ==
// B = 64, [128,128] (config 3): one wave per env.  The wave runs all four H2
// tiles itself (layer 1 recomputed per tile, as each of rollout_step_kernel's
// four waves does), keeps the partial logits in registers and samples its own
// env, so no barrier separates the forward from the sampler and, at four
// waves per SIMD, one wave's softmax / double-precision sampling / env update
// issues beside the other waves' MFMAs.  Every operation and its order match
// rollout_step_kernel (layer1, layer2, logit_part, the o-ordered logit sum),
// so logits, probabilities and actions are bit-identical.
template <class S>
__global__ __launch_bounds__(64 * kRollWaves64, roll_occ(kRollWaves64)) void rollout_wave_kernel(RolloutArgs a) {
  static_assert(S::B == 64 && S::NIT == 4 && S::NOT == 4, "wave rollout: B=64, [128,128]");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  stage_params<S>(a.params, lds);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 31,
            h = lane >> 5;
  const int wpb = blockDim.x >> 6;
  for (int env = blockIdx.x * wpb + w; env < a.b.N; env += gridDim.x * wpb) {
    RowRaw<S> cur;
    fetch_rows<S>(a.b, a.t, env, cur);
    float xb[2][S::S1];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int s = 0; s < S::S1; ++s) xb[rt][s] = row_feature<S>(cur, rt, 2 * s + h);
    float zl[2] = {0.0f, 0.0f};  // partial logit sums of rows lr / 32 + lr
    if (XH_V_RPASS) wave_logits_rpass<S, XH_V_RTILES64>(lds, cur, zl);
#pragma unroll 1
    for (int o2t = 0; o2t < (XH_V_RPASS ? 0 : 4); ++o2t) {
      const float *wrow = lds + S::L_W2 + (o2t * 32 + lr) * S::W2S + 4 * h;
      f32x16 pre[2];
      pre[0] = zero16();
      pre[1] = zero16();
#pragma unroll 1
      for (int it = 0; it < 4; ++it) {
        // layer-1 tile it, exactly as layer1(): chain, + bias, relu
        f32x16 t1[2];
        t1[0] = zero16();
        t1[1] = zero16();
#pragma unroll
        for (int s = 0; s < S::S1; ++s) {
          const int k = 2 * s + h;
          const float wa = k < S::F0 ? lds[S::L_W1 + (it * 32 + lr) * S::F0 + k] : 0.0f;
          t1[0] = mfma32(wa, xb[0][s], t1[0]);
          t1[1] = mfma32(wa, xb[1][s], t1[1]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 bb = lds4(lds + S::L_B1 + it * 32 + 8 * q + 4 * h);
          const float bq[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            t1[0][4 * q + u] = relu(t1[0][4 * q + u] + bq[u]);
            t1[1][4 * q + u] = relu(t1[1][4 * q + u] + bq[u]);
          }
        }
        // layer 2 k-steps of tile it, exactly as layer2<S, 2>()
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 a4 = lds4(wrow + it * 32 + 8 * q);
          const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            pre[0] = mfma32(av[u], t1[0][4 * q + u], pre[0]);
            pre[1] = mfma32(av[u], t1[1][4 * q + u], pre[1]);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bb = lds4(lds + S::L_B2 + o2t * 32 + 8 * q + 4 * h);
        const float bq[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          pre[0][4 * q + u] += bq[u];
          pre[1][4 * q + u] += bq[u];
        }
      }
      zl[0] += logit_part<S>(lds, pre[0], o2t);
      zl[1] += logit_part<S>(lds, pre[1], o2t);
    }
    // lane = row = bin: rows 0..31 in lane half 0, 32..63 in half 1
    const float z = (h ? zl[1] : zl[0]) + lds[S::L_B3];
    sample_step<S>(a, z, env, 0, lane, cur);
  }
}

// ============================== rollout step, wave per env, f16 pairs ==
// The wave-per-group rollout of the [128,128] and [64,64] shapes with layer 2 on the f16
// matrix cores at f32-class accuracy (xh_split.h, f16 pairs: W2 and H1 each
// scaled by a power of two chosen per launch -- max|W2|, and the bound
// |H1[r][i]| <= sum_k |W1[i][k]| + |b1[i]| since every observation feature
// is in [-1, 1] -- and split exactly into two f16 parts; three f16 products
// per K slice).  Layer 1 (f32 MFMA, the same chain, bias and relu as
// rollout_wave_kernel) leaves H1 tile `it` of an r-tile in accumulator
// registers (lane = row, register j = feature acc_row(j, h)); its registers
// 8s .. 8s+7, scaled and split, are directly the B operand of K-slice s of
// the 32x32x16 MFMA, whose k order is then feature it*32 + 16s + 8(e>>2) +
// 4h + (e&3) for element e of lane half h.  W2 is staged with the columns
// of every 16-block permuted to that order (bits 2 and 3 of the column
// swapped), so each A fragment is one ds_read_b128 of the swizzled image.
// Layer 1 is staged times S_H (weights and bias: its output is S_H H1
// exactly), b2 times S_W S_H as layer 2's C input and w3 divided by it, so
// the partial logits take the same roundings as unscaled values; both
// biases enter as the MFMA chains' C inputs.  The logits differ from rollout_wave_kernel's in the
// last places (f32-class: tests/test_gpu_scale.py); the sampler, the env
// step and everything after are the same code.
// Layer 1 runs its k-steps over the D bin features only: the item (an
// item-table entry in every slot these kernels see, RolloutArgs::wide
// otherwise) is folded into a per-entry bias, (b1 + W1_item . item / 8) S_H,
// as in the train kernels -- D = 2: one f32 MFMA per tile instead of two,
// D = 3: two instead of three.
// LDS (bytes): two W2 part images [o][permuted i] (H2 rows of 256 bytes: 64
// KB at [128,128]), then f32 W1 [H1][F0], b1, b2 S_W S_H, w3 / (S_W S_H), b3,
// S_H, the scale reduction, the two folded biases [2][H1].
template <class S>
struct RollSplitLds {
  static constexpr int W2 = 0;
  static constexpr int F = 2 * S::H2 * kImgRow;
  static constexpr int W1 = 0, B1 = S::H1 * S::F0, B2 = B1 + S::H1, W3 = B2 + S::H2,
                       B3 = W3 + S::H2, SH = B3 + 1, SC = B3 + 4, B1F = SC + 2 * 16;
  static constexpr int S1F = (S::D + 1) / 2;  // layer-1 k-steps over the bins
  static constexpr size_t bytes = F + sizeof(float) * (B1F + 2 * S::H1);
};

// Stage the f16-pair W2 images (columns permuted, see above) and the small
// parameters of the split rollouts; every thread of the block calls it (it
// synchronises the block).
template <class S>
__device__ __forceinline__ void stage_split_rollout(const float *__restrict__ P,
                                                    const EnvDesc &env, char *lds) {
  using L = RollSplitLds<S>;
  float *lf = reinterpret_cast<float *>(lds + L::F);
  const PolicyLayout PL{S::F0, S::H1, S::H2};
  // the scales: max|W2| and the H1 bound, reduced over the block
  float mw = 0.0f, mh = 0.0f;
  for (int e = threadIdx.x; e < S::H2 * S::H1; e += blockDim.x)
    mw = fmaxf(mw, fabsf(P[PL.oW2() + e]));
  for (int i = threadIdx.x; i < S::H1; i += blockDim.x) {
    float v = fabsf(P[PL.ob1() + i]);
    for (int k = 0; k < S::F0; ++k) v += fabsf(P[PL.oW1() + i * S::F0 + k]);
    mh = fmaxf(mh, v);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    mw = fmaxf(mw, __shfl_xor(mw, o, kWave));
    mh = fmaxf(mh, __shfl_xor(mh, o, kWave));
  }
  const int nw = blockDim.x >> 6, wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    lf[L::SC + wv] = mw;
    lf[L::SC + 16 + wv] = mh;
  }
  __syncthreads();
  float MW = 0.0f, MH = 0.0f;
  for (int v = 0; v < nw; ++v) {
    MW = fmaxf(MW, lf[L::SC + v]);
    MH = fmaxf(MH, lf[L::SC + 16 + v]);
  }
  const float SW = f16_scale_for(MW), SH = f16_scale_for(MH), S2 = SW * SH;
  for (int e = threadIdx.x; e < S::H2 * S::H1; e += blockDim.x) {
    const int o = e / S::H1, i = e % S::H1;
    // logical column i -> its slot: bits 2 and 3 swapped within the 16-block
    const int c = (i & ~12) | ((i & 4) << 1) | ((i & 8) >> 1);
    _Float16 x0, x1;
    split2h(P[PL.oW2() + e] * SW, x0, x1);
    const int off = img_off(o, c >> 3) + 2 * (c & 7);
    *reinterpret_cast<_Float16 *>(lds + L::W2 + off) = x0;
    *reinterpret_cast<_Float16 *>(lds + L::W2 + S::H2 * kImgRow + off) = x1;
  }
  // layer 1 staged times S_H (its output is H1 S_H exactly: a power of two),
  // b2 times S_W S_H (layer 2's C input), w3 divided by it
  for (int i = threadIdx.x; i < S::H1 * S::F0; i += blockDim.x)
    lf[L::W1 + i] = P[PL.oW1() + i] * SH;
  for (int i = threadIdx.x; i < S::H1; i += blockDim.x) {
    lf[L::B1 + i] = P[PL.ob1() + i] * SH;
    lf[L::B2 + i] = P[PL.ob2() + i] * S2;
    lf[L::W3 + i] = P[PL.ow3() + i] * (1.0f / S2);
    float ba = P[PL.ob1() + i], bb = ba;
#pragma unroll
    for (int d = 0; d < S::D; ++d) {
      const float wv = P[PL.oW1() + i * S::F0 + S::D + d];
      ba += wv * ((float)env.item_a[d] / (float)kCapacity);
      bb += wv * ((float)env.item_b[d] / (float)kCapacity);
    }
    lf[L::B1F + i] = ba * SH;
    lf[L::B1F + S::H1 + i] = bb * SH;
  }
  if (threadIdx.x == 0) {
    lf[L::B3] = P[PL.ob3()];
    lf[L::SH] = SH;
  }
}

// Partial logits (without b3) of the two r-tiles of `cur` (64 rows) by the
// f16-pair layer 2: zl[rt] = the logit sum of row rt*32 + (lane & 31).
// b1r[rt]: the folded layer-1 bias (LDS, x S_H) of r-tile rt's item.
template <class S>
__device__ __forceinline__ void wave_logits_split(const char *lds,
                                                  const RowRaw<S> &cur,
                                                  const float *const (&b1r)[2],
                                                  float (&zl)[2]) {
  using L = RollSplitLds<S>;
  const float *lf = reinterpret_cast<const float *>(lds + L::F);
  const int lane = threadIdx.x & 63, lr = lane & 31, h = lane >> 5;
  const char *w2i[2] = {lds + L::W2, lds + L::W2 + S::H2 * kImgRow};
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    // the bin features only (feature 2 s1 + h < D; the item is in the bias)
    float xb[L::S1F];
#pragma unroll
    for (int s1 = 0; s1 < L::S1F; ++s1) {
      const int f = 2 * s1 + h;
      xb[s1] = f < S::D ? row_feature<S>(cur, rt, f) : 0.0f;
    }
    // layer 2's accumulators start at b2 S_W S_H (C layout: register 4q + u
    // = feature ot*32 + 8q + 4h + u)
    f32x16s pre[S::NOT];
#pragma unroll
    for (int ot = 0; ot < S::NOT; ++ot)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bb = *reinterpret_cast<const float4 *>(lf + L::B2 + ot * 32 + 8 * q + 4 * h);
        pre[ot][4 * q + 0] = bb.x;
        pre[ot][4 * q + 1] = bb.y;
        pre[ot][4 * q + 2] = bb.z;
        pre[ot][4 * q + 3] = bb.w;
      }
    // (fully unrolled: the next tile's layer 1 and split schedule beside this
    // tile's layer-2 MFMAs; 0.75 -> 0.72 ms per config-3 iteration)
#pragma unroll
    for (int it = 0; it < S::NIT; ++it) {
      // layer-1 tile it, times S_H: the bias as the chain's C input, relu
      f32x16 t1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bb = *reinterpret_cast<const float4 *>(b1r[rt] + it * 32 + 8 * q + 4 * h);
        t1[4 * q + 0] = bb.x;
        t1[4 * q + 1] = bb.y;
        t1[4 * q + 2] = bb.z;
        t1[4 * q + 3] = bb.w;
      }
#pragma unroll
      for (int s1 = 0; s1 < L::S1F; ++s1) {
        const int k = 2 * s1 + h;
        const float wa = k < S::D ? lf[L::W1 + (it * 32 + lr) * S::F0 + k] : 0.0f;
        t1 = mfma32(wa, xb[s1], t1);
      }
      f16x8 bfr[2][2];
      {
        typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
        u32x4_t hb[2], lb[2];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          unsigned h2, l2;
          split2h_x2(relu(t1[2 * jj]), relu(t1[2 * jj + 1]), h2, l2);
          hb[jj >> 2][jj & 3] = h2;
          lb[jj >> 2][jj & 3] = l2;
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bfr[s][0] = __builtin_bit_cast(f16x8, hb[s]);
          bfr[s][1] = __builtin_bit_cast(f16x8, lb[s]);
        }
      }
#pragma unroll
      for (int ot = 0; ot < S::NOT; ++ot) {
        const int rb = row_base(ot * 32 + lr, h);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          f16x8 af[2];
#pragma unroll
          for (int p = 0; p < 2; ++p)
            af[p] = __builtin_bit_cast(f16x8, ld_row(w2i[p], rb, 2 * it + s));
          // the three f16 products, small terms first
          pre[ot] = mfma_f16(af[1], bfr[s][0], pre[ot]);
          pre[ot] = mfma_f16(af[0], bfr[s][1], pre[ot]);
          pre[ot] = mfma_f16(af[0], bfr[s][0], pre[ot]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    float z = 0.0f;
#pragma unroll
    for (int ot = 0; ot < S::NOT; ++ot) {
      float zp = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 ww = *reinterpret_cast<const float4 *>(lf + L::W3 + ot * 32 + 8 * q + 4 * h);
        const float wq[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) zp = fmaf(relu(pre[ot][4 * q + u]), wq[u], zp);
      }
      z += zp + __shfl_xor(zp, 32, kWave);
    }
    zl[rt] = z;
  }
}

// The split rollout over whole row groups of 64 (one env of 64 bins, or two
// of 32: G = 64 / B envs, env e0 + h in lane half h), WAVES waves per
// workgroup, each wave stepping its group through slots a.t .. a.t +
// a.nsteps - 1 in one launch: slot t+1's rows come from the sampler's
// registers (this lane's row, the partner half's by a lane swap), the minstd
// state stays in a register and is stored once, after the launch's last
// step.  Per step the same operations as one launch per step, so states,
// actions and logits are bit-identical to stepping slot by slot.
template <class S>
constexpr int roll_split_waves() { return S::B == 64 ? kRollWaves64 : 4; }
template <class S>
constexpr int roll_split_occ() { return S::B == 64 ? roll_occ(kRollWaves64) : 2; }

template <class S>
__global__ __launch_bounds__(64 * roll_split_waves<S>(), roll_split_occ<S>()) void rollout_split_kernel(RolloutArgs a) {
  static_assert((S::B == 64 && S::NIT == 4 && S::NOT == 4) ||
                    (S::B == 32 && S::NIT == 2 && S::NOT == 2),
                "split rollout: B=64 [128,128] or B=32 [64,64]");
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  char *lds = reinterpret_cast<char *>(ldsf);
  stage_split_rollout<S>(a.params, a.env, lds);
  __syncthreads();
  const float *lfr = reinterpret_cast<const float *>(lds + RollSplitLds<S>::F);
  const float b3 = lfr[RollSplitLds<S>::B3];
  const float *b1fa = lfr + RollSplitLds<S>::B1F, *b1fb = b1fa + S::H1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, lr = lane & 31;
  const int wpb = blockDim.x >> 6;
  const int ngroups = a.b.N / S::G;
  const int t_last = a.t + (a.nsteps > 1 ? a.nsteps : 1) - 1;
  // lane = row 32 h + lr of the group: env e0 + h and bin lr when G = 2,
  // bin = lane when G = 1
  const int eoff = S::G == 2 ? h : 0, seg0 = S::G == 2 ? 32 * h : 0;
  const int bin = S::G == 2 ? lr : lane;
  // this workgroup's groups: a contiguous block of ceil(ngroups / grid),
  // dealt round-robin to its waves, so that every CU steps the same number
  // (the grid-strided order gave a sixth of the CUs one round more)
  const int per = (ngroups + (int)gridDim.x - 1) / (int)gridDim.x;
  const int g_end = min(ngroups, ((int)blockIdx.x + 1) * per);
  for (int g = (int)blockIdx.x * per + w; g < g_end; g += wpb) {
    const int e0 = g * S::G, env = e0 + eoff;
    RowRaw<S> cur;
    fetch_rows<S>(a.b, a.src_slot > 0 ? a.src_slot : a.t, e0, cur);
    if (a.src_slot > 0) {  // slot 0 := slot src_slot: this lane's row
      int8_t *ob = a.b.bins + (size_t)env * S::BD + bin * S::D;
#pragma unroll
      for (int d = 0; d < S::D; ++d) ob[d] = (int8_t)(h ? cur.bv[1][d] : cur.bv[0][d]);
      if (bin == 0) {
        int8_t *oi = a.b.items + (size_t)env * 4;
#pragma unroll
        for (int d = 0; d < 4; ++d)
          oi[d] = d < S::D ? (int8_t)(h ? cur.iv[1][d] : cur.iv[0][d]) : 0;
      }
    }
    uint32_t x = a.b.rng[env];
    for (int t = a.t; t <= t_last; ++t) {
      // each r-tile's env's item -> its folded bias (item-table entries only)
      const float *b1r[2];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        bool ia = true;
#pragma unroll
        for (int d = 0; d < S::D; ++d) ia &= cur.iv[rt][d] == a.env.item_a[d];
        b1r[rt] = ia ? b1fa : b1fb;
      }
      float zl[2];
      wave_logits_split<S>(lds, cur, b1r, zl);
      const float z = (h ? zl[1] : zl[0]) + b3;
      int nbv[S::D];
      bool first;
      sample_step_x<S>(a, t, t == t_last, z, env, seg0, bin, cur, x, nbv, first);
      if (t < t_last) {
        // rows lr / 32 + lr of slot t+1: this half's and the partner's
#pragma unroll
        for (int d = 0; d < S::D; ++d) {
          const int own = nbv[d], oth = __shfl_xor(own, 32, kWave);
          const int ito = first ? a.env.item_a[d] : a.env.item_b[d];
          const int itp = S::G == 2 ? __shfl_xor(ito, 32, kWave) : ito;
          cur.bv[0][d] = h ? oth : own;
          cur.bv[1][d] = h ? own : oth;
          cur.iv[0][d] = h ? itp : ito;
          cur.iv[1][d] = h ? ito : itp;
        }
      }
    }
    if (bin == 0) a.b.rng[env] = (t_last == a.b.T - 1) ? mstd_mulmod(x, a.jump_mul) : x;
  }
}

// Softmax of one env's 128 candidate-bin scores (lane holds bins lane and
// 64 + lane: z[0], z[1]), the categorical sample (sequential
// discrete_distribution order, the exact restatement near a boundary) or the
// forced action, and the env transition of slot t into slot t+1 -- one wave.
// x: the env's minstd state (the caller loads / stores it); last: the
// launch's last step (logits / probabilities outputs).  In: nbv[k] = bin
// k * 64 + lane of slot t and iv = slot t's item (the caller's registers: the
// state is not read back from HBM); out: nbv[k] in slot t+1, first = the
// next item is item_a.
template <class S>
__device__ __forceinline__ void sample_step128_x(const RolloutArgs &a, int t, bool last,
                                                 int env, const float (&z)[2],
                                                 uint32_t &x, int (&nbv)[2][S::D],
                                                 const int (&iv)[S::D], bool &first) {
  const int lane = threadIdx.x & 63;
  const int N = a.b.N;
  float p[2];
  float se = 0.0f;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    p[k] = expf(z[k]);
    se += p[k];
  }
  se = seg_sum<64>(se);
  p[0] = p[0] / se;
  p[1] = p[1] / se;
  if (last && a.logits_out) {
    a.logits_out[(size_t)env * 128 + lane] = z[0];
    a.logits_out[(size_t)env * 128 + 64 + lane] = z[1];
  }
  if (last && a.probs_out) {
    a.probs_out[(size_t)env * 128 + lane] = p[0];
    a.probs_out[(size_t)env * 128 + 64 + lane] = p[1];
  }
  if (a.qold_out) {  // KL-PPO / record_distrib: every step's distribution
    a.qold_out[((size_t)t * N + env) * 128 + lane] = p[0];
    a.qold_out[((size_t)t * N + env) * 128 + 64 + lane] = p[1];
  }
  int choice;
  if (a.forced) {
    choice = a.forced[(size_t)t * N + env];
    (void)canonical(x);
  } else {
    const double pd0 = (double)p[0], pd1 = (double)p[1];
    const double sd = seg_sum_d<64>(pd0 + pd1);
    const double c0 = seg_scan_d<64>(pd0 / sd, lane);
    const double tot0 = wave_shfl_d(c0, 63);
    double c1 = tot0 + seg_scan_d<64>(pd1 / sd, lane);
    if (lane == 63) c1 = 1.0;
    const double u = canonical(x);
    choice = __popcll(__ballot(c0 < u)) + __popcll(__ballot(c1 < u));
    const float gap = (float)fmin(fabs(c0 - u), fabs(c1 - u));
    if (seg_min<64>(gap) < 1e-9f) {  // exact sequential restatement
      double s2 = 0.0;
      for (int k = 0; k < 128; ++k)
        s2 += (double)wave_shfl(p[k >> 6], k & 63);
      double acc = 0.0;
      int c2 = 127;
      for (int k = 0; k < 128; ++k) {
        const double qk = (double)wave_shfl(p[k >> 6], k & 63) / s2;
        acc = k == 0 ? qk : acc + qk;
        const double cpk = k == 127 ? 1.0 : acc;
        if (!(cpk < u) && k < c2) c2 = k;
      }
      choice = c2;
    }
  }
  const float pold = choice < 64 ? wave_shfl(p[0], choice)
                                 : wave_shfl(p[1], choice - 64);
  int nb[2][S::D];
  int neg[2] = {0, 0};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int bin = k * 64 + lane;
#pragma unroll
    for (int d = 0; d < S::D; ++d) {
      nb[k][d] = bin == choice ? nbv[k][d] - iv[d] : nbv[k][d];
      neg[k] |= nb[k][d] < 0;
    }
  }
  const int done = __shfl(choice < 64 ? neg[0] : neg[1], choice & 63, kWave);
  first = canonical(x) < a.env.p_a;
  const size_t o = (size_t)(t + 1) * N + env;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    int8_t *ob = a.b.bins + o * S::BD + (k * 64 + lane) * S::D;
#pragma unroll
    for (int d = 0; d < S::D; ++d) {
      nbv[k][d] = done ? kCapacity : nb[k][d];
      ob[d] = (int8_t)nbv[k][d];
    }
  }
  if (lane == 0) {
    int8_t *oi = a.b.items + o * 4;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      oi[d] = d < S::D ? (int8_t)(first ? a.env.item_a[d] : a.env.item_b[d]) : 0;
    a.b.action[(size_t)t * N + env] = choice;
    a.b.pold[(size_t)t * N + env] = pold;
    a.b.done[(size_t)t * N + env] = (uint8_t)done;
  }
}

// One step (slot a.t): sample_step128_x with the stream state read from and
// written back to a.b.rng (jumped after step T-1).
template <class S>
__device__ __forceinline__ void sample_step128(const RolloutArgs &a, int env,
                                               const float (&z)[2]) {
  const int lane = threadIdx.x & 63;
  uint32_t x = a.b.rng[env];
  // slot a.t's bins of this lane and its item, from HBM
  const size_t e = (size_t)a.t * a.b.N + env;
  int nbv[2][S::D], iv[S::D];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int d = 0; d < S::D; ++d) nbv[k][d] = a.b.bins[e * S::BD + (k * 64 + lane) * S::D + d];
#pragma unroll
  for (int d = 0; d < S::D; ++d) iv[d] = a.b.items[e * 4 + d];
  bool first;
  sample_step128_x<S>(a, a.t, true, env, z, x, nbv, iv, first);
  if (lane == 0) a.b.rng[env] = (a.t == a.b.T - 1) ? mstd_mulmod(x, a.jump_mul) : x;
}

// ================================================ rollout step, 128 bins ===
// One env per group (B = 128 = two 64-row half-groups, BASELINE config 5).
// Forward as rollout_step_kernel per half-group, scores of all 128
// candidate bins staged in LDS, then wave 0 samples with two bins per lane
// (bins lane and 64 + lane; sequential discrete_distribution order).
template <class S>
__global__ __launch_bounds__(256, 2) void rollout_step128_kernel(RolloutArgs a) {
  static_assert(S::B == 128 && S::HG == 2, "128-bin rollout");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  stage_params<S>(a.params, lds);
  __syncthreads();
  constexpr int R = S::R;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 31;
  const int N = a.b.N, t = a.t;
  const int o2t = w % S::NOT;
  const int rt0 = S::NOT >= 4 ? 0 : w / S::NOT;
  const bool fwd_active = (w / S::NOT) * S::FJ < 2;
  for (int env = blockIdx.x; env < N; env += gridDim.x) {
#pragma unroll
    for (int hg = 0; hg < 2; ++hg) {
      RowRaw<S> rr;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int bin = hg * 64 + k * 32 + lr;
        const size_t e = (size_t)t * N + env;
        const int8_t *bp = a.b.bins + e * S::BD + bin * S::D;
        const int8_t *ip = a.b.items + e * 4;
#pragma unroll
        for (int d = 0; d < S::D; ++d) {
          rr.bv[k][d] = bp[d];
          rr.iv[k][d] = ip[d];
        }
      }
      f32x16 h1[S::NIT][2];
      layer1<S>(rr, lds, h1);
      if (fwd_active) {
        f32x16 pre[S::FJ];
        layer2<S, S::FJ>(lds, h1, o2t, rt0, pre);
#pragma unroll
        for (int q = 0; q < S::FJ; ++q) {
          const float zp = logit_part<S>(lds, pre[q], o2t);
          if (lane < 32) lds[S::L_Z + o2t * R + hg * 64 + (rt0 + q) * 32 + lr] = zp;
        }
      }
    }
    __syncthreads();
    if (w == 0) {
      float z[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        float zs = 0.0f;
#pragma unroll
        for (int o = 0; o < S::NOT; ++o) zs += lds[S::L_Z + o * R + k * 64 + lane];
        z[k] = zs + lds[S::L_B3];
      }
      sample_step128<S>(a, env, z);
    }
    __syncthreads();
  }
}

// ========================================= rollout step, 128 bins, wave/env ==
// B = 128, [128,128] (config 5): one wave per env, the wave_kernel scheme
// over the env's two 64-row half-groups in turn (every layer operation and
// its order as rollout_step128_kernel's, so logits and actions are
// bit-identical), then the wave samples its own env: no barrier between the
// forward and the sampler and four waves per SIMD to hide the
// double-precision sampler under the other waves' MFMAs.
template <class S>
__global__ __launch_bounds__(64 * kRollWaves128, roll_occ(kRollWaves128)) void rollout_wave128_kernel(RolloutArgs a) {
  static_assert(S::B == 128 && S::NIT == 4 && S::NOT == 4,
                "wave rollout: B=128, [128,128]");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  stage_params<S>(a.params, lds);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 31,
            h = lane >> 5;
  const int wpb = blockDim.x >> 6;
  const int N = a.b.N, t = a.t;
  for (int env = blockIdx.x * wpb + w; env < N; env += gridDim.x * wpb) {
    float z0 = 0.0f, z1 = 0.0f;
#pragma unroll 1
    for (int hg = 0; hg < 2; ++hg) {
      RowRaw<S> cur;
      const size_t e = (size_t)t * N + env;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int bin = hg * 64 + rt * 32 + lr;
        const int8_t *bp = a.b.bins + e * S::BD + bin * S::D;
        const int8_t *ip = a.b.items + e * 4;
#pragma unroll
        for (int d = 0; d < S::D; ++d) {
          cur.bv[rt][d] = bp[d];
          cur.iv[rt][d] = ip[d];
        }
      }
      float xb[2][S::S1];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int s = 0; s < S::S1; ++s) xb[rt][s] = row_feature<S>(cur, rt, 2 * s + h);
      float zl[2] = {0.0f, 0.0f};
      if (XH_V_RPASS) wave_logits_rpass<S, XH_V_RTILES128>(lds, cur, zl);
#pragma unroll 1
      for (int o2t = 0; o2t < (XH_V_RPASS ? 0 : 4); ++o2t) {
        const float *wrow = lds + S::L_W2 + (o2t * 32 + lr) * S::W2S + 4 * h;
        f32x16 pre[2];
        pre[0] = zero16();
        pre[1] = zero16();
#pragma unroll 1
        for (int it = 0; it < 4; ++it) {
          f32x16 t1[2];
          t1[0] = zero16();
          t1[1] = zero16();
#pragma unroll
          for (int s = 0; s < S::S1; ++s) {
            const int k = 2 * s + h;
            const float wa = k < S::F0 ? lds[S::L_W1 + (it * 32 + lr) * S::F0 + k] : 0.0f;
            t1[0] = mfma32(wa, xb[0][s], t1[0]);
            t1[1] = mfma32(wa, xb[1][s], t1[1]);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 bb = lds4(lds + S::L_B1 + it * 32 + 8 * q + 4 * h);
            const float bq[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              t1[0][4 * q + u] = relu(t1[0][4 * q + u] + bq[u]);
              t1[1][4 * q + u] = relu(t1[1][4 * q + u] + bq[u]);
            }
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 a4 = lds4(wrow + it * 32 + 8 * q);
            const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              pre[0] = mfma32(av[u], t1[0][4 * q + u], pre[0]);
              pre[1] = mfma32(av[u], t1[1][4 * q + u], pre[1]);
            }
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 bb = lds4(lds + S::L_B2 + o2t * 32 + 8 * q + 4 * h);
          const float bq[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            pre[0][4 * q + u] += bq[u];
            pre[1][4 * q + u] += bq[u];
          }
        }
        zl[0] += logit_part<S>(lds, pre[0], o2t);
        zl[1] += logit_part<S>(lds, pre[1], o2t);
      }
      // lane = row of the half-group = bin hg*64 + lane
      const float zh = (h ? zl[1] : zl[0]) + lds[S::L_B3];
      if (hg == 0)
        z0 = zh;
      else
        z1 = zh;
    }
    const float z[2] = {z0, z1};
    sample_step128<S>(a, env, z);
  }
}

// The 128-bin wave rollout (config 5) with the split layer 2: each env's two
// 64-row half-groups through wave_logits_split, then sample_step128 as in
// rollout_wave128_kernel.  3 waves per SIMD (168 VGPRs).
constexpr int kRollWavesS128 = 12;
template <class S>
__global__ __launch_bounds__(64 * kRollWavesS128, 3) void rollout_split128_kernel(RolloutArgs a) {
  static_assert(S::B == 128 && S::NIT == 4 && S::NOT == 4,
                "split rollout: B=128, [128,128]");
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  char *lds = reinterpret_cast<char *>(ldsf);
  stage_split_rollout<S>(a.params, a.env, lds);
  __syncthreads();
  const float *lfr = reinterpret_cast<const float *>(lds + RollSplitLds<S>::F);
  const float b3 = lfr[RollSplitLds<S>::B3];
  const float *b1fa = lfr + RollSplitLds<S>::B1F, *b1fb = b1fa + S::H1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int wpb = blockDim.x >> 6;
  const int N = a.b.N;
  const int t_last = a.t + (a.nsteps > 1 ? a.nsteps : 1) - 1;
  // this workgroup's envs: a contiguous block of ceil(N / grid), dealt
  // round-robin to its waves, so that every CU steps the same number (the
  // grid-strided order gave a third of the CUs six rounds against 5.33 on
  // average at config 5)
  const int per = (N + (int)gridDim.x - 1) / (int)gridDim.x;
  const int env_end = min(N, ((int)blockIdx.x + 1) * per);
  for (int env = (int)blockIdx.x * per + w; env < env_end; env += wpb) {
    // slot t's rows of this lane: bins hg * 64 + rt * 32 + lr (the sampler's
    // lane 32 rt + lr, slot hg), from global for slot a.t, then from the
    // sampler's registers (this half's value and the partner half's)
    int own[2][S::D], it[S::D];
    {
      const size_t e = (size_t)(a.src_slot > 0 ? a.src_slot : a.t) * N + env;
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int d = 0; d < S::D; ++d) own[k][d] = a.b.bins[e * S::BD + (k * 64 + lane) * S::D + d];
#pragma unroll
      for (int d = 0; d < S::D; ++d) it[d] = a.b.items[e * 4 + d];
      if (a.src_slot > 0) {  // slot 0 := slot src_slot
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int d = 0; d < S::D; ++d)
            a.b.bins[(size_t)env * S::BD + (k * 64 + lane) * S::D + d] = (int8_t)own[k][d];
        if (lane == 0)
#pragma unroll
          for (int d = 0; d < 4; ++d) a.b.items[(size_t)env * 4 + d] = d < S::D ? (int8_t)it[d] : 0;
      }
    }
    uint32_t x = a.b.rng[env];
    for (int t = a.t; t <= t_last; ++t) {
      bool ia = true;
#pragma unroll
      for (int d = 0; d < S::D; ++d) ia &= it[d] == a.env.item_a[d];
      const float *b1r[2] = {ia ? b1fa : b1fb, ia ? b1fa : b1fb};
      float z[2];
#pragma unroll 1
      for (int hg = 0; hg < 2; ++hg) {
        RowRaw<S> cur;
#pragma unroll
        for (int d = 0; d < S::D; ++d) {
          const int v = hg ? own[1][d] : own[0][d];
          const int o = __shfl_xor(v, 32, kWave);
          cur.bv[0][d] = h ? o : v;
          cur.bv[1][d] = h ? v : o;
          cur.iv[0][d] = it[d];
          cur.iv[1][d] = it[d];
        }
        float zl[2];
        wave_logits_split<S>(lds, cur, b1r, zl);
        // lane = row of the half-group = bin hg*64 + lane
        const float zh = (h ? zl[1] : zl[0]) + b3;
        if (hg == 0)
          z[0] = zh;
        else
          z[1] = zh;
      }
      bool first;
      sample_step128_x<S>(a, t, t == t_last, env, z, x, own, it, first);
#pragma unroll
      for (int d = 0; d < S::D; ++d) it[d] = first ? a.env.item_a[d] : a.env.item_b[d];
    }
    if (lane == 0) a.b.rng[env] = (t_last == a.b.T - 1) ? mstd_mulmod(x, a.jump_mul) : x;
  }
}


// ======================================================= argmax evaluation ==
// Whole episodes inside one launch: the G envs of a group keep their state in
// LDS and step until each has finished `episodes` episodes (argmax action: no
// sampling draws, 2 engine draws per step for the item / reset).
template <class S>
__global__ __launch_bounds__(256, 1) void eval_argmax_kernel(EvalArgs a) {
  static_assert(S::HG == 1, "groups of whole envs");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  stage_params<S>(a.params, lds);
  constexpr int B = S::B, G = S::G, D = S::D;
  int *sbins = reinterpret_cast<int *>(lds + S::L_ROLLOUT_END);  // [G][B*D]
  int *sitem = sbins + G * S::BD;                                // [G][4]
  uint32_t *srng = reinterpret_cast<uint32_t *>(sitem + G * 4);  // [G]
  int *sleft = reinterpret_cast<int *>(srng + G);                // [G]
  int *sflag = sleft + G;                                        // [1]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 31;
  const int o2t = w % S::NOT;
  const int rt0 = S::NOT >= 4 ? 0 : w / S::NOT;
  const bool fwd_active = (w / S::NOT) * S::FJ < 2;
  const int ngroups = a.n_envs / G;
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    __syncthreads();
    if (w == 0) {  // construct: bins at capacity, one item (2 draws)
      const int e = lane / B, bin = lane % B, env = g * G + e;
      uint32_t x = mstd_jump(a.x0, (uint64_t)env * a.stream_stride);
      bool first = false;
      if (!a.init_items) first = canonical(x) < a.env.p_a;
      for (int d = 0; d < D; ++d) sbins[e * S::BD + bin * D + d] = kCapacity;
      if (bin == 0) {
        for (int d = 0; d < 4; ++d)
          sitem[e * 4 + d] =
              d >= D ? 0
              : a.init_items ? a.init_items[env * D + d]
              : (first ? a.env.item_a[d] : a.env.item_b[d]);
        srng[e] = x;
        sleft[e] = a.episodes;
        a.total[env] = 0.0;
        a.steps[env] = 0;
      }
    }
    __syncthreads();
    double reward = 0.0;  // per segment leader
    long nsteps = 0;
    for (long it = 0; it < a.max_steps; ++it) {
      RowRaw<S> rr;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int r = rt * 32 + lr, e = r / B, bin = r % B;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          rr.bv[rt][d] = sbins[e * S::BD + bin * D + d];
          rr.iv[rt][d] = sitem[e * 4 + d];
        }
      }
      {
        f32x16 h1[S::NIT][2];
        layer1<S>(rr, lds, h1);
        if (fwd_active) {
          f32x16 pre[S::FJ];
          layer2<S, S::FJ>(lds, h1, o2t, rt0, pre);
#pragma unroll
          for (int q = 0; q < S::FJ; ++q) {
            const float zp = logit_part<S>(lds, pre[q], o2t);
            if (lane < 32) lds[S::L_Z + o2t * 64 + (rt0 + q) * 32 + lr] = zp;
          }
        }
      }
      __syncthreads();
      if (w == 0) {
        const int e = lane / B, bin = lane % B, seg0 = e * B;
        float zs = 0.0f;
#pragma unroll
        for (int o = 0; o < S::NOT; ++o) zs += lds[S::L_Z + o * 64 + lane];
        float v = zs + lds[S::L_B3];
        if (a.argmax_probs) {
          const float ex = expf(v);
          v = ex / seg_sum<B>(ex);
        }
        const int choice = seg_argmax_first<B>(v, bin);  // tensor.cc:464-466
        const bool active = sleft[e] > 0;
        int nb[D];
        int neg = 0;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const int b0 = sbins[e * S::BD + bin * D + d];
          nb[d] = bin == choice ? b0 - sitem[e * 4 + d] : b0;
          neg |= nb[d] < 0;
        }
        const int done = __shfl(neg, seg0 + choice, kWave);
        if (active) {
          uint32_t x = srng[e];
          const bool first = canonical(x) < a.env.p_a;  // get_item / reset
#pragma unroll
          for (int d = 0; d < D; ++d)
            sbins[e * S::BD + bin * D + d] = done ? kCapacity : nb[d];
          // all lanes of the segment read srng/sitem above before this write
          __builtin_amdgcn_wave_barrier();
          if (bin == 0) {
            for (int d = 0; d < D; ++d)
              sitem[e * 4 + d] = first ? a.env.item_a[d] : a.env.item_b[d];
            srng[e] = x;
            if (done) sleft[e] -= 1;
            reward += done ? 0.0 : 1.0;
            if (a.trace && g == 0 && e == 0 && nsteps < a.trace_cap)
              a.trace[nsteps] = choice;
            ++nsteps;
          }
        }
        // sleft was updated above by this wave's segment leaders
        const int any = __any(sleft[e] > 0);
        if (lane == 0) *sflag = any;
      }
      __syncthreads();
      if (*sflag == 0) break;
    }
    if (w == 0 && lane % B == 0) {
      const int env = g * G + lane / B;
      a.total[env] = reward;
      a.steps[env] = nsteps;
      a.rng_out[env] = srng[lane / B];
      for (int d = 0; d < D; ++d)
        a.final_items[env * D + d] = sitem[(lane / B) * 4 + d];
    }
  }
}

// 4-wave train kernel schedule knobs (A/B variants, make variant), applied
// to the shapes with one dW2 / dH1 tile per wave (JW = JH = 1: config 2):
//   XH_V4_UNROLL: bit0 fully unroll the dW2 row loop, bit1 the dH1 loop
//   XH_V4_L3:     1 = the layer-3 weights loaded before the softmax
// config 2 (tools/gpu_ab_vars.sh): 0.171 ms per epoch -> 0.169 (bit0),
// 0.165 (bit1), 0.163 (both), 0.160 (both + L3); same arithmetic order
#ifndef XH_V4_UNROLL
#define XH_V4_UNROLL 3
#endif
#ifndef XH_V4_L3
#define XH_V4_L3 1
#endif


// ============================================================ train epoch ==
// KL = true: kl_ppo_learner's epoch (policy_gradient.h:310-335) -- every row
// of the state matrix: transitions, then the open trajectories' end rows
// (slot T, q of step T-1), then the terminal end rows E_t of end_list (the
// overflowed view, rl.h:336-343); end rows have A = 0 and the previous
// action's distribution (policy_gradient.h:178).
template <class S, bool KL>
__global__ __launch_bounds__(256, S::TOCC) void policy_train_kernel(PolicyTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // kernel-level stamps in the last trace group's slots (trace build)
  XH_SPAN(a, 0);
  XH_STAMP4(a, kTraceGroups - 1, threadIdx.x >> 6, threadIdx.x & 63, 0);
  stage_params<S>(a.params, lds);
  __syncthreads();
  XH_STAMP4(a, kTraceGroups - 1, threadIdx.x >> 6, threadIdx.x & 63, 1);
  XH_SPAN(a, 1);
  constexpr int B = S::B, NIT = S::NIT, NOT = S::NOT;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 31,
            h = lane >> 5;
  const int N = a.b.N, T = a.b.T;
  const int gpt = N / S::G;  // groups per step
  const int gmain = T * gpt;
  const int n_end = KL ? *a.n_end : 0;
  const int ngroups = KL ? gmain + gpt + (n_end + S::G - 1) / S::G : gmain;
  const float beta = KL ? *a.beta : 0.0f;
  double kl_acc = 0.0;
  float *H1img = lds + S::L_H1;
  float *DAimg = lds + S::L_DA2;

  // wave roles (see header comment)
  const int o2t = w % NOT;
  const int rt0 = NOT >= 4 ? 0 : w / NOT;
  const bool fwd_active = (w / NOT) * S::FJ < 2;
  const int it_own = w % NIT;             // dH1 / dW1 tile
  const int hrt0 = NIT >= 4 ? 0 : w / NIT;  // first dH1 r-tile
  constexpr int HSTEP = 4 / NIT;          // r-tile stride between slots

  // persistent accumulators
  f32x16 accW2[S::JW];
#pragma unroll
  for (int q = 0; q < S::JW; ++q) accW2[q] = zero16();
  float accW1[16][S::F0], accB1[16], accW3[16], accB2[16], accB3 = 0.0f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    accB1[j] = accW3[j] = accB2[j] = 0.0f;
#pragma unroll
    for (int f = 0; f < S::F0; ++f) accW1[j][f] = 0.0f;
  }

  // prefetched per-group inputs: two rows per lane + this lane's env record
  RowRaw<S> cur, nxt;
  int c_cur = 0, c_nxt = 0, v_cur = 1, v_nxt = 1;
  float po_cur = 1.0f, po_nxt = 1.0f, A_cur = 0.0f, A_nxt = 0.0f;
  float q_cur = 1.0f, q_nxt = 1.0f;
  auto fetch = [&](int g, RowRaw<S> &rr, int &c, float &po, float &A, float &q,
                   int &valid) {
    if constexpr (!KL) {
      const int t = g / gpt, e0 = (g - t * gpt) * S::G;
      fetch_rows<S>(a.b, t, e0, rr);
      const size_t ti = (size_t)t * N + e0 + lane / B;
      c = a.b.action[ti];
      po = a.b.pold[ti];
      A = a.adv[ti];
    } else {
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int r = rt * 32 + lr, el = r / B, bin = r % B;
        int t, e, kind, ok = 1;
        if (g < gmain) {
          t = g / gpt;
          e = (g - t * gpt) * S::G + el;
          kind = 0;
        } else if (g < gmain + gpt) {
          t = T;
          e = (g - gmain) * S::G + el;
          kind = 1;
          ok = a.b.done[(size_t)(T - 1) * N + e] == 0;
        } else {
          const int j = (g - gmain - gpt) * S::G + el;
          kind = 2;
          ok = j < n_end;
          const int te = ok ? a.end_list[j] : 0;
          t = te / N;
          e = te - t * N;
        }
        const size_t env = (size_t)t * N + e;
        const int8_t *bp = a.b.bins + env * S::BD + bin * S::D;
        const int8_t *ip = a.b.items + env * 4;
        const bool sub = kind == 2 && a.b.action[env] == bin;
#pragma unroll
        for (int d = 0; d < S::D; ++d) {
          rr.iv[rt][d] = ip[d];
          rr.bv[rt][d] = bp[d] - (sub ? ip[d] : 0);
        }
        if (rt == h) {  // this lane's own row (= lane) of the loss head
          c = kind == 0 ? a.b.action[env] : 0;
          A = kind == 0 ? a.adv[env] : 0.0f;
          po = 1.0f;
          const size_t qrow = kind == 1 ? (size_t)(T - 1) * N + e : env;
          q = a.qold[qrow * B + bin];
          valid = ok;
        }
      }
    }
  };
  if ((int)blockIdx.x < ngroups)
    fetch(blockIdx.x, cur, c_cur, po_cur, A_cur, q_cur, v_cur);

  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int gi = (g - (int)blockIdx.x) / (int)gridDim.x;
    (void)gi;
    XH_STAMP4(a, gi, w, lane, 0);
    const int gn = g + gridDim.x;
    if (gn < ngroups) fetch(gn, nxt, c_nxt, po_nxt, A_nxt, q_nxt, v_nxt);
    f32x16 pre[S::FJ];
    f32x16 h1own[2];
    {
      f32x16 h1[NIT][2];
      layer1<S>(cur, lds, h1);
      // H1 image for dW2 (each H1 tile written by one wave)
      if (w < NIT) {
#pragma unroll
        for (int it = 0; it < NIT; ++it)
          if (it == w) {
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
              for (int j = 0; j < 16; ++j)
                H1img[(rt * 32 + lr) * S::HS + it * 32 + acc_row(j, h)] =
                    h1[it][rt][j];
          }
      }
#pragma unroll
      for (int it = 0; it < NIT; ++it)
        if (it == it_own) {
          h1own[0] = h1[it][0];
          h1own[1] = h1[it][1];
        }
      if (fwd_active) {
        if (!XH_ABL(a, 4)) {
          layer2<S, S::FJ>(lds, h1, o2t, rt0, pre);
        } else {
#pragma unroll
          for (int q = 0; q < S::FJ; ++q) pre[q] = h1[0][q & 1];
        }
#pragma unroll
        for (int q = 0; q < S::FJ; ++q) {
          const float zp = logit_part<S>(lds, pre[q], o2t);
          if (lane < 32) lds[S::L_Z + o2t * 64 + (rt0 + q) * 32 + lr] = zp;
        }
      }
    }
    XH_STAMP4(a, gi, w, lane, 1);
    __syncthreads();
    XH_STAMP4(a, gi, w, lane, 2);

    constexpr bool kOne = S::JW == 1 && S::JH == 1 && !KL;  // KL: spills
    constexpr int kU4 = kOne ? XH_V4_UNROLL : 0;
    constexpr bool kL34 = kOne && XH_V4_L3;
    float4 w3v[4];
    if (kL34) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        w3v[qq] = lds4(lds + S::L_W3 + o2t * 32 + 8 * qq + 4 * h);
    }

    // ---- logits -> softmax -> loss gradient w.r.t. logits (lane = row)
    float gz;
    {
      const int bin = lane % B, seg0 = (lane / B) * B;
      float zs = 0.0f;
#pragma unroll
      for (int o = 0; o < NOT; ++o) zs += lds[S::L_Z + o * 64 + lane];
      const float z = zs + lds[S::L_B3];
      const float ex = expf(z);
      const float p = ex / seg_sum<B>(ex);
      const int c = c_cur;
      const float A = A_cur;
      if constexpr (KL) {
        // kl_regulated_loss: softmax_gradient_log + beta (p - q), applied as
        // a probability-space gradient through softmax_layer::backward
        // (nn.h:393-417): gz_j = p_j (g_j - sum_k p_k g_k)
        float gp = p * A + beta * (p - q_cur);
        if (bin == c) gp -= A;
        const float sg = seg_sum<B>(p * gp);
        gz = v_cur ? p * (gp - sg) : 0.0f;
        if (w == 0 && v_cur)
          kl_acc += (double)q_cur * log((double)q_cur / (double)p);
      } else if (XH_ABL(a, 8)) {
        gz = z * 1e-3f;
      } else if (a.algo == kPPO) {
        // clipped_gradient (rl.h:54-74) then softmax_layer::backward
        // (nn.h:393-417): gz_j = (diag(p) - p p^T)[j][c] * g_c
        const float pc = wave_shfl(p, seg0 + c);
        const float ratio = pc / po_cur;
        float clipped = ratio;
        if (ratio > 1.0f + a.clip_eps)
          clipped = 1.0f + a.clip_eps;
        else if (ratio < 1.0f - a.clip_eps)
          clipped = 1.0f - a.clip_eps;
        const float ig = fminf(clipped * A, ratio * A) * -1.0f;
        const float gc = ig / pc;
        const float lin = bin == c ? p : 0.0f;
        gz = (lin - p * pc) * gc;
      } else {
        // softmax_gradient_log (rl.h:45-52) through softmax-xent (identity)
        gz = p * A;
        if (bin == c) gz -= A;
      }
      if (w == 0) accB3 += gz;
    }
    XH_STAMP4(a, gi, w, lane, 3);

    // ---- backward through layer 3 and the layer-2 relu (fwd tiles)
    if (fwd_active) {
#pragma unroll
      for (int q = 0; q < S::FJ; ++q) {
        const int rt = rt0 + q;
        const float gr = wave_shfl(gz, rt * 32 + lr);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const float4 ww =
              kL34 ? w3v[qq] : lds4(lds + S::L_W3 + o2t * 32 + 8 * qq + 4 * h);
          const float wq[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = 4 * qq + u;
            const float v = pre[q][j];
            const float h2 = relu(v);
            accW3[j] += gr * h2;
            const float d = v > 0.0f ? gr * wq[u] : 0.0f;
            accB2[j] += d;
            DAimg[(rt * 32 + lr) * S::AS + o2t * 32 + acc_row(j, h)] = d;
          }
        }
      }
    }
    XH_STAMP4(a, gi, w, lane, 4);
    __syncthreads();
    XH_STAMP4(a, gi, w, lane, 5);

    // ---- dW2[o2][i] += sum_r dA2[r][o2] H1[r][i]   (K = 64 rows); the JW
    // independent accumulation chains share the dA2 operand
    auto dw2_step = [&](int s) {
      const int r = 2 * s + h;
      const float av = DAimg[r * S::AS + o2t * 32 + lr];
#pragma unroll
      for (int q = 0; q < S::JW; ++q) {
        const int it = NOT >= 4 ? q : w / NOT + q * (4 / NOT);
        if (NOT >= 4 || it < NIT)
          accW2[q] = mfma32(av, H1img[r * S::HS + it * 32 + lr], accW2[q]);
      }
    };
    if constexpr (kU4 & 1) {
#pragma unroll
      for (int s = 0; s < 32; ++s) dw2_step(s);
    } else {
#pragma unroll 4
      for (int s = 0; s < (XH_ABL(a, 1) ? 0 : 32); ++s) dw2_step(s);
    }
    XH_STAMP4(a, gi, w, lane, 6);

    // ---- dH1^T[i][r] = sum_o2 W2[o2][i] dA2[r][o2]; relu'; dW1, db1
    {
      f32x16 dh[S::JH];
#pragma unroll
      for (int q = 0; q < S::JH; ++q) dh[q] = zero16();
      auto dh1_step = [&](int s) {
        const int k = 2 * s + h;
        const float av = lds[S::L_W2 + k * S::W2S + it_own * 32 + lr];
#pragma unroll
        for (int q = 0; q < S::JH; ++q) {
          const int rt = NIT >= 4 ? q : hrt0 + q * HSTEP;
          if (NIT >= 4 || rt < 2)
            dh[q] = mfma32(av, DAimg[(rt * 32 + lr) * S::AS + k], dh[q]);
        }
      };
      if constexpr (kU4 & 2) {
#pragma unroll
        for (int s = 0; s < S::H2 / 2; ++s) dh1_step(s);
      } else {
#pragma unroll 4
        for (int s = 0; s < (XH_ABL(a, 2) ? 0 : S::H2 / 2); ++s) dh1_step(s);
      }
#pragma unroll
      for (int q = 0; q < S::JH; ++q) {
        const int rt = NIT >= 4 ? q : hrt0 + q * HSTEP;
        if (NIT >= 4 || rt < 2) {
          float xf[S::F0];
#pragma unroll
          for (int f = 0; f < S::F0; ++f)
            xf[f] = rt == 0 ? row_feature<S>(cur, 0, f) : row_feature<S>(cur, 1, f);
          const f32x16 hv = (rt == 0) ? h1own[0] : h1own[1];
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const float d = hv[j] > 0.0f ? dh[q][j] : 0.0f;
            accB1[j] += d;
#pragma unroll
            for (int f = 0; f < S::F0; ++f) accW1[j][f] += d * xf[f];
          }
        }
      }
    }
    XH_STAMP4(a, gi, w, lane, 7);
    __syncthreads();
    cur = nxt;
    c_cur = c_nxt;
    po_cur = po_nxt;
    A_cur = A_nxt;
    q_cur = q_nxt;
    v_cur = v_nxt;
  }
  XH_STAMP4(a, kTraceGroups - 1, w, lane, 2);
  XH_SPAN(a, 2);
  if constexpr (KL) {
    if (w == 0) {
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) kl_acc += __shfl_xor(kl_acc, o, kWave);
      if (lane == 0) a.kl_part[blockIdx.x] = kl_acc;
    }
  }

  // ---------------------------------------------------- slab write-out ----
  const PolicyLayout L{S::F0, S::H1, S::H2};
  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int q = 0; q < S::JW; ++q) {
    const int it = w / NOT + q * (4 / NOT);
    if (it < NIT) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int o2 = o2t * 32 + acc_row(j, h);
        slab[L.oW2() + o2 * S::H1 + it * 32 + lr] = accW2[q][j];
      }
    }
  }
  // per-lane partials -> sum over the 32 lanes of each half -> LDS scratch
  // [wave][RED] -> ordered sum over waves.
  float *scr = lds + S::L_H1;
  for (int i = threadIdx.x; i < 4 * S::RED; i += blockDim.x) scr[i] = 0.0f;
  __syncthreads();
  float *my = scr + w * S::RED;
  // layout inside RED: [dW1 (H1*F0)] [db1 (H1)] [dw3 (H2)] [db2 (H2)] [db3]
  const bool h_active = hrt0 < 2;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    // sums over the 32 rows of each lane half (DPP: valid in lr >= 16)
    const float vb1 = half_sum32(accB1[j]), vw3 = half_sum32(accW3[j]),
                vb2 = half_sum32(accB2[j]);
    float vw1[S::F0];
#pragma unroll
    for (int f = 0; f < S::F0; ++f) vw1[f] = half_sum32(accW1[j][f]);
    if (lr == 31) {
      const int i = it_own * 32 + acc_row(j, h);
      const int o2 = o2t * 32 + acc_row(j, h);
      if (h_active) {
#pragma unroll
        for (int f = 0; f < S::F0; ++f) my[i * S::F0 + f] = vw1[f];
        my[S::H1 * S::F0 + i] = vb1;
      }
      if (fwd_active) {
        my[S::H1 * S::F0 + S::H1 + o2] = vw3;
        my[S::H1 * S::F0 + S::H1 + S::H2 + o2] = vb2;
      }
    }
  }
  {
    float v = accB3;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o, kWave);
    if (w == 0 && lane == 0) my[S::RED - 1] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < S::RED; i += blockDim.x) {
    const float v = ((scr[i] + scr[S::RED + i]) + scr[2 * S::RED + i]) +
                    scr[3 * S::RED + i];
    int dst;
    if (i < S::H1 * S::F0)
      dst = L.oW1() + i;
    else if (i < S::H1 * S::F0 + S::H1)
      dst = L.ob1() + (i - S::H1 * S::F0);
    else if (i < S::H1 * S::F0 + S::H1 + S::H2)
      dst = L.ow3() + (i - S::H1 * S::F0 - S::H1);
    else if (i < S::RED - 1)
      dst = L.ob2() + (i - S::H1 * S::F0 - S::H1 - S::H2);
    else
      dst = L.ob3();
    slab[dst] = v;
  }
  XH_STAMP4(a, kTraceGroups - 1, w, lane, 3);
  XH_SPAN(a, 3);
}

// 8-wave train kernel schedule knobs (A/B variants, make variant; the
// defaults are the measured best, tools/gpu_ab_vars.sh; the dropped variants
// are listed in DESIGN.md §8):
//   XH_V_DH1: bit0 fully unroll the dH1 k-loop (64-row groups; the 128-row
//             kernel spills), bit1 K split by lane half (half h takes
//             o2 = s + 64h: consecutive steps are adjacent image rows)
//   XH_V_DH1W: the dH1 loop's unroll factor in the 128-row kernel
//   XH_V_L3:  1 = the layer-3 weights loaded before the softmax phase
//             (64-row groups): the layer-3 phase 1070 -> 660 cycles;
//             XH_V_L3W the same for 128-row groups (15.91 -> 15.82 ms)
//   measured without the trace stamps, config 3: 7.08 -> 6.67 ms per epoch
//   (XH_V_DH1 = 1 with XH_V_L3: the same arithmetic, bit-identical)
#ifndef XH_V_DH1
#define XH_V_DH1 1
#endif
#ifndef XH_V_DH1W
#define XH_V_DH1W 16
#endif
//   XH_V_W2U: the dW2 loop's unroll factor in the 128-row kernel: 8 (8 B
//             of spills) 14.53 ms per epoch against 15.55 ms at 4 (0 B)
#ifndef XH_V_W2U
#define XH_V_W2U 8
#endif
#ifndef XH_V_L3
#define XH_V_L3 1
#endif
#ifndef XH_V_L3W
#define XH_V_L3W 1
#endif
//   XH_V_FOLDW: the same for 128-row groups (config 5: 15.90 -> 15.60 ms)
#ifndef XH_V_FOLDW
#define XH_V_FOLDW 1
#endif
//   XH_V_FOLD: 1 = one env per 64-row group, D = 2: the item features'
//             layer-1 contribution (the same for every row of the group)
//             folded into the bias, one of the two layer-1 MFMA steps per
//             tile instead of two (per item-table entry, precomputed once):
//             config 3 6.71 -> 6.58 ms per epoch.  Train kernel only: the
//             rollout's logits feed the bit-exact sampler and keep the
//             reference's per-row sum
#ifndef XH_V_FOLD
#define XH_V_FOLD 1
#endif

// ================================================ train epoch, 8 waves ====
// H1 = H2 = 128 (BASELINE configs 3/4/5): 512-thread workgroup = 2 waves per
// SIMD so one wave's LDS / VALU / barrier time hides behind its partner's
// MFMAs.  Wave w = (q = w&3, rt = w>>2) owns:
//   forward    H2 tile q of r-tile rt (layer 1 fused tile by tile into the
//              layer-2 k-loop, so only one 16-register H1 tile is live)
//   dW2        tiles (q, 2rt) and (q, 2rt+1), K = all 64 rows
//   dH1 / dW1  H1 tile q of r-tile rt
template <class S>
__global__ __launch_bounds__(512, 2) void policy_train8_kernel(PolicyTrainArgs a) {
  static_assert(S::NIT == 4 && S::NOT == 4, "8-wave kernel is for 128x128");
  static_assert(8 * S::RED <= (S::H1 + S::H2) * S::TS, "scratch fits");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  stage_params<S>(a.params, lds);
  // one env per group (G == 1, B >= 64): the item is the same on every row
  constexpr bool kFold = XH_V_FOLD && S::G == 1 && (S::HG > 1 ? XH_V_FOLDW : 1);
  // kFold: layer-1 k-steps over the D bin features only (k = 2s + h < D)
  constexpr int kS1 = kFold ? (S::D + 1) / 2 : S::S1;
  if (kFold) {
    __syncthreads();
    // b1 + W1[:, item dims] . item / 8 for item_a (e = 0) and item_b (e = 1)
    for (int i = threadIdx.x; i < 2 * S::H1; i += blockDim.x) {
      const int e = i / S::H1, u = i - e * S::H1;
      const int *it = e == 0 ? a.env.item_a : a.env.item_b;
      float v = lds[S::L_B1 + u];
#pragma unroll
      for (int d = 0; d < S::D; ++d)
        v += lds[S::L_W1 + u * S::F0 + S::D + d] * ((float)it[d] / (float)kCapacity);
      lds[S::L_B1F + i] = v;
    }
  }
  __syncthreads();
  constexpr int B = S::B, HG = S::HG, R = S::R;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 31,
            h = lane >> 5;
  const int q = w & 3, rt = w >> 2;
  const int N = a.b.N, T = a.b.T;
  const int gpt = N / S::G;
  const int ngroups = T * gpt;
  float *H1T = lds + S::L_H1T;  // [H1][TS]: H1 transposed (feature-major)
  float *DAT = lds + S::L_DAT;  // [H2][TS]: dL/dA2 transposed

  f32x16 accW2[2];
  accW2[0] = zero16();
  accW2[1] = zero16();
  // dW1 columns of the bin features are accumulated per row; the item
  // features are constant per env and take one of the two table values
  // (bin_packing.h:73-74), so their columns (and db1) are carried as the
  // dA1 sums over rows holding item_a (sA) and item_b (sB).
  // kB2Late (128-row groups, the register-bound D=3 variant): db2 of H2 unit
  // q*32 + lr is summed from the dA2 image rows the dW2 loop reads anyway
  // (wave rt takes row quads 4rt..4rt+3 of its lane half): 15 registers
  // fewer than accB2[16] (spills 344 -> 272 B per lane).  The 64-row kernel
  // keeps the adds in the layer-3 phase (measured 0.1% faster there).
  constexpr bool kB2Late = S::HG > 1;
  // kMW1 (128-row groups): dW1 and db1 are not per-lane VALU sums but one
  // v_mfma_f32_16x16x4_f32 GEMM per half-group, dW1^T[f][i] = sum_r X[r][f]
  // dA1[r][i] with X = [bins/8, item/8, 1], over an LDS image of dA1 (the
  // freed H1 image) -- 80 accumulator registers fewer (the D=3 variant
  // spilled 208-340 B per lane), 4 more for the wave's 16-feature tile.
  constexpr bool kMW1 = S::HG > 1;
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 accW1m = {0.0f, 0.0f, 0.0f, 0.0f};
  float b2s = 0.0f;
  float accW1[16][S::D], sA[16], sB[16], accW3[16], accB2[16], accB3 = 0.0f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    sA[j] = sB[j] = accW3[j] = accB2[j] = 0.0f;
#pragma unroll
    for (int f = 0; f < S::D; ++f) accW1[j][f] = 0.0f;
  }

  // This lane's row (hg*64 + rt*32 + lr) is fetched one group ahead when a
  // group is one 64-row tile; its env record (action, p_old, advantage) at
  // the start of the group it is used in (consumed after the forward pass).
  int bv_c[S::D], iv_c[S::D], bv_n[S::D], iv_n[S::D];
  auto fetch_row = [&](int g, int hg, int (&bv)[S::D], int (&iv)[S::D]) {
    const int t = g / gpt, e0 = (g - t * gpt) * S::G;
    const int r = hg * 64 + rt * 32 + lr;
    const size_t env = (size_t)t * N + e0 + r / B;
    const int8_t *bp = a.b.bins + env * S::BD + (r % B) * S::D;
    const int8_t *ip = a.b.items + env * 4;
#pragma unroll
    for (int d = 0; d < S::D; ++d) {
      bv[d] = bp[d];
      iv[d] = ip[d];
    }
  };
  auto feat = [&](int f) {  // feature f of this lane's row (current tile)
    int v = 0;
#pragma unroll
    for (int d = 0; d < S::D; ++d) {
      if (f == d) v = bv_c[d];
      if (f == S::D + d) v = iv_c[d];
    }
    return f < S::F0 ? (float)v / (float)kCapacity : 0.0f;
  };
  // layer-1 input feature f: under kFold the item features are in the bias
  auto fold_feat = [&](int f) { return (kFold && f >= S::D) ? 0.0f : feat(f); };
  // kFold: this group's env holds item_b (set per group; wave-uniform)
  bool item_b_grp = false;
  // Layer 1 tile by tile, fused into the layer-2 k-loop, for this wave's
  // H2 tile q of r-tile rt; optionally writes its H1 tile q to the image.
  auto forward = [&](bool write_h1) {
    // accumulators start from the biases (no separate bias pass)
    f32x16 pre;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const float4 bb = lds4(lds + S::L_B2 + q * 32 + 8 * qq + 4 * h);
      pre[4 * qq + 0] = bb.x;
      pre[4 * qq + 1] = bb.y;
      pre[4 * qq + 2] = bb.z;
      pre[4 * qq + 3] = bb.w;
    }
    float xb[S::S1];
#pragma unroll
    for (int s = 0; s < S::S1; ++s) xb[s] = fold_feat(2 * s + h);
    const float *wrow = lds + S::L_W2 + (q * 32 + lr) * S::W2S + 4 * h;
    // layer-1 tile it's MFMA chain (from its biases)
    auto l1 = [&](int it) {
      f32x16 t;
      // kFold: the item's part folded into the bias of this group's item
      const float *bsrc = kFold ? lds + S::L_B1F + (item_b_grp ? S::H1 : 0)
                                : lds + S::L_B1;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const float4 bb = lds4(bsrc + it * 32 + 8 * qq + 4 * h);
        t[4 * qq + 0] = bb.x;
        t[4 * qq + 1] = bb.y;
        t[4 * qq + 2] = bb.z;
        t[4 * qq + 3] = bb.w;
      }
#pragma unroll
      for (int s = 0; s < kS1; ++s) {
        const int k = 2 * s + h;
        const float wa = k < S::F0 ? lds[S::L_W1 + (it * 32 + lr) * S::F0 + k] : 0.0f;
        t = mfma32(wa, xb[s], t);
      }
      return t;
    };
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      f32x16 t1 = l1(it);
#pragma unroll
      for (int j = 0; j < 16; ++j) t1[j] = relu(t1[j]);
      if (write_h1 && it == q) {
#pragma unroll
        for (int j = 0; j < 16; ++j)
          H1T[(it * 32 + acc_row(j, h)) * S::TS + rt * 32 + lr] = t1[j];
      }
      if (XH_ABL(a, 4)) continue;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const float4 a4 = lds4(wrow + it * 32 + 8 * qq);
        pre = mfma32(a4.x, t1[4 * qq + 0], pre);
        pre = mfma32(a4.y, t1[4 * qq + 1], pre);
        pre = mfma32(a4.z, t1[4 * qq + 2], pre);
        pre = mfma32(a4.w, t1[4 * qq + 3], pre);
      }
    }
    return pre;
  };
  // Layer-1 tile q of this wave's rows into the H1 image only: the same
  // operations as forward()'s it == q step, so the image is bit-identical
  // (128-row groups: the earlier half-group's H1 image is rebuilt from here
  // while its layer-2 pre-activations stay in registers).
  auto write_h1_tile = [&]() {
    float xb[S::S1];
#pragma unroll
    for (int s = 0; s < S::S1; ++s) xb[s] = fold_feat(2 * s + h);
    f32x16 t1;
    const float *bsrc = kFold ? lds + S::L_B1F + (item_b_grp ? S::H1 : 0)
                              : lds + S::L_B1;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const float4 bb = lds4(bsrc + q * 32 + 8 * qq + 4 * h);
      t1[4 * qq + 0] = bb.x;
      t1[4 * qq + 1] = bb.y;
      t1[4 * qq + 2] = bb.z;
      t1[4 * qq + 3] = bb.w;
    }
#pragma unroll
    for (int s = 0; s < kS1; ++s) {
      const int k = 2 * s + h;
      const float wa = k < S::F0 ? lds[S::L_W1 + (q * 32 + lr) * S::F0 + k] : 0.0f;
      t1 = mfma32(wa, xb[s], t1);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      H1T[(q * 32 + acc_row(j, h)) * S::TS + rt * 32 + lr] = relu(t1[j]);
  };

  if (HG == 1 && (int)blockIdx.x < ngroups) fetch_row(blockIdx.x, 0, bv_c, iv_c);
  constexpr int kDH1 = HG == 1 ? XH_V_DH1 : 0;
  constexpr bool kL3 = HG == 1 ? XH_V_L3 : XH_V_L3W;

  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int gi = (g - (int)blockIdx.x) / (int)gridDim.x;
    (void)gi;
    XH_STAMP(a, gi, w, lane, 0);
    const int gn = g + gridDim.x;
    if (HG == 1 && gn < ngroups) fetch_row(gn, 0, bv_n, iv_n);
    int c_cur;
    float po_cur, A_cur;
    {
      const int t = g / gpt, e0 = (g - t * gpt) * S::G;
      const size_t ti = (size_t)t * N + e0 + lane / (B <= 64 ? B : 64);
      c_cur = a.b.action[ti];
      po_cur = a.b.pold[ti];
      A_cur = a.adv[ti];
    }

    if (kFold && HG == 1) {  // bv_c / iv_c: this group's prefetched row
      bool is_a = true;
#pragma unroll
      for (int d = 0; d < S::D; ++d) is_a &= iv_c[d] == a.env.item_a[d];
      item_b_grp = !is_a;
    }
    // ---- forward (all R rows) -> per-tile partial logits in LDS
    f32x16 pre, pre0 = zero16();  // pre0: 128-row groups only
#pragma unroll
    for (int hg = 0; hg < HG; ++hg) {
      if (HG > 1) {
        fetch_row(g, hg, bv_c, iv_c);
        if (kFold && hg == 0) {  // the group's env (both halves)
          bool is_a = true;
#pragma unroll
          for (int d = 0; d < S::D; ++d) is_a &= iv_c[d] == a.env.item_a[d];
          item_b_grp = !is_a;
        }
      }
      // the last half-group's H1 image is written here; every half-group's
      // pre-activations stay in registers for the backward
      pre = forward(hg == HG - 1);
      if (HG > 1 && hg == 0) pre0 = pre;
      const float zp = logit_part<S, true>(lds, pre, q);
      if (lane < 32) lds[S::L_Z + q * R + hg * 64 + rt * 32 + lr] = zp;
    }
    XH_STAMP(a, gi, w, lane, 1);
    __syncthreads();
    XH_STAMP(a, gi, w, lane, 2);
    float4 w3v[4];
    if (kL3) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        w3v[qq] = lds4(lds + S::L_W3 + q * 32 + 8 * qq + 4 * h);
    }

    // ---- logits -> softmax -> loss gradient w.r.t. logits; lane holds the
    // rows lane + 64*k (k < HG)
    float gzk[HG];
    {
      constexpr int SEG = B <= 64 ? B : 64;
      float z[HG], ex[HG], p[HG];
      float se = 0.0f;
#pragma unroll
      for (int k = 0; k < HG; ++k) {
        const int r = k * 64 + lane;
        const float zs = ((lds[S::L_Z + r] + lds[S::L_Z + R + r]) +
                          lds[S::L_Z + 2 * R + r]) + lds[S::L_Z + 3 * R + r];
        z[k] = zs + lds[S::L_B3];
        ex[k] = __expf(z[k]);
        se += ex[k];
      }
      se = seg_sum<SEG>(se);
      // serial phase (no MFMA beside it): v_exp / v_rcp forms (<= 2 ulp)
      // instead of the IEEE sequences, well inside the 1e-4 parity bound
      const float rse = __builtin_amdgcn_rcpf(se);
#pragma unroll
      for (int k = 0; k < HG; ++k) p[k] = ex[k] * rse;
      const int c = c_cur;
      const float A = A_cur;
      const int seg0 = (lane / SEG) * SEG;
      // p of the chosen bin (bin c lives in lane c % 64 of row block c / 64)
      float pc = 0.0f;
      if constexpr (B == 64) {  // one env per wave: c is wave-uniform
        const int cu = __builtin_amdgcn_readfirstlane(c);
        pc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p[0]), cu));
      } else {
#pragma unroll
        for (int k = 0; k < HG; ++k) {
          const float v = wave_shfl(p[k], seg0 + (c % SEG));
          if (HG == 1 || c / 64 == k) pc = v;
        }
      }
#pragma unroll
      for (int k = 0; k < HG; ++k) {
        const int bin = (k * 64 + lane) % B;
        float gz;
        if (XH_ABL(a, 8)) {
          gz = z[k] * 1e-3f;
        } else if (a.algo == kPPO) {
          // clipped_gradient (rl.h:54-74) + softmax_layer::backward
          // (nn.h:393-417): gz_j = (diag(p) - p p^T)[j][c] * g_c
          const float ratio = pc * __builtin_amdgcn_rcpf(po_cur);
          float clipped = ratio;
          if (ratio > 1.0f + a.clip_eps)
            clipped = 1.0f + a.clip_eps;
          else if (ratio < 1.0f - a.clip_eps)
            clipped = 1.0f - a.clip_eps;
          const float ig = fminf(clipped * A, ratio * A) * -1.0f;
          const float gc = ig * __builtin_amdgcn_rcpf(pc);
          const float lin = bin == c ? p[k] : 0.0f;
          gz = (lin - p[k] * pc) * gc;
        } else {
          // softmax_gradient_log (rl.h:45-52) through softmax-xent (identity)
          gz = p[k] * A;
          if (bin == c) gz -= A;
        }
        gzk[k] = gz;
        if (w == 0) accB3 += gz;
      }
    }
    XH_STAMP(a, gi, w, lane, 3);

    // backward, last half-group first: it reuses the forward's registers and
    // H1 image; the earlier half-group keeps its layer-2 pre-activations in
    // registers and rebuilds only its H1 image (layer 1: a second 64-row
    // image does not fit in LDS beside W2 and the dA2 image)
#pragma unroll
    for (int hb = 0; hb < HG; ++hb) {
      const int hg = HG - 1 - hb;
      if (hb > 0) {
        __syncthreads();  // previous half-group's images consumed
        fetch_row(g, hg, bv_c, iv_c);
        write_h1_tile();  // the H1 image again (layer 1 only)
        pre = pre0;       // layer 2 kept from the forward
      }
      // ---- backward through layer 3 and the layer-2 relu
      {
        // row rt*32 + lr's gradient: own lane in half rt, else lane ^ 32
        const float sw = half_swap(gzk[hg]);
        const float gr = h == rt ? gzk[hg] : sw;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const float4 ww =
              kL3 ? w3v[qq] : lds4(lds + S::L_W3 + q * 32 + 8 * qq + 4 * h);
          const float wq[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = 4 * qq + u;
            const float v = pre[j];
            accW3[j] += gr * relu(v);
            const float d = v > 0.0f ? gr * wq[u] : 0.0f;
            if (!kB2Late) accB2[j] += d;
            DAT[(q * 32 + acc_row(j, h)) * S::TS + rt * 32 + lr] = d;
          }
        }
      }
      XH_STAMP(a, gi, w, lane, 4);
      __syncthreads();
      XH_STAMP(a, gi, w, lane, 5);

      // ---- dH1 tile q of r-tile rt (K = H2)
      f32x16 dh = zero16();
      auto dh1_step = [&](int s) {
        const int k = (kDH1 & 2) ? s + (S::H2 / 2) * h : 2 * s + h;
        dh = mfma32(lds[S::L_W2 + k * S::W2S + q * 32 + lr],
                    DAT[k * S::TS + rt * 32 + lr], dh);
      };
      if constexpr (kDH1 & 1) {
#pragma unroll
        for (int s = 0; s < S::H2 / 2; ++s) {
          if (XH_ABL(a, 16)) break;
          dh1_step(s);
        }
      } else {
        constexpr int kU = XH_V_DH1W;  // 128-row groups
#pragma unroll kU
        for (int s = 0; s < S::H2 / 2; ++s) {
          if (XH_ABL(a, 16)) break;
          dh1_step(s);
        }
      }
      XH_STAMP(a, gi, w, lane, 6);
      float xf[S::D];
#pragma unroll
      for (int f = 0; f < S::D; ++f) xf[f] = feat(f);
      bool item_is_a = true;
#pragma unroll
      for (int d = 0; d < S::D; ++d) item_is_a &= iv_c[d] == a.env.item_a[d];
      // d * 1 and d * 0 are exact: sA / sB take d or nothing
      const float fa = item_is_a ? 1.0f : 0.0f, fb = 1.0f - fa;
      const float *hcol = H1T + (q * 32) * S::TS + rt * 32 + lr;
      // ---- dW2 tiles (q, 2rt), (q, 2rt+1): K = 64 rows.  Step s gives lane
      // half h row 32h + s, so 4 consecutive steps are one ds_read_b128 of a
      // transposed image row (A: dA2 of H2 unit q*32+lr, B: H1 of unit i).
      // The dH1 tile's relu' / dW1 / db1 VALU work rides along, two
      // accumulator registers per 4-row step, in the MFMAs' shadow
      // (7.63 -> 7.44 ms per epoch against running it after dW2).
      constexpr int kUnrollW2 = S::HG > 1 ? XH_V_W2U : 8;
      const float *pa = DAT + (q * 32 + lr) * S::TS + 32 * h;
      const float *pb0 = H1T + ((2 * rt) * 32 + lr) * S::TS + 32 * h;
      const float *pb1 = H1T + ((2 * rt + 1) * 32 + lr) * S::TS + 32 * h;
#pragma unroll kUnrollW2
      for (int s4 = 0; s4 < 8; ++s4) {
        if (XH_ABL(a, 32)) break;
        const float4 av = lds4(pa + 4 * s4);
        const float4 b0 = lds4(pb0 + 4 * s4);
        const float4 b1 = lds4(pb1 + 4 * s4);
        if (kB2Late && (s4 >> 2) == rt) b2s += (av.x + av.y) + (av.z + av.w);
        accW2[0] = mfma32(av.x, b0.x, accW2[0]);
        accW2[1] = mfma32(av.x, b1.x, accW2[1]);
        accW2[0] = mfma32(av.y, b0.y, accW2[0]);
        accW2[1] = mfma32(av.y, b1.y, accW2[1]);
        accW2[0] = mfma32(av.z, b0.z, accW2[0]);
        accW2[1] = mfma32(av.z, b1.z, accW2[1]);
        accW2[0] = mfma32(av.w, b0.w, accW2[0]);
        accW2[1] = mfma32(av.w, b1.w, accW2[1]);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int j = 2 * s4 + jj;
          // relu' from the H1 image (post-relu > 0 <=> pre > 0)
          const float d = hcol[acc_row(j, h) * S::TS] > 0.0f ? dh[j] : 0.0f;
          if constexpr (kMW1) {
            dh[j] = d;  // dA1, imaged below
          } else {
            sA[j] = fmaf(d, fa, sA[j]);
            sB[j] = fmaf(d, fb, sB[j]);
#pragma unroll
            for (int f = 0; f < S::D; ++f) accW1[j][f] += d * xf[f];
          }
        }
      }
      XH_STAMP(a, gi, w, lane, 7);
      if constexpr (kMW1) {
        // ---- dW1 / db1 of this half-group by MFMA (see kMW1 above)
        __syncthreads();  // every wave is done with the H1 / dA2 images
        float *A1T = H1T;  // [H1][TS]: dA1 transposed (feature-major)
        float *XT = DAT;   // [F0 + 1][TS]: X transposed, row 2D = ones
#pragma unroll
        for (int j = 0; j < 16; ++j)
          A1T[(q * 32 + acc_row(j, h)) * S::TS + rt * 32 + lr] = dh[j];
        if (q == 0) {
#pragma unroll
          for (int f = 0; f < S::F0; ++f) XT[f * S::TS + rt * 32 + lr] = feat(f);
          XT[S::F0 * S::TS + rt * 32 + lr] = 1.0f;
        }
        __syncthreads();
        // wave w: feature tile i = 16w .. 16w+15; M = f (16, F0 + 1 used),
        // N = i, K = the 64 rows in 16 steps of 4 (lane quarter kq = row
        // 4s + kq): A[f][k] = X[row][f], B[k][i] = dA1[row][i]
        const int fi = lane & 15, kq = lane >> 4;
        const float *xa = XT + fi * S::TS + kq;
        const float *ab = A1T + (w * 16 + fi) * S::TS + kq;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const float av = fi <= S::F0 ? xa[4 * s] : 0.0f;
          accW1m = __builtin_amdgcn_mfma_f32_16x16x4f32(av, ab[4 * s], accW1m,
                                                       0, 0, 0);
        }
      }
    }
    __syncthreads();
    if (HG == 1) {
#pragma unroll
      for (int d = 0; d < S::D; ++d) {
        bv_c[d] = bv_n[d];
        iv_c[d] = iv_n[d];
      }
    }
  }

  // ---------------------------------------------------- slab write-out ----
  const PolicyLayout L{S::F0, S::H1, S::H2};
  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int it = 2 * rt + k;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int o2 = q * 32 + acc_row(j, h);
      slab[L.oW2() + o2 * S::H1 + it * 32 + lr] = accW2[k][j];
    }
  }
  float *scr = lds + S::L_H1T;  // [8][RED] wave partials (aliases the images)
  for (int i = threadIdx.x; i < 8 * S::RED; i += blockDim.x) scr[i] = 0.0f;
  __syncthreads();
  float *my = scr + w * S::RED;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    // sums over the 32 rows of each lane half (DPP: valid in lr >= 16)
    const float va = half_sum32(sA[j]), vb = half_sum32(sB[j]),
                vw3 = half_sum32(accW3[j]), vb2 = half_sum32(accB2[j]);
    float vw1[S::D];
#pragma unroll
    for (int f = 0; f < S::D; ++f) vw1[f] = half_sum32(accW1[j][f]);
    if (lr == 31) {
      const int i = q * 32 + acc_row(j, h);
      if constexpr (!kMW1) {
#pragma unroll
        for (int f = 0; f < S::D; ++f) my[i * S::F0 + f] = vw1[f];
#pragma unroll
        for (int d = 0; d < S::D; ++d)
          my[i * S::F0 + S::D + d] =
              va * ((float)a.env.item_a[d] / (float)kCapacity) +
              vb * ((float)a.env.item_b[d] / (float)kCapacity);
        my[S::H1 * S::F0 + i] = va + vb;
      }
      my[S::H1 * S::F0 + S::H1 + i] = vw3;  // o2 = q*32 + acc_row too
      if (!kB2Late) my[S::H1 * S::F0 + S::H1 + S::H2 + i] = vb2;
    }
  }
  if (kB2Late) {  // db2: lane halves hold the two 32-row halves of a unit
    const float v = b2s + __shfl_xor(b2s, 32, kWave);
    if (h == 0) my[S::H1 * S::F0 + S::H1 + S::H2 + q * 32 + lr] = v;
  }
  {
    float v = accB3;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o, kWave);
    if (lane == 0) my[S::RED - 1] = w == 0 ? v : 0.0f;
  }
  __syncthreads();
  if constexpr (kMW1) {  // dW1^T tile of wave w: rows f = 4 kq + r, col i
    const int fi = lane & 15, kq = lane >> 4, i = w * 16 + fi;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * kq + r;
      if (f < S::F0)
        slab[L.oW1() + i * S::F0 + f] = accW1m[r];
      else if (f == S::F0)
        slab[L.ob1() + i] = accW1m[r];
    }
  }
  for (int i = threadIdx.x; i < S::RED; i += blockDim.x) {
    if (kMW1 && i < S::H1 * S::F0 + S::H1) continue;  // written above
    float v = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) v += scr[k * S::RED + i];
    int dst;
    if (i < S::H1 * S::F0)
      dst = L.oW1() + i;
    else if (i < S::H1 * S::F0 + S::H1)
      dst = L.ob1() + (i - S::H1 * S::F0);
    else if (i < S::H1 * S::F0 + S::H1 + S::H2)
      dst = L.ow3() + (i - S::H1 * S::F0 - S::H1);
    else if (i < S::RED - 1)
      dst = L.ob2() + (i - S::H1 * S::F0 - S::H1 - S::H2);
    else
      dst = L.ob3();
    slab[dst] = v;
  }
}

// ================================================================ dispatch ==
#define XH_POLICY_SHAPES(X) \
  X(8, 2, 128, 64)          \
  X(8, 2, 64, 32)           \
  X(16, 2, 64, 64)          \
  X(32, 1, 64, 64)          \
  X(64, 2, 128, 128)        \
  X(128, 3, 128, 128)

#ifndef XH_TRAIN4
#define XH_TRAIN4 0  // 1: force the 4-wave train kernel everywhere (A/B)
#endif

template <class S>
constexpr size_t rollout_lds() {
  return sizeof(float) * S::L_ROLLOUT_END;
}
template <class S>
constexpr size_t train_lds() {
  return sizeof(float) *
         (S::L_TRAIN_END > S::L_TRAIN8_END ? S::L_TRAIN_END : S::L_TRAIN8_END);
}

// XH_ROLLOUT_KERNEL=4 keeps the 4-wave rollout where the wave-per-env kernel
// would run (A/B measurements and the bit-identity test); read per launch.
static bool rollout4() {
  const char *e = std::getenv("XH_ROLLOUT_KERNEL");
  return e && std::atoi(e) == 4;
}
// XH_ROLLOUT_KERNEL=f32 keeps the f32-MFMA wave rollouts where the
// bf16-split ones would run (64 / 128 bins, [128,128]); read per launch.
static bool rollout_split() {
  const char *e = std::getenv("XH_ROLLOUT_KERNEL");
  return !(e && (e[0] == 'f' || std::atoi(e) == 4));
}

bool policy_shape_supported(int B, int D, int H1, int H2) {
#define X(XB, XD, XH1, XH2) \
  if (B == XB && D == XD && H1 == XH1 && H2 == XH2) return true;
  XH_POLICY_SHAPES(X)
#undef X
  return false;
}

static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
            hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

int rollout_grid(int B, int D, int H1, int H2) {
  (void)B; (void)D; (void)H1; (void)H2;
  return 2 * cu_count();
}
int policy_train_grid(int B, int D, int H1, int H2, int kl) {
  // the wave-specialised config-2 kernel (opt-in): one 8-wave workgroup per CU
  if (train_spec4_default(B, D, H1, H2, kl)) return cu_count();
#define X(XB, XD, XH1, XH2)                                     \
  if (B == XB && D == XD && H1 == XH1 && H2 == XH2) {          \
    using S = PShape<XB, XD, XH1, XH2>;                         \
    (void)kl;                                                   \
    return (S::NIT == 4 && S::NOT == 4) ? cu_count()            \
                                        : S::TOCC * cu_count(); \
  }
  XH_POLICY_SHAPES(X)
#undef X
  return cu_count();
}

// Whether launch_rollout_one would run a register-stepping split kernel for
// a (which applies src_slot as it fetches).
static bool rollout_fetch_shifts(const RolloutArgs &a, int H1, int H2) {
  if (!rollout_split() || a.wide) return false;
  const int B = a.env.B;
  return (B == 64 && H1 == 128 && H2 == 128) || (B == 32 && H1 == 64 && H2 == 64) ||
         (B == 128 && H1 == 128 && H2 == 128);
}

// One launch: slot a.t (multi = false), or slots a.t .. a.t + a.nsteps - 1
// by the register-stepping split kernel (multi = true).
static hipError_t launch_rollout_one(const RolloutArgs &a, int H1, int H2,
                                     int grid, hipStream_t s, KernelInfo *info,
                                     bool &multi) {
  const int B = a.env.B, D = a.env.D;
  multi = false;
  info->math = kMathF32Mfma;
#define X(XB, XD, XH1, XH2)                                                  \
  if (B == XB && D == XD && H1 == XH1 && H2 == XH2) {                        \
    using S = PShape<XB, XD, XH1, XH2>;                                      \
    static bool attr = false;                                                \
    if (!attr) {                                                             \
      if constexpr (S::HG == 1)                                              \
        (void)hipFuncSetAttribute((const void *)rollout_step_kernel<S>,      \
                                  hipFuncAttributeMaxDynamicSharedMemorySize,\
                                  (int)rollout_lds<S>());                    \
      else                                                                   \
        (void)hipFuncSetAttribute((const void *)rollout_step128_kernel<S>,   \
                                  hipFuncAttributeMaxDynamicSharedMemorySize,\
                                  (int)rollout_lds<S>());                    \
      attr = true;                                                           \
    }                                                                        \
    const int ng = a.b.N / S::G;                                             \
    if constexpr (S::B == 128 && S::NIT == 4 && S::NOT == 4) {               \
      if (rollout_split() && !a.wide) {                                      \
        static bool sattr = false;                                           \
        if (!sattr) {                                                        \
          (void)hipFuncSetAttribute((const void *)rollout_split128_kernel<S>,\
                                    hipFuncAttributeMaxDynamicSharedMemorySize,\
                                    (int)RollSplitLds<S>::bytes);            \
          sattr = true;                                                      \
        }                                                                    \
        constexpr int kRW = kRollWavesS128;                                  \
        const int wg = (a.b.N + kRW - 1) / kRW;                              \
        const int wgr = cu_count();                                          \
        info->name = "rollout_split128_kernel";                              \
        info->math = kMathSplitRollout;                                      \
        multi = true;                                                        \
        hipLaunchKernelGGL(rollout_split128_kernel<S>,                       \
                           dim3(wgr < wg ? wgr : wg), dim3(64 * kRW),        \
                           RollSplitLds<S>::bytes, s, a);                    \
        return hipGetLastError();                                            \
      }                                                                      \
    }                                                                        \
    if constexpr (S::B == 128 && S::NIT == 4 && S::NOT == 4) {               \
      if (!rollout4()) {                                                     \
        static bool wattr = false;                                           \
        if (!wattr) {                                                        \
          (void)hipFuncSetAttribute((const void *)rollout_wave128_kernel<S>, \
                                    hipFuncAttributeMaxDynamicSharedMemorySize,\
                                    (int)rollout_lds<S>());                  \
          wattr = true;                                                      \
        }                                                                    \
        constexpr int kRW = kRollWaves128;                                   \
        const int wg = (a.b.N + kRW - 1) / kRW;                              \
        const int wgr = kRW == 8 ? grid : cu_count();                        \
        info->name = "rollout_wave128_kernel";                               \
        hipLaunchKernelGGL(rollout_wave128_kernel<S>,                        \
                           dim3(wgr < wg ? wgr : wg), dim3(64 * kRW),        \
                           rollout_lds<S>(), s, a);                          \
        return hipGetLastError();                                            \
      }                                                                      \
    }                                                                        \
    if constexpr ((S::B == 64 && S::NIT == 4 && S::NOT == 4) ||             \
                  (S::B == 32 && S::NIT == 2 && S::NOT == 2)) {              \
      if (rollout_split() && !a.wide) {                                      \
        static bool sattr = false;                                           \
        if (!sattr) {                                                        \
          (void)hipFuncSetAttribute((const void *)rollout_split_kernel<S>,   \
                                    hipFuncAttributeMaxDynamicSharedMemorySize,\
                                    (int)RollSplitLds<S>::bytes);               \
          sattr = true;                                                      \
        }                                                                    \
        constexpr int kRW = roll_split_waves<S>();                           \
        const int wg = (ng + kRW - 1) / kRW;                                 \
        /* 64 bins: one 12-wave workgroup per CU; 32 bins: every group's  */ \
        /* wave resident at once (2048 groups at config 2)                */ \
        const int wgr = S::B == 64 ? (kRW == 8 ? grid : cu_count()) : wg;    \
        info->name = "rollout_split_kernel";                                 \
        info->math = kMathSplitRollout;                                      \
        multi = true;                                                        \
        hipLaunchKernelGGL(rollout_split_kernel<S>,                          \
                           dim3(wgr < wg ? wgr : wg), dim3(64 * kRW),        \
                           RollSplitLds<S>::bytes, s, a);                       \
        return hipGetLastError();                                            \
      }                                                                      \
    }                                                                        \
    if constexpr (S::B == 64 && S::NIT == 4 && S::NOT == 4) {                \
      if (!rollout4()) {                                                     \
        static bool wattr = false;                                           \
        if (!wattr) {                                                        \
          (void)hipFuncSetAttribute((const void *)rollout_wave_kernel<S>,    \
                                    hipFuncAttributeMaxDynamicSharedMemorySize,\
                                    (int)rollout_lds<S>());                  \
          wattr = true;                                                      \
        }                                                                    \
        constexpr int kRW = kRollWaves64;                                    \
        const int wg = (ng + kRW - 1) / kRW;                                 \
        const int wgr = kRW == 8 ? grid : cu_count();                        \
        info->name = "rollout_wave_kernel";                                  \
        hipLaunchKernelGGL(rollout_wave_kernel<S>,                           \
                           dim3(wgr < wg ? wgr : wg), dim3(64 * kRW),        \
                           rollout_lds<S>(), s, a);                          \
        return hipGetLastError();                                            \
      }                                                                      \
    }                                                                        \
    info->name = S::HG == 1 ? "rollout_step_kernel" : "rollout_step128_kernel";\
    if constexpr (S::HG == 1)                                                \
      hipLaunchKernelGGL(rollout_step_kernel<S>, dim3(grid < ng ? grid : ng),\
                         dim3(256), rollout_lds<S>(), s, a);                 \
    else                                                                     \
      hipLaunchKernelGGL(rollout_step128_kernel<S>,                          \
                         dim3(grid < ng ? grid : ng), dim3(256),             \
                         rollout_lds<S>(), s, a);                            \
    return hipGetLastError();                                                \
  }
  XH_POLICY_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_rollout_step(const RolloutArgs &a, int H1, int H2, int grid,
                               hipStream_t s, KernelInfo *info) {
  KernelInfo dummy;
  if (!info) info = &dummy;
  const int n = a.nsteps > 1 ? a.nsteps : 1;
  bool multi = false;
  if (a.src_slot > 0 && !rollout_fetch_shifts(a, H1, H2)) {
    // the one-slot kernels read slot 0 as it is: copy slot src_slot there
    const size_t N = (size_t)a.b.N, BD = (size_t)a.env.B * a.env.D;
    hipError_t e = hipMemcpyAsync(a.b.bins, a.b.bins + (size_t)a.src_slot * N * BD,
                                  N * BD, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess)
      e = hipMemcpyAsync(a.b.items, a.b.items + (size_t)a.src_slot * N * 4, N * 4,
                         hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    RolloutArgs a0 = a;
    a0.src_slot = -1;
    return launch_rollout_step(a0, H1, H2, grid, s, info);
  }
  hipError_t e = launch_rollout_one(a, H1, H2, grid, s, info, multi);
  // a one-slot kernel ran slot a.t (its logits / probabilities are rewritten
  // by the later slots'); the rest in one launch if the kernel allows
  for (int k = 1; e == hipSuccess && !multi && k < n; ++k) {
    RolloutArgs ak = a;
    ak.t = a.t + k;
    ak.nsteps = n - k;
    ak.wide = 0;  // `wide` describes slot a.t only
    ak.src_slot = -1;
    e = launch_rollout_one(ak, H1, H2, grid, s, info, multi);
  }
  return e;
}

hipError_t launch_eval_argmax(const EvalArgs &a, int H1, int H2,
                              hipStream_t s) {
  const int B = a.env.B, D = a.env.D;
#define X(XB, XD, XH1, XH2)                                                  \
  if (B == XB && D == XD && H1 == XH1 && H2 == XH2) {                        \
    using S = PShape<XB, XD, XH1, XH2>;                                      \
    if constexpr (S::HG == 1) {                                              \
      constexpr size_t bytes =                                               \
          rollout_lds<S>() + sizeof(int) * (S::G * (S::BD + 4 + 2) + 4);     \
      static bool attr = false;                                              \
      if (!attr) {                                                           \
        (void)hipFuncSetAttribute((const void *)eval_argmax_kernel<S>,       \
                                  hipFuncAttributeMaxDynamicSharedMemorySize,\
                                  (int)bytes);                               \
        attr = true;                                                         \
      }                                                                      \
      const int ng = a.n_envs / S::G;                                        \
      hipLaunchKernelGGL(eval_argmax_kernel<S>,                              \
                         dim3(ng < 1024 ? ng : 1024), dim3(256), bytes, s, a);\
      return hipGetLastError();                                              \
    }                                                                        \
  }
  XH_POLICY_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_policy_train(const PolicyTrainArgs &a, int H1, int H2,
                               int grid, hipStream_t s, KernelInfo *info) {
  const int B = a.env.B, D = a.env.D;
  KernelInfo dummy;
  if (!info) info = &dummy;
  info->math = kMathF32Mfma;
  if (policy_train_split_supported(a, H1, H2) && train_split_enabled() &&
      !a.wide)
    return launch_policy_train_split(a, grid, s, info);
#define X(XB, XD, XH1, XH2)                                                  \
  if (B == XB && D == XD && H1 == XH1 && H2 == XH2) {                        \
    using S = PShape<XB, XD, XH1, XH2>;                                      \
    static bool attr = false;                                                \
    if (!attr) {                                                             \
      if constexpr (S::HG == 1) {                                            \
        (void)hipFuncSetAttribute((const void *)policy_train_kernel<S, false>,\
                                  hipFuncAttributeMaxDynamicSharedMemorySize,\
                                  (int)train_lds<S>());                      \
        (void)hipFuncSetAttribute((const void *)policy_train_kernel<S, true>,\
                                  hipFuncAttributeMaxDynamicSharedMemorySize,\
                                  (int)train_lds<S>());                      \
      }                                                                      \
      if constexpr (S::NIT == 4 && S::NOT == 4)                              \
        (void)hipFuncSetAttribute((const void *)policy_train8_kernel<S>,     \
                                  hipFuncAttributeMaxDynamicSharedMemorySize,\
                                  (int)train_lds<S>());                      \
      attr = true;                                                           \
    }                                                                        \
    if (a.algo == kKLPPO) {                                                  \
      info->name = "policy_train_kernel<kl>";                                \
      if constexpr (S::HG == 1)                                              \
        hipLaunchKernelGGL((policy_train_kernel<S, true>), dim3(grid),       \
                           dim3(256), train_lds<S>(), s, a);                 \
      else                                                                   \
        return hipErrorInvalidValue;                                         \
      return hipGetLastError();                                              \
    }                                                                        \
    info->name = (S::NIT == 4 && S::NOT == 4 && (!XH_TRAIN4 || S::HG > 1))   \
                     ? "policy_train8_kernel" : "policy_train_kernel";       \
    if constexpr (S::NIT == 4 && S::NOT == 4 && (!XH_TRAIN4 || S::HG > 1))  \
      hipLaunchKernelGGL(policy_train8_kernel<S>, dim3(grid), dim3(512),     \
                         train_lds<S>(), s, a);                              \
    else if constexpr (S::HG == 1)                                           \
      hipLaunchKernelGGL((policy_train_kernel<S, false>), dim3(grid),        \
                         dim3(256), train_lds<S>(), s, a);                   \
    return hipGetLastError();                                                \
  }
  XH_POLICY_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace xh
