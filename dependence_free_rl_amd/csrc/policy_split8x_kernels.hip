// policy_split8x_kernels.hip -- the actor-critic / PPO train epoch of the
// 128-bin 3-D [128,128] policy (BASELINE config 5): the pipelined 8-wave
// kernel of policy_split8wh_kernels.hip (f16 pairs for layer 2 and dH1, the
// exact bf16 split for dW2, rank-1 backward; see its header and xh_split.h)
// for envs of 128 rows, processed as 64-row half-groups ("units": unit u is
// half u & 1 of the workgroup's env u >> 1).
//
// The softmax couples an env's two units, so the pipeline runs layer 2 two
// units ahead.  Iteration v (the backward of unit v):
//
//   X(v): MFMA  layer 2 of unit v+2 (48 f16 MFMAs per wave)
//         VALU  at an env's first unit (v even) the 128-bin softmax and loss
//               gradient of the env (its two units' partial logits are in
//               LDS: unit v+1's layer 2 ran in X(v-1)); unit v's relu masks
//               (images), dW3 / db2 sums, g (x) H1 of its K-step 0; then unit
//               v+2's partial logits                         -> barrier
//   Y(v): MFMA  dW2 (bf16 split) and dH1 (f16 pairs) of unit v
//         VALU  g (x) H1 of K-step 1, layer 1 of unit v+3 (-> the H1 image),
//               dW1 / db1 / item sums of unit v            -> barrier
//
// Three units' pre-activations are live (v: its masks in X(v); v+1 waiting;
// v+2 accumulating).  Wave 0 stages unit v+3 during X(v): its 64 rows' bins
// and its env's record (action 0..127, old probability, advantage, item).
// Layouts, swizzles and operand maps as variants/policy_split8wp_kernels.hip.
#include <cstdlib>

#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

// Built twice (Makefile), as policy_split8wh_kernels.hip: the actor-critic /
// PPO kernel, and with XH_8X_KL_TU=1 (policy_split8x_kl_kernels.o) its
// KL-PPO form, policy_train_split8x_kl_kernel.  The KL additions are
// preprocessor blocks, so the first object compiles from exactly its
// measured source.
#ifndef XH_8X_KL_TU
#define XH_8X_KL_TU 0
#endif
#if XH_8X_KL_TU
#define KLTU(...) __VA_ARGS__
#else
#define KLTU(...)
#endif

namespace xh {
namespace s8x {

constexpr int kB = 128, kD = 3, kF0 = 2 * kD, kH = 128;
constexpr int kThreads = 512;
constexpr int kImg = 64 * kImgRow;  // one 64-row part image, 16 KB
// LDS carve (bytes): the H1 image (two f16 parts, scaled by S_H), the mask
// image as bf16 (dW2's A operand) and as f16 (dH1's A operand), the lo parts
// of every lane's W2 / W2' f16-pair fragments (register pressure: each lane
// reads back its own 16 bytes, [wave][K-slice][lane]), then f32
constexpr int L_H1 = 0;
constexpr int L_MASK = 2 * kImg;
constexpr int L_MASKH = 3 * kImg;
constexpr int L_WLO = 4 * kImg;
constexpr int L_WDLO = 6 * kImg;
constexpr int L_F = 8 * kImg;
constexpr int F_W1T = 0;                // [3 k][128 i]: W1[i][k], the bin columns
constexpr int F_B1F = F_W1T + 3 * kH;   // [2 items][128]: b1 + the item's part
constexpr int F_B2 = F_B1F + 2 * kH;    // [128] b2 S_W S_H
constexpr int F_W3 = F_B2 + kH;         // [128] w3 / (S_W S_H)
constexpr int F_B3 = F_W3 + kH;         // [4]
constexpr int F_Z = F_B3 + 4;           // [2 env parity][2 halves][64 rows][8 waves]
constexpr int F_GW = F_Z + 2 * 2 * 64 * 8;  // [8 waves][2 unit parity][64 rows] g
constexpr int F_GP = F_GW + 8 * 2 * 64;     // [8 waves][2][16 li][4 rt] g, C-layout order
constexpr int F_X = F_GP + 8 * 2 * 64;      // [4 slots][3 dims][64 rows] bins / 8
constexpr int F_XP = F_X + 4 * kD * 64;     // [4 slots][3 dims][16 li][4 rt]
constexpr int F_IT = F_XP + 4 * kD * 64;    // [4 slots] the unit's item is item_a
constexpr int F_REC = F_IT + 4;             // [4 slots][action, pold, adv, -]
constexpr int F_SC = F_REC + 4 * 4;         // [16] the scales' reduction
#if XH_8X_KL_TU
constexpr int F_Q = F_SC + 16;              // KL-PPO: [4 slots][64 rows] old distribution
constexpr int F_END = F_Q + 4 * 64;
#else
constexpr int F_END = F_SC + 16;
#endif
constexpr size_t kLds = L_F + sizeof(float) * F_END;
static_assert(kLds <= 160 * 1024, "LDS");
static_assert(F_REC % 4 == 0 && F_GW % 4 == 0 && F_GP % 4 == 0 && F_X % 4 == 0 &&
                  F_XP % 4 == 0 && F_Z % 4 == 0 && F_W1T % 4 == 0 && F_B1F % 4 == 0 &&
                  F_B2 % 4 == 0 && F_W3 % 4 == 0,
              "16-byte aligned f32 vectors");

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x8 lbf16x8;
typedef __attribute__((address_space(3))) bf16x4 lbf16x4;
typedef __attribute__((address_space(3))) s16x4 ls16x4;

typedef __attribute__((address_space(3))) f16x8 lf16x8;
typedef __attribute__((address_space(3))) f16x4 lf16x4;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16h(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16x8 ld8h(int off) {
  return *(const lf16x8 *)(size_t)(unsigned)off;
}
__device__ __forceinline__ void st4h(int off, f16x4 v) {
  *(lf16x4 *)(size_t)(unsigned)off = v;
}
// image accesses at absolute LDS byte addresses
__device__ __forceinline__ bf16x8 ld8(int off) {
  return *(const lbf16x8 *)(size_t)(unsigned)off;
}
__device__ __forceinline__ void st4(int off, bf16x4 v) {
  *(lbf16x4 *)(size_t)(unsigned)off = v;
}
// two ds_read_b64_tr_b16 (EXEC full): elements 0-3 from o0, 4-7 from o1
__device__ __forceinline__ bf16x8 ldtr(int o0, int o1) {
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ls16x4 *)(size_t)(unsigned)o0);
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ls16x4 *)(size_t)(unsigned)o1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// the images' swizzle: chunk ^= swz2(row & 15)
__device__ __forceinline__ constexpr int swz2(int r) {
  return ((r & 7) << 1) ^ ((r & 8) ? 9 : 0);
}
__device__ __forceinline__ int ioff2(int row, int ch) {
  return kImgRow * row + 16 * (ch ^ swz2(row & 15));
}
// row reads: lane (G, li) reads row 16 rt + li, chunk 4s + G at
// (rd_base ^ 64 s) + 4096 rt
__device__ __forceinline__ int rd_base(int G, int li) {
  return kImgRow * li + 16 * (G ^ swz2(li));
}
// dW2's A operand M^T by transposed reads: K-step ks element j of lane group
// G is row 32 ks + 4G + j (j < 4) or 32 ks + 16 + 4G + j - 4 (the T layout's
// r-tiles 2 ks, 2 ks + 1); read t: lane 4q + p supplies row 16t + 4G + q,
// columns 16 ot + 4p .. +3, at (trm_base(t) ^ 32 ot) + 8192 ks
__device__ __forceinline__ int trm_base(int l, int t) {
  const int G = l >> 4, li = l & 15, q = li >> 2, p = li & 3;
  const int row = 16 * t + 4 * G + q;
  return kImgRow * row + 16 * ((p >> 1) ^ swz2(row & 15)) + 8 * (p & 1);
}
// stores from the C layout (row 16 rt + li, features 16 ft + 4G .. +3):
// (st_base ^ 32 ft) + 4096 rt
__device__ __forceinline__ int st_base(int G, int li) {
  return kImgRow * li + 16 * ((G >> 1) ^ swz2(li)) + 8 * (G & 1);
}
__device__ __forceinline__ f32x4 lds4v(const float *p) {
  return *reinterpret_cast<const f32x4 *>(p);
}
__device__ __forceinline__ float relu(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}
// relu'(x) in {0, 1} from x's bits: v_med3_i32(bits, 0, 1) (a compare would
// write VCC, and its consumer would wait the VCC hazard's s_nop)
__device__ __forceinline__ int relu_bit(float x) {
  int m;
  asm("v_med3_i32 %0, %1, 0, 1" : "=v"(m) : "v"(__float_as_int(x)));
  return m;
}
// the integer relu masks of policy_split8wh_kernels.hip: here the inline asm
// costs 74 spilled registers (4.88 -> 33.6 ms per epoch): off
#ifndef XH_8X_IMASK
#define XH_8X_IMASK 0
#endif
// sum over the four lane groups (rows of 16 lanes) without an LDS round
// trip: ((g0 + g1) + (g2 + g3)) in every lane, as two __shfl_xor steps
__device__ __forceinline__ float sum_groups(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v),
                                                  false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v),
                                                  false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
#define FENCE() __builtin_amdgcn_sched_barrier(0)

#if XH_8X_KL_TU
// kl_ppo_learner's epoch over every row of its state matrix, as
// policy_split8wh_kernels.hip's KL build: envs 0..TN-1 the transitions,
// TN..TN+N-1 the open trajectories' end rows, then the n_end terminal end
// rows of end_list; the two 64-row units of an env stage their halves of q.
__global__ __launch_bounds__(kThreads, 2) void policy_train_split8x_kl_kernel(
#else
__global__ __launch_bounds__(kThreads, 2) void policy_train_split8x_kernel(
#endif
    PolicyTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH, kH};
  const float *P = a.params;
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int l = tid & 63, G = l >> 4, li = l & 15;
#if XH_8X_KL_TU
  const int NT = a.b.T * a.b.N;
  const int n_end = *a.n_end;
  const int nenv = NT + a.b.N + n_end;
  const float beta = *a.beta;
#else
  const int nenv = a.b.T * a.b.N;
#endif
  // this workgroup's envs: e_j = blockIdx.x + j gridDim.x, j < J (the host
  // caps the grid at the env count); units u < U = 2 J, u >> 1 the env, u & 1
  // the half; units past the end are clamped to the last one (layer 1 /
  // layer 2 run ahead; their work is discarded)
  const int J = (int)blockIdx.x < nenv
                    ? (nenv - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x
                    : 0;
  if (J == 0) return;  // uniform over the workgroup
  const int U = 2 * J;
  int gstep = (int)gridDim.x;
  // env (transition) index of unit u: its row of the [T][N] arrays
  auto tindex = [&](int u) {
    return (size_t)((int)blockIdx.x + (min(u, U - 1) >> 1) * gstep);
  };
  auto uhalf = [&](int u) { return min(u, U - 1) & 1; };

  // ---- prologue: the scales (every workgroup the same), small parameters,
  // the W2 / W2' fragments of tile w as f16 pairs
  {
    float mw = 0.0f, md = 0.0f, mh = 0.0f;
    for (int e = tid; e < kH * kH; e += kThreads) {
      const float v = P[PL.oW2() + e];
      mw = fmaxf(mw, fabsf(v));
      md = fmaxf(md, fabsf(v * P[PL.ow3() + (e >> 7)]));
    }
    if (tid < kH) {
      float ba = P[PL.ob1() + tid], bb = ba, ws = 0.0f;
#pragma unroll
      for (int d = 0; d < kD; ++d) {
        const float wv = P[PL.oW1() + tid * kF0 + kD + d];
        ba += wv * ((float)a.env.item_a[d] / (float)kCapacity);
        bb += wv * ((float)a.env.item_b[d] / (float)kCapacity);
        ws += fabsf(P[PL.oW1() + tid * kF0 + d]);
      }
      mh = ws + fmaxf(fabsf(ba), fabsf(bb));
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      mw = fmaxf(mw, __shfl_xor(mw, o, kWave));
      md = fmaxf(md, __shfl_xor(md, o, kWave));
      mh = fmaxf(mh, __shfl_xor(mh, o, kWave));
    }
    if (l == 0) {
      lf[F_SC + w] = mw;
      lf[F_SC + 8 + w] = md;
    }
    __syncthreads();
    float MW = 0.0f, MD = 0.0f;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      MW = fmaxf(MW, lf[F_SC + v]);
      MD = fmaxf(MD, lf[F_SC + 8 + v]);
    }
    __syncthreads();
    if (l == 0 && w < 2) lf[F_SC + w] = mh;  // waves 0-1 hold the 128 features
    __syncthreads();
    const float MH = fmaxf(lf[F_SC + 0], lf[F_SC + 1]);
    __syncthreads();
    if (tid == 0) {
      lf[F_SC + 0] = f16_scale_for(MW);  // S_W
      lf[F_SC + 1] = f16_scale_for(MD);  // S_D
      lf[F_SC + 2] = f16_scale_for(MH);  // S_H
    }
    __syncthreads();
  }
  const float SW = lf[F_SC + 0], SD = lf[F_SC + 1], SH = lf[F_SC + 2];
  const float S2 = SW * SH;  // layer 2's pre-activations are in units of S2
  for (int e = tid; e < kD * kH; e += kThreads) {
    const int k = e / kH, i = e - k * kH;
    lf[F_W1T + e] = P[PL.oW1() + i * kF0 + k];
  }
  for (int e = tid; e < 2 * kH; e += kThreads) {
    const int it = e / kH, u = e - it * kH;
    const int *item = it == 0 ? a.env.item_a : a.env.item_b;
    float v = P[PL.ob1() + u];
#pragma unroll
    for (int d = 0; d < kD; ++d)
      v += P[PL.oW1() + u * kF0 + kD + d] * ((float)item[d] / (float)kCapacity);
    lf[F_B1F + e] = v;
  }
  for (int i = tid; i < kH; i += kThreads) {
    lf[F_B2 + i] = P[PL.ob2() + i] * S2;
    lf[F_W3 + i] = P[PL.ow3() + i] * (1.0f / S2);
  }
  if (tid == 0) lf[F_B3] = P[PL.ob3()];
  f16x8 wl[4], wd[4];  // the hi parts; the lo parts in LDS (L_WLO, L_WDLO)
  const int rdb0 = rd_base(G, li);
  const int flo0 = 4096 * w + 16 * l;  // this lane's lo fragments: + 1024 s
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float4 *src = reinterpret_cast<const float4 *>(
        P + PL.oW2() + (16 * w + li) * kH + 32 * s + 8 * G);
    const float4 v0 = src[0], v1 = src[1];
    const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    f16x8 lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 x0, x1;
      split2h(v[j] * SW, x0, x1);
      wl[s][j] = x0;
      lo[j] = x1;
    }
    *reinterpret_cast<f16x8 *>(lds + L_WLO + flo0 + 1024 * s) = lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = 32 * s + 8 * G + j, col = 16 * w + li;
      _Float16 x0, x1;
      split2h((P[PL.oW2() + o * kH + col] * P[PL.ow3() + o]) * SD, x0, x1);
      wd[s][j] = x0;
      lo[j] = x1;
    }
    *reinterpret_cast<f16x8 *>(lds + L_WDLO + flo0 + 1024 * s) = lo;
  }
  const int trm00 = trm_base(l, 0), trm10 = trm_base(l, 1);  // ^ 32 ot, + L_MASK
  const int stb0 = st_base(G, li) ^ (32 * w);  // + L_H1 / L_MASK + 4096 rt
  const int fo = 16 * w + 4 * G;  // this lane's 4 features in the C layout
  float *const gwb = lf + F_GW + 128 * w;  // this wave's copies of the rows' g
  float *const gpb = lf + F_GP + 128 * w;

  f32x4 accW2[8];
#pragma unroll
  for (int ot = 0; ot < 8; ++ot)
#pragma unroll
    for (int j = 0; j < 4; ++j) accW2[ot][j] = 0.0f;
  float accW3[4] = {0.0f, 0.0f, 0.0f, 0.0f}, accB2[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float accB3 = 0.0f, w0 = 0.0f, w1 = 0.0f, w2 = 0.0f, sa = 0.0f, sb = 0.0f;
#if XH_8X_KL_TU
  double kl_acc = 0.0;  // sum of KL(q || p) over this wave's rows
#endif

  // wave 0 stages unit u: branch-free loads (lane = row: the row's three
  // bins as a byte triple; lanes 0-2 the env's action, old probability and
  // advantage, the others the item's coordinates), then the stores into
  // slot u & 3 (bins / 8 in row order and in the C layout's order, whether
  // the item is item_a, the record)
#if XH_8X_KL_TU
  struct Raw {
    int bi, rec;
    float q;     // the old distribution's entry of row l of the unit
    int ended;   // open end rows: step T - 1 of the env ended
  };
  // the row of the [T+1][N] arrays env g reads and the row of its old
  // distribution (kind 0 transition, 1 open end row, 2 terminal end row)
  auto kl_rows = [&](int g, size_t &ti, size_t &qi) {
    const int N = a.b.N;
    g = __builtin_amdgcn_readfirstlane(g);
    if (g < NT) {
      ti = qi = (size_t)g;
    } else if (g < NT + N) {
      ti = (size_t)NT + (g - NT);
      qi = (size_t)(NT - N) + (g - NT);
    } else {
      const int jj = min(g - NT - N, max(n_end - 1, 0));
      const int te = __builtin_amdgcn_readfirstlane(a.end_list[jj]);
      ti = qi = (size_t)te;
    }
  };
  auto stage_load = [&](int u) {
    size_t ti = tindex(u), qi = 0;
    kl_rows((int)ti, ti, qi);
    const size_t ri = qi;
#else
  struct Raw {
    int bi, rec;
  };
  auto stage_load = [&](int u) {
    const size_t ti = tindex(u);
    const size_t ri = ti;
#endif
    int lo = (uhalf(u) * 64 + l) * kD;
    asm volatile("" : "+v"(lo));
    const unsigned char *bp = reinterpret_cast<const unsigned char *>(
        a.b.bins + ti * (kB * kD) + lo);
    const int bins = (int)bp[0] | ((int)bp[1] << 8) | ((int)bp[2] << 16);
    const int *src = l == 0   ? a.b.action + ri
                     : l == 1 ? reinterpret_cast<const int *>(a.b.pold + ri)
                     : l == 2 ? reinterpret_cast<const int *>(a.adv + ri)
                              : reinterpret_cast<const int *>(a.b.items + ti * 4);
#if XH_8X_KL_TU
    Raw r{bins, *src, a.qold[qi * kB + uhalf(u) * 64 + l], 0};
    const int g = __builtin_amdgcn_readfirstlane((int)tindex(u));
    if (g >= NT && g < NT + a.b.N) r.ended = a.b.done[qi];
    return r;
  };
  auto stage_store = [&](const Raw &r, int s, int u) {
    const int g = __builtin_amdgcn_readfirstlane((int)tindex(u));
    const int kind = g < NT ? 0 : g < NT + a.b.N ? 1 : 2;
    // the terminal view: the chosen bin without the item (rl.h:336-343)
    const int itm = __builtin_amdgcn_readlane(r.rec, 3);
    const bool sub = kind == 2 && uhalf(u) * 64 + l == __builtin_amdgcn_readfirstlane(r.rec);
    lf[F_Q + s * 64 + l] = r.q;
#else
    return Raw{bins, *src};
  };
  auto stage_store = [&](const Raw &r, int s) {
#endif
    const int pl = 4 * (l & 15) + (l >> 4);
#pragma unroll
    for (int d = 0; d < kD; ++d) {
#if XH_8X_KL_TU
      const int bd = (signed char)((r.bi >> (8 * d)) & 0xff) -
                     (sub ? (signed char)((itm >> (8 * d)) & 0xff) : 0);
      const float x = (float)bd / (float)kCapacity;
#else
      const float x = (float)(signed char)((r.bi >> (8 * d)) & 0xff) / (float)kCapacity;
#endif
      lf[F_X + s * (kD * 64) + d * 64 + l] = x;
      lf[F_XP + s * (kD * 64) + d * 64 + pl] = x;
    }
    const int item = __builtin_amdgcn_readlane(r.rec, 3);
    bool ia = true;
#pragma unroll
    for (int d = 0; d < kD; ++d)
      ia &= (signed char)((item >> (8 * d)) & 0xff) == a.env.item_a[d];
    if (l == 0) lf[F_IT + s] = ia ? 1.0f : 0.0f;
#if XH_8X_KL_TU
    // action (lane 0), advantage (lane 2, 0 for end rows), whether the row
    // counts (lane 3)
    const int ended = __builtin_amdgcn_readfirstlane(r.ended);
    const bool valid = kind == 0 || (kind == 1 ? ended == 0 : g - NT - a.b.N < n_end);
    if (l == 0 || l == 2) lf[F_REC + 4 * s + l] = kind == 0 ? __int_as_float(r.rec) : 0.0f;
    if (l == 3) lf[F_REC + 4 * s + 3] = valid ? 1.0f : 0.0f;
#else
    if (l < 3) lf[F_REC + 4 * s + l] = __int_as_float(r.rec);
#endif
  };
  // H1 values (C layout, r-tile rt) scaled by S_H -> the two f16 part images
  auto store_h1 = [&](const f32x4 &t, int sb, int rt) {
    f16x4 ph, pl;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      _Float16 x0, x1;
      split2h(t[u] * SH, x0, x1);
      ph[u] = x0;
      pl[u] = x1;
    }
    st4h(sb + L_H1 + 4096 * rt, ph);
    st4h(sb + L_H1 + kImg + 4096 * rt, pl);
  };
  // layer 1 (C layout) of the unit in slot s, all four r-tiles -> H1 image
  auto layer1_all = [&](int s, int stb) {
    const bool ia = lf[F_IT + s] != 0.0f;
    const f32x4 wa = lds4v(lf + F_W1T + fo), wb = lds4v(lf + F_W1T + kH + fo);
    const f32x4 wc = lds4v(lf + F_W1T + 2 * kH + fo);
    const f32x4 bb = lds4v(lf + F_B1F + (ia ? 0 : kH) + fo);
    const float *xp = lf + F_XP + s * (kD * 64);
    const f32x4 x0 = lds4v(xp + 4 * li), x1 = lds4v(xp + 64 + 4 * li),
                x2 = lds4v(xp + 128 + 4 * li);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      f32x4 t;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        t[j] = relu(fmaf(x2[rt], wc[j], fmaf(x1[rt], wb[j], fmaf(x0[rt], wa[j], bb[j]))));
      store_h1(t, stb, rt);
    }
  };
  // layer 2 of the unit whose H1 is in the image: 16 steps of 3 f16 MFMAs,
  // task(k) after each MFMA (k = 0 .. 47)
  auto layer2 = [&](int rdb, int flo, f32x4 (&pre)[4], auto &&task) {
    const f32x4 b2 = lds4v(lf + F_B2 + fo);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) pre[rt] = b2;
    f16x8 b_c[2], b_n[2], lo_c = ld8h(flo + L_WLO), lo_n = lo_c;
#pragma unroll
    for (int p = 0; p < 2; ++p) b_c[p] = ld8h(rdb + L_H1 + p * kImg);
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int s = st >> 2, rt = st & 3;
      if (st + 1 < 16) {
        const int s1 = (st + 1) >> 2, r1 = (st + 1) & 3;
#pragma unroll
        for (int p = 0; p < 2; ++p)
          b_n[p] = ld8h((rdb ^ (64 * s1)) + L_H1 + p * kImg + 4096 * r1);
        if (r1 == 0) lo_n = ld8h(flo + L_WLO + 1024 * s1);
      }
      FENCE();
      pre[rt] = mfma16h(lo_c, b_c[0], pre[rt]);
      FENCE();
      task(3 * st);
      FENCE();
      pre[rt] = mfma16h(wl[s], b_c[1], pre[rt]);
      FENCE();
      task(3 * st + 1);
      FENCE();
      pre[rt] = mfma16h(wl[s], b_c[0], pre[rt]);
      FENCE();
      task(3 * st + 2);
      FENCE();
#pragma unroll
      for (int p = 0; p < 2; ++p) b_c[p] = b_n[p];
      if (rt == 3) lo_c = lo_n;
    }
  };
  // partial logits of unit u's rows 16 rt + li over this wave's features
  auto partial_rt = [&](const f32x4 &pre, const f32x4 &w3, int u, int rt) {
    float zp = relu(pre[0]) * w3[0];
    zp = fmaf(relu(pre[1]), w3[1], zp);
    zp = fmaf(relu(pre[2]), w3[2], zp);
    zp = fmaf(relu(pre[3]), w3[3], zp);
    zp = sum_groups(zp);
    const int zoff = (((u >> 1) & 1) * 2 + (u & 1)) * 512;
    if (G == 0) lf[F_Z + zoff + (16 * rt + li) * 8 + w] = zp;
  };
  auto partials = [&](const f32x4 (&pre)[4], const f32x4 &w3, int u) {
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) partial_rt(pre[rt], w3, u, rt);
  };
  auto no_task = [](int) {};

  // ---- pipeline prologue: units 0-2 staged, layer 1 + layer 2 of units 0
  // and 1 (their partial logits), layer 1 of unit 2
  f32x4 pre_v[4], pre_v1[4];
  Raw raw = {0, 0};
  if (w == 0) {
    stage_store(stage_load(0), 0 KLTU(, 0));
    stage_store(stage_load(1), 1 KLTU(, 1));
    stage_store(stage_load(2), 2 KLTU(, 2));
  }
  __syncthreads();
  layer1_all(0, stb0);
  __syncthreads();
  layer2(rdb0, flo0, pre_v, no_task);
  partials(pre_v, lds4v(lf + F_W3 + fo), 0);
  __syncthreads();
  layer1_all(1, stb0);
  __syncthreads();
  layer2(rdb0, flo0, pre_v1, no_task);
  partials(pre_v1, lds4v(lf + F_W3 + fo), 1);
  __syncthreads();
  layer1_all(2, stb0);
  __syncthreads();

  for (int v = 0; v < U; ++v) {
    const int cs = v & 3, ns = (v + 3) & 3;  // slots of units v and v + 3
    const bool first = (v & 1) == 0;        // the env's first unit: its softmax
    int rdb = rdb0, trm0 = trm00, trm1 = trm10, stb = stb0, flo = flo0;
    asm volatile("" : "+v"(rdb), "+v"(trm0), "+v"(trm1), "+v"(stb), "+v"(flo),
                 "+s"(gstep));
    if (w == 0) raw = stage_load(v + 3);
    const float *xim = lf + F_X + cs * (kD * 64);
    float *gw = gwb + 64 * (v & 1);  // unit v's g, row order
    float *gp = gpb + 64 * (v & 1);
    const float w1a = lf[F_W1T + 16 * w + li], w1b = lf[F_W1T + kH + 16 * w + li],
                w1c = lf[F_W1T + 2 * kH + 16 * w + li];

    // ================= X(v): layer 2 of unit v+2 with unit v's VALU ======
    const float *zb = lf + F_Z + ((v >> 1) & 1) * 1024;  // the env's partials
    const f32x4 za0 = lds4v(zb + 8 * l), za1 = lds4v(zb + 8 * l + 4);
    const f32x4 zc0 = lds4v(zb + 512 + 8 * l), zc1 = lds4v(zb + 512 + 8 * l + 4);
    const float b3 = lf[F_B3];
    const f32x4 rec = lds4v(lf + F_REC + 4 * cs);
    const float itc = lf[F_IT + cs];
#if XH_8X_KL_TU
    // the env's old distribution: its first unit's half, then its second's
    const float qv0 = lf[F_Q + cs * 64 + l], qv1 = lf[F_Q + ((v + 1) & 3) * 64 + l];
    float kp0 = 0.0f, kp1 = 0.0f, kg0 = 0.0f, kg1 = 0.0f;
#endif
    f32x4 gx0[2], gx1[2], gx2[2];
    float ex0 = 0.0f, ex1 = 0.0f, se = 0.0f, g0 = 0.0f, g1 = 0.0f;
    f32x4 gr4, ggk[2], hT[2];
    bf16x8 bq0[3];
    bool item_cur = false;
    float b1t = 0.0f;
    f32x4 w3;
    auto xtask = [&](int k) {
      if (k == 0) {
        if (first) {
          const float z0 = ((za0[0] + za0[1]) + (za0[2] + za0[3])) +
                           ((za1[0] + za1[1]) + (za1[2] + za1[3]));
          const float z1 = ((zc0[0] + zc0[1]) + (zc0[2] + zc0[3])) +
                           ((zc1[0] + zc1[1]) + (zc1[2] + zc1[3]));
          ex0 = __expf(z0 + b3);
          ex1 = __expf(z1 + b3);
        }
      } else if (k == 1) {
        if (first) se = seg_sum<64>(ex0 + ex1);
#if XH_8X_KL_TU
      } else if (k == 2) {
        if (first) {
          // kl_regulated_loss (policy_gradient.h:41-85) through
          // softmax_layer::backward (the Jacobian's sum in the next slot);
          // the KL sum on one wave per env, in turn
          const int cu = __builtin_amdgcn_readfirstlane(__float_as_int(rec[0]));
          const float Ac = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rec[2])));
          const float rse = __builtin_amdgcn_rcpf(se);
          kp0 = ex0 * rse;
          kp1 = ex1 * rse;
          kg0 = fmaf(beta, kp0 - qv0, kp0 * Ac);
          kg1 = fmaf(beta, kp1 - qv1, kp1 * Ac);
          if (l == cu) kg0 -= Ac;
          if (64 + l == cu) kg1 -= Ac;
          const bool vld = __builtin_amdgcn_readfirstlane(__float_as_int(rec[3])) != 0;
          if (vld && ((v >> 1) & 7) == w)
            kl_acc += (double)(qv0 * logf(qv0 / kp0)) + (double)(qv1 * logf(qv1 / kp1));
        }
#else
      } else if (k == 2) {
        if (first) {
          const int cu = __builtin_amdgcn_readfirstlane(__float_as_int(rec[0]));
          const float po = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rec[1])));
          const float Ac = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rec[2])));
          const float rse = __builtin_amdgcn_rcpf(se);
          const float p0 = ex0 * rse, p1 = ex1 * rse;
          const float pc = __int_as_float(
              __builtin_amdgcn_readlane(__float_as_int(cu < 64 ? p0 : p1), cu & 63));
          if (a.algo == kPPO) {
            // clipped_gradient (rl.h:54-74) through softmax_layer::backward
            const float ratio = pc * __builtin_amdgcn_rcpf(po);
            float ce = a.clip_eps;
            asm volatile("" : "+s"(ce));
            const float clipped = fminf(fmaxf(ratio, 1.0f - ce), 1.0f + ce);
            const float ig = fminf(clipped * Ac, ratio * Ac) * -1.0f;
            const float gc = ig * __builtin_amdgcn_rcpf(pc);
            g0 = ((l == cu ? p0 : 0.0f) - p0 * pc) * gc;
            g1 = ((64 + l == cu ? p1 : 0.0f) - p1 * pc) * gc;
          } else {
            // softmax_gradient_log (rl.h:45-52) through softmax-xent
            g0 = p0 * Ac;
            g1 = p1 * Ac;
            if (l == cu) g0 -= Ac;
            if (64 + l == cu) g1 -= Ac;
          }
        }
#endif
      } else if (k == 3) {
        if (first) {
#if XH_8X_KL_TU
          {
            const float sgv = seg_sum<64>(fmaf(kp1, kg1, kp0 * kg0));
            const bool vld = __builtin_amdgcn_readfirstlane(__float_as_int(rec[3])) != 0;
            g0 = vld ? kp0 * (kg0 - sgv) : 0.0f;
            g1 = vld ? kp1 * (kg1 - sgv) : 0.0f;
          }
#endif
          // both units' g (this wave's copies): unit v, then unit v + 1
          gw[l] = g0;
          gp[4 * (l & 15) + (l >> 4)] = g0;
          gw[64 + l] = g1;  // gwb + 64 ((v + 1) & 1): v is even
          gp[64 + 4 * (l & 15) + (l >> 4)] = g1;
          accB3 += g0;  // wave 0's is written out
          accB3 += g1;
        }
        item_cur = __builtin_amdgcn_readfirstlane(__float_as_int(itc)) != 0;
        b1t = lf[F_B1F + (item_cur ? 0 : kH) + 16 * w + li];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          gx0[h] = lds4v(xim + 16 * h + 4 * G);
          gx1[h] = lds4v(xim + 64 + 16 * h + 4 * G);
          gx2[h] = lds4v(xim + 128 + 16 * h + 4 * G);
        }
      } else if (k == 5) {
        gr4 = lds4v(gp + 4 * li);  // g of rows 16 rt + li
#pragma unroll
        for (int h = 0; h < 2; ++h) ggk[h] = lds4v(gw + 16 * h + 4 * G);
      } else if (k == 7 || k == 8) {
        // layer-1 values of K-step 0's rows (T layout), r-tile h
        const int h = k - 7;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          hT[h][jj] = relu(fmaf(gx2[h][jj], w1c,
                                fmaf(gx1[h][jj], w1b, fmaf(gx0[h][jj], w1a, b1t))));
      } else if (k >= 11 && k < 15) {
        // dW3 / db2 of r-tile rt (pre-activations in units of S2)
        const int rt = k - 11;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float pv = pre_v[rt][jj];
#if XH_8X_IMASK
          const float gm = gr4[rt] * (float)relu_bit(pv);
#else
          const float gm = pv > 0.0f ? gr4[rt] : 0.0f;
#endif
          accW3[jj] = fmaf(gm, pv, accW3[jj]);
          accB2[jj] += gm;
        }
      } else if (k >= 16 && k < 20) {
        // g (x) H1 of K-step 0, two values per slot
        const int h = (k - 16) >> 1, j0 = 2 * ((k - 16) & 1);
#pragma unroll
        for (int jj = j0; jj < j0 + 2; ++jj) {
          __bf16 p0, p1, p2;
          split3(hT[h][jj] * ggk[h][jj], p0, p1, p2);
          bq0[0][4 * h + jj] = p0;
          bq0[1][4 * h + jj] = p1;
          bq0[2][4 * h + jj] = p2;
        }
      } else if (k >= 20 && k < 24) {
        // the relu masks of r-tile k - 20 -> the bf16 and f16 mask images
        const int rt = k - 20;
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#if XH_8X_IMASK
        unsigned m[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) m[jj] = (unsigned)relu_bit(pre_v[rt][jj]);
        const u32x2 mm = {m[0] | (m[1] << 16), m[2] | (m[3] << 16)};
        st4(stb + L_MASK + 4096 * rt, __builtin_bit_cast(bf16x4, mm * 0x3F80u));
        st4h(stb + L_MASKH + 4096 * rt, __builtin_bit_cast(f16x4, mm * 0x3C00u));
#else
        bf16x4 mk;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          mk[jj] = pre_v[rt][jj] > 0.0f ? (__bf16)1.0f : (__bf16)0.0f;
        st4(stb + L_MASK + 4096 * rt, mk);
        const u32x2 mb = __builtin_bit_cast(u32x2, mk) & 0x3C003C00u;
        st4h(stb + L_MASKH + 4096 * rt, __builtin_bit_cast(f16x4, mb));
#endif
      } else if (k == 36) {
        w3 = lds4v(lf + F_W3 + fo);  // for the partial logits after layer 2
      } else if (k == 44) {
        if (w == 0) stage_store(raw, ns KLTU(, v + 3));  // unit v+3's rows
      }
    };
    f32x4 pre_v2[4];
    layer2(rdb, flo, pre_v2, xtask);
    partials(pre_v2, w3, v + 2);
    __syncthreads();

    // ================= Y(v): dW2 / dH1 of unit v with VALU of v, v+3 =====
    {
      float sg = 0.0f;
      bf16x8 bq1[3];
      f32x4 rx0[2], rx1[2], rx2[2], rgg[2], hT1[2];
      f32x4 wa, wb, wc, bb, xp0, xp1, xp2, t1;
      float itn = 0.0f;
      f32x4 dx0, dx1, dx2, dgg;
      f32x4 dh[2];
      auto load_ops = [&](int b, bf16x8 &A, f16x8 &L) {
        if (b < 16) {
          const int ks = b >> 3, ot = b & 7;
          A = ldtr((trm0 ^ (32 * ot)) + L_MASK + 8192 * ks,
                   (trm1 ^ (32 * ot)) + L_MASK + 8192 * ks);
        } else {
          const int rt = (b - 16) >> 2, s = (b - 16) & 3;
          A = ld8((rdb ^ (64 * s)) + L_MASKH + 4096 * rt);  // f16 bits
          L = ld8h(flo + L_WDLO + 1024 * s);
        }
      };
      // dW1 / db1 / item sums of value jj of r-tile rt (T layout)
      auto dw1 = [&](int jj, int rt) {
        const int q = rt & 1;
        const float tT = fmaf(dx2[jj], w1c, fmaf(dx1[jj], w1b, fmaf(dx0[jj], w1a, b1t)));
        const float d = tT > 0.0f ? dh[q][jj] * dgg[jj] : 0.0f;
        sg += d;
        w0 = fmaf(d, dx0[jj], w0);
        w1 = fmaf(d, dx1[jj], w1);
        w2 = fmaf(d, dx2[jj], w2);
      };
      auto layer1_rt = [&](int rt, int half, int sb) {
        if (half == 0) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            t1[jj] = relu(fmaf(xp2[rt], wc[jj],
                               fmaf(xp1[rt], wb[jj], fmaf(xp0[rt], wa[jj], bb[jj]))));
        } else {
          store_h1(t1, sb, rt);
        }
      };
      auto ytask = [&](int b) {
        if (b == 0) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int r0 = 32 + 16 * h + 4 * G;
            rx0[h] = lds4v(xim + r0);
            rx1[h] = lds4v(xim + 64 + r0);
            rx2[h] = lds4v(xim + 128 + r0);
            rgg[h] = lds4v(gw + r0);
          }
          itn = lf[F_IT + ns];
        } else if (b == 2 || b == 3) {
          const int h = b - 2;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            hT1[h][jj] = relu(fmaf(rx2[h][jj], w1c,
                                   fmaf(rx1[h][jj], w1b, fmaf(rx0[h][jj], w1a, b1t))));
        } else if (b >= 4 && b < 8) {
          const int h = (b - 4) >> 1, j0 = 2 * ((b - 4) & 1);
#pragma unroll
          for (int jj = j0; jj < j0 + 2; ++jj) {
            __bf16 p0, p1, p2;
            split3(hT1[h][jj] * rgg[h][jj], p0, p1, p2);
            bq1[0][4 * h + jj] = p0;
            bq1[1][4 * h + jj] = p1;
            bq1[2][4 * h + jj] = p2;
          }
          if (b == 4) {
            // unit v+3's layer-1 operands (C layout)
            wa = lds4v(lf + F_W1T + fo);
            wb = lds4v(lf + F_W1T + kH + fo);
            wc = lds4v(lf + F_W1T + 2 * kH + fo);
            const float *xp = lf + F_XP + ns * (kD * 64);
            xp0 = lds4v(xp + 4 * li);
            xp1 = lds4v(xp + 64 + 4 * li);
            xp2 = lds4v(xp + 128 + 4 * li);
          } else if (b == 5) {
            const bool ia = __builtin_amdgcn_readfirstlane(__float_as_int(itn)) != 0;
            bb = lds4v(lf + F_B1F + (ia ? 0 : kH) + fo);
          }
        } else if (b >= 8 && b < 16) {
          layer1_rt((b - 8) >> 1, b & 1, stb);
        } else {
          const int rt = (b - 16) >> 2, s = (b - 16) & 3;
          if (rt > 0) dw1(s, rt - 1);
          if (s == 3) {
            const int r0 = 16 * rt + 4 * G;
            dx0 = lds4v(xim + r0);
            dx1 = lds4v(xim + 64 + r0);
            dx2 = lds4v(xim + 128 + r0);
            dgg = lds4v(gw + r0);
          }
        }
      };
      bf16x8 A_c, A_n;
      f16x8 L_c, L_n;
      load_ops(0, A_c, L_c);
#pragma unroll
      for (int b = 0; b < 32; ++b) {
        if (b + 1 < 32) load_ops(b + 1, A_n, L_n);
        FENCE();
        if (b < 16) {
          const int ot = b & 7;
          const bf16x8(&bq)[3] = b < 8 ? bq0 : bq1;
          accW2[ot] = mfma16(A_c, bq[2], accW2[ot]);
          accW2[ot] = mfma16(A_c, bq[1], accW2[ot]);
          accW2[ot] = mfma16(A_c, bq[0], accW2[ot]);
        } else {
          const int rt = (b - 16) >> 2, s = (b - 16) & 3, q = rt & 1;
          if (s == 0) dh[q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
          const f16x8 Ah = __builtin_bit_cast(f16x8, A_c);
          dh[q] = mfma16h(Ah, L_c, dh[q]);
          dh[q] = mfma16h(Ah, wd[s], dh[q]);
        }
        FENCE();
        ytask(b);
        FENCE();
        A_c = A_n;
        L_c = L_n;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) dw1(s, 3);
      if (item_cur)
        sa += sg;
      else
        sb += sg;
    }
    __syncthreads();
    // rotate the pipeline
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      pre_v[rt] = pre_v1[rt];
      pre_v1[rt] = pre_v2[rt];
    }
  }

#if XH_8X_KL_TU
  {
    // the workgroup's KL sum (the loop's last barrier is behind: F_Z is free)
    double dv = kl_acc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) dv += __shfl_xor(dv, o, kWave);
    double *kd = reinterpret_cast<double *>(lf + F_Z);
    if (l == 0) kd[w] = dv;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
#pragma unroll
      for (int v8 = 0; v8 < 8; ++v8) t += kd[v8];
      a.kl_part[blockIdx.x] = t;
    }
  }
#endif

  // ---------------------------------------------------- slab write-out ----
  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
  const float *w3g = P + PL.ow3();
#pragma unroll
  for (int ot = 0; ot < 8; ++ot)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = 16 * ot + 4 * G + j;
      slab[PL.oW2() + o * kH + 16 * w + li] = accW2[ot][j] * w3g[o];
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float s3 = seg_sum<16>(accW3[j]);
    const float s2 = seg_sum<16>(accB2[j]);
    const int o = 16 * w + 4 * G + j;
    if (li == 0) {
      slab[PL.ow3() + o] = s3 * (1.0f / S2);
      slab[PL.ob2() + o] = s2 * w3g[o];
    }
  }
  if (w == 0) {
    const float v3 = seg_sum<64>(accB3);
    if (l == 0) slab[PL.ob3()] = v3;
  }
  {
    float tw0 = w0 + __shfl_xor(w0, 16, kWave);
    float tw1 = w1 + __shfl_xor(w1, 16, kWave);
    float tw2 = w2 + __shfl_xor(w2, 16, kWave);
    float va = sa + __shfl_xor(sa, 16, kWave);
    float vb = sb + __shfl_xor(sb, 16, kWave);
    tw0 += __shfl_xor(tw0, 32, kWave);
    tw1 += __shfl_xor(tw1, 32, kWave);
    tw2 += __shfl_xor(tw2, 32, kWave);
    va += __shfl_xor(va, 32, kWave);
    vb += __shfl_xor(vb, 32, kWave);
    // dH1 was in units of S_D
    tw0 *= 1.0f / SD;
    tw1 *= 1.0f / SD;
    tw2 *= 1.0f / SD;
    va *= 1.0f / SD;
    vb *= 1.0f / SD;
    if (G == 0) {
      const int i = 16 * w + li;
      slab[PL.oW1() + i * kF0 + 0] = tw0;
      slab[PL.oW1() + i * kF0 + 1] = tw1;
      slab[PL.oW1() + i * kF0 + 2] = tw2;
#pragma unroll
      for (int d = 0; d < kD; ++d)
        slab[PL.oW1() + i * kF0 + kD + d] =
            va * ((float)a.env.item_a[d] / (float)kCapacity) +
            vb * ((float)a.env.item_b[d] / (float)kCapacity);
      slab[PL.ob1() + i] = va + vb;
    }
  }
}
#undef FENCE

}  // namespace s8x

#if XH_8X_KL_TU
hipError_t launch_policy_train_split8x_kl(const PolicyTrainArgs &a, int grid,
                                          hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s8x::policy_train_split8x_kl_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s8x::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s8x::policy_train_split8x_kl_kernel, dim3(grid),
                     dim3(s8x::kThreads), s8x::kLds, s, a);
  return hipGetLastError();
}
#else
hipError_t launch_policy_train_split8x(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s) {
  if (a.algo == kKLPPO) return launch_policy_train_split8x_kl(a, grid, s);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s8x::policy_train_split8x_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s8x::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s8x::policy_train_split8x_kernel, dim3(grid),
                     dim3(s8x::kThreads), s8x::kLds, s, a);
  return hipGetLastError();
}
#endif

}  // namespace xh
