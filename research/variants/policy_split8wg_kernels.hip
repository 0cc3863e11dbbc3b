// policy_split8wg_kernels.hip -- the PPO / actor-critic train epoch of the
// 64-bin 2-D [128,128] policy (BASELINE configs 3 and 4): the pipelined
// 8-wave f16-pair kernel of policy_split8wh_kernels.hip (see its header: f16
// pairs, pipeline, layouts) with dW2 on f16 pairs as well, taking both of its
// operands from LDS images instead of building them in registers:
//
//     dW2 = M^T (g (x) H1) = (M o g)^T H1
//
// B = H1 itself, the f16-pair H1 image of the group (three images, one per
// pipeline slot, so the group's H1 is still there in Y(j)); A = the relu mask
// weighted by the row's loss gradient, g S_g M, as an f16-pair image (hi and
// lo), written in X(j) where the plain 0/1 mask image used to be.  S_g is a
// per-group power of two (|g S_g| < 2^14 from the group's max |g|, the
// exponent rounded up to a multiple of 4 so that consecutive groups mostly
// share it); the dW2 accumulators are kept in units of the current group's
// S_g S_H and rescaled by an exact power of two when it changes.  Per wave
// per group this drops the recomputed H1 values (T layout) and the
// three-part bf16 split of g (x) H1 (about 170 VALU) for a second mask image
// and three f16 MFMAs per dW2 block instead of three bf16 ones.
//
#include <cstdlib>

#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

// Phase stamps (trace build, tools/build_trace8wp.sh: -DXH_DIAG_TRACE=1, run
// with XH_PHASE_TRACE=1): lane 0 of every wave of the first kTraceBlocks
// workgroups records the cycle counter at 0 X start, 1 layer 2 (+ group j's
// VALU) done, 2 partial logits written, 3 after the X barrier, 4 dW2 / dH1
// blocks done, 5 dW1 tail done, 6 after the Y barrier (7 = 6), for its first
// kTraceGroups groups.
#ifndef XH_DIAG_TRACE
#define XH_DIAG_TRACE 0
#endif
#if XH_DIAG_TRACE
#define S8G_STAMP(a, gi, w, lane, slot)                                         \
  do {                                                                        \
    if ((a).trace && blockIdx.x < kTraceBlocks && (gi) < kTraceGroups &&      \
        (lane) == 0)                                                          \
      (a).trace[((blockIdx.x * kTraceGroups + (gi)) * 8 + (w)) * kTraceSlots + \
                (slot)] = clock64();                                          \
  } while (0)
#else
#define S8G_STAMP(a, gi, w, lane, slot) \
  do {                                  \
  } while (0)
#endif

// XH_TRACE_X=1 (diagnostic trace builds only): the stamps 1-7 inside X
// instead (after tasks 15, 31, 43, 45, layer 2's end, the partial logits,
// the barrier)
#ifndef XH_TRACE_X
#define XH_TRACE_X 0
#endif
#define S8G_STAMP_Y(a, gi, w, lane, slot) \
  do {                                    \
    if (!XH_TRACE_X) S8G_STAMP(a, gi, w, lane, slot); \
  } while (0)
#define S8G_STAMP_X(a, gi, w, lane, slot) \
  do {                                    \
    if (XH_TRACE_X) S8G_STAMP(a, gi, w, lane, slot); \
  } while (0)

namespace xh {
namespace s8g {

constexpr int kB = 64, kD = 2, kF0 = 2 * kD, kH = 128;
constexpr int kThreads = 512;
constexpr int kImg = 64 * kImgRow;  // one 64-row part image, 16 KB
// LDS carve (bytes): the H1 image (two f16 parts, scaled by S_H), the mask
// image as bf16 (dW2's A operand, transposed reads) and as f16 (dH1's A
// operand, row reads), then f32.  W2 / W2' live in registers as f16 pairs.
constexpr int L_H1 = 0;              // [3 slots][2 parts] H1 images (S_H)
constexpr int kH1Slot = 2 * kImg;    // bytes per slot
constexpr int L_GM = 6 * kImg;       // [2 parts] g S_g M (dW2's A operand)
constexpr int L_MASKH = 8 * kImg;    // f16 0/1 mask (dH1's A operand)
constexpr int L_F = 9 * kImg;
constexpr int F_W1T = 0;               // [2 k][128 i]: W1[i][k], the bin columns
constexpr int F_B1F = F_W1T + 2 * kH;  // [2 items][128]: b1 + the item's part
constexpr int F_B2 = F_B1F + 2 * kH;   // [128]
constexpr int F_W3 = F_B2 + kH;        // [128]
constexpr int F_B3 = F_W3 + kH;        // [4]
constexpr int F_Z = F_B3 + 4;          // [2 parity][64 rows][8 waves] partial logits
constexpr int F_GW = F_Z + 2 * 64 * 8;  // [8 waves][64 rows] g, row order
constexpr int F_GP = F_GW + 8 * 64;    // [8 waves][16 li][4 rt] g, C-layout order
constexpr int F_X = F_GP + 8 * 64;     // [3 slots][2 dims][64 rows] bins / 8
constexpr int F_XP = F_X + 3 * kD * 64;  // [3 slots][2 dims][16 li][4 rt]
constexpr int F_IT = F_XP + 3 * kD * 64;  // [3 slots] the group's item is item_a
constexpr int F_REC = F_IT + 4;        // [3 slots][action bits, pold, adv, -]
constexpr int F_SC = F_REC + 3 * 4;    // [16]: scale reduction scratch, the scales
constexpr int F_END = F_SC + 16;
constexpr size_t kLds = L_F + sizeof(float) * F_END;
static_assert(kLds <= 160 * 1024, "LDS");
static_assert(F_REC % 4 == 0 && F_GW % 4 == 0 && F_GP % 4 == 0 && F_X % 4 == 0 && F_XP % 4 == 0 &&
                  F_Z % 4 == 0 && F_W1T % 4 == 0 && F_B1F % 4 == 0,
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
// dH1's B operand lo part (W2' lo image [o][i]): K-step s element j of lane
// group G is row 32 s + 8G + j; read t: rows 32 s + 8G + 4t + q, columns
// 16 w + 4p .. +3
__device__ __forceinline__ int trw_base(int l, int t) {
  const int G = l >> 4, li = l & 15, q = li >> 2, p = li & 3;
  const int row = 8 * G + 4 * t + q;
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

__global__ __launch_bounds__(kThreads, 2) void policy_train_split8wg_kernel(
    PolicyTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH, kH};
  const float *P = a.params;
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int l = tid & 63, G = l >> 4, li = l & 15;
  const int ngroups = a.b.T * a.b.N;
  // this workgroup's groups: g_j = blockIdx.x + j gridDim.x, j < J; indices
  // past the end are clamped to the last group (their work is discarded)
  const int J = (int)blockIdx.x < ngroups
                    ? (ngroups - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x
                    : 0;
  if (J == 0) return;  // uniform over the workgroup
  // group g = t N + e is transition (t, e): its row of the [T][N] arrays
  int gstep = (int)gridDim.x;
  auto tindex = [&](int j) {
    return (size_t)((int)blockIdx.x + min(j, J - 1) * gstep);
  };

  // ---- prologue: the scales (maxima over the parameters, every workgroup
  // the same), small parameters into LDS, the W2 / W2' fragments of tile w
  // into registers as f16 pairs
  {
    float mw = 0.0f, md = 0.0f, mh = 0.0f;
    for (int e = tid; e < kH * kH; e += kThreads) {
      const float v = P[PL.oW2() + e];
      mw = fmaxf(mw, fabsf(v));
      md = fmaxf(md, fabsf(v * P[PL.ow3() + (e >> 7)]));
    }
    if (tid < kH) {
      float ba = P[PL.ob1() + tid], bb = ba;
#pragma unroll
      for (int d = 0; d < kD; ++d) {
        const float wv = P[PL.oW1() + tid * kF0 + kD + d];
        ba += wv * ((float)a.env.item_a[d] / (float)kCapacity);
        bb += wv * ((float)a.env.item_b[d] / (float)kCapacity);
      }
      mh = fabsf(P[PL.oW1() + tid * kF0]) + fabsf(P[PL.oW1() + tid * kF0 + 1]) +
           fmaxf(fabsf(ba), fabsf(bb));
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
    // mh: waves 0-1 hold the 128 features
    __syncthreads();
    float MW = 0.0f, MD = 0.0f;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      MW = fmaxf(MW, lf[F_SC + v]);
      MD = fmaxf(MD, lf[F_SC + 8 + v]);
    }
    __syncthreads();
    if (l == 0 && w < 2) lf[F_SC + w] = mh;
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
  for (int e = tid; e < 2 * kH; e += kThreads) {
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
    lf[F_B2 + i] = P[PL.ob2() + i] * S2;           // scaled: layer 2's C input
    lf[F_W3 + i] = P[PL.ow3() + i] * (1.0f / S2);  // unscales the partial logits
  }
  if (tid == 0) lf[F_B3] = P[PL.ob3()];
  f16x8 wl[4][2], wd[4][2];
  const int rdb0 = rd_base(G, li);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float4 *src = reinterpret_cast<const float4 *>(
        P + PL.oW2() + (16 * w + li) * kH + 32 * s + 8 * G);
    const float4 v0 = src[0], v1 = src[1];
    const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 x0, x1;
      split2h(v[j] * SW, x0, x1);
      wl[s][0][j] = x0;
      wl[s][1][j] = x1;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = 32 * s + 8 * G + j, col = 16 * w + li;
      _Float16 x0, x1;
      split2h((P[PL.oW2() + o * kH + col] * P[PL.ow3() + o]) * SD, x0, x1);
      wd[s][0][j] = x0;
      wd[s][1][j] = x1;
    }
  }
  // per-lane absolute LDS bases (the region offsets that exceed the 16-bit
  // immediate folded in)
  const int trm00 = trm_base(l, 0), trm10 = trm_base(l, 1);  // ^ 32 ot, + L_GM / L_H1
  const int stb0 = st_base(G, li) ^ (32 * w);  // + L_H1 / L_GM / L_MASKH + 4096 rt
  const int fo = 16 * w + 4 * G;  // this lane's 4 features in the C layout
  float *gw = lf + F_GW + 64 * w;  // this wave's copies of the rows' g
  float *gp = lf + F_GP + 64 * w;

  f32x4 accW2[8];
#pragma unroll
  for (int ot = 0; ot < 8; ++ot)
#pragma unroll
    for (int j = 0; j < 4; ++j) accW2[ot][j] = 0.0f;
  float accW3[4] = {0.0f, 0.0f, 0.0f, 0.0f}, accB2[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float accB3 = 0.0f, w0 = 0.0f, w1 = 0.0f, sa = 0.0f, sb = 0.0f;

  // wave 0 stages group j+2 during X(j): raw loads at its start (two
  // registers: the row's bins; lanes 0-3 the action, old probability,
  // advantage and the item's first two coordinates), the stores into slot s
  // (bins / 8 in row order and in the C layout's order, whether the item is
  // item_a, the record) late in the same phase, so the loads' latency hides
  // under layer 2
  struct Raw {
    int bi, rec;
  };
  auto stage_load = [&](int j) {
    const size_t ti = tindex(j);
    int lo = l * kD;  // recomputed per use rather than held (register pressure)
    asm volatile("" : "+v"(lo));
    const int bins =
        *reinterpret_cast<const unsigned short *>(a.b.bins + ti * (kB * kD) + lo);
    // one branch-free load per lane (lanes 3.. the item's first two
    // coordinates), so nothing waits for it before its use
    // (the address chosen by selects, not branches)
    const unsigned long long p0 = (unsigned long long)(a.b.action + ti);
    const unsigned long long p1 = (unsigned long long)(a.b.pold + ti);
    const unsigned long long p2 = (unsigned long long)(a.adv + ti);
    const unsigned long long p3 = (unsigned long long)(a.b.items + ti * 4);
    unsigned long long pa = l >= 3 ? p3 : p2;
    pa = l == 1 ? p1 : pa;
    pa = l == 0 ? p0 : pa;
    return Raw{bins, *reinterpret_cast<const int *>(pa)};
  };
  auto stage_store = [&](const Raw &r, int s) {
    const float x0 = (float)(signed char)(r.bi & 0xff) / (float)kCapacity;
    const float x1 = (float)(signed char)((r.bi >> 8) & 0xff) / (float)kCapacity;
    const int pl = 4 * (l & 15) + (l >> 4);
    lf[F_X + s * 128 + l] = x0;
    lf[F_X + s * 128 + 64 + l] = x1;
    lf[F_XP + s * 128 + pl] = x0;
    lf[F_XP + s * 128 + 64 + pl] = x1;
    const int item = __builtin_amdgcn_readlane(r.rec, 3);
    const int i0 = (signed char)(item & 0xff), i1 = (signed char)((item >> 8) & 0xff);
    if (l == 0)
      lf[F_IT + s] = (i0 == a.env.item_a[0] && i1 == a.env.item_a[1]) ? 1.0f : 0.0f;
    if (l < 3) lf[F_REC + 4 * s + l] = __int_as_float(r.rec);
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
  // layer 1 (C layout) of the group in slot s, all four r-tiles -> its H1
  // image (stb: the store base with the slot's offset folded in)
  auto layer1_all = [&](int s, int stb) {
    const bool ia = lf[F_IT + s] != 0.0f;
    const f32x4 wa = lds4v(lf + F_W1T + fo), wb = lds4v(lf + F_W1T + kH + fo);
    const f32x4 bb = lds4v(lf + F_B1F + (ia ? 0 : kH) + fo);
    const f32x4 x0 = lds4v(lf + F_XP + s * 128 + 4 * li);
    const f32x4 x1 = lds4v(lf + F_XP + s * 128 + 64 + 4 * li);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      f32x4 t;
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = relu(fmaf(x1[rt], wb[j], fmaf(x0[rt], wa[j], bb[j])));
      store_h1(t, stb, rt);
    }
  };
  // layer 2 of the group whose H1 is in the image: 16 steps of 3 f16 MFMAs
  // (A = S_W W2 tile w, B = S_H H1 rows 16 rt + li, f16 pairs), pre = S2 (b2
  // + W2 . H1); task(k) runs after each MFMA (k = 0 .. 47)
  auto layer2 = [&](int rdb, f32x4 (&pre)[4], auto &&task) {
    const f32x4 b2 = lds4v(lf + F_B2 + fo);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) pre[rt] = b2;
    f16x8 b_c[2], b_n[2];
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
      }
      FENCE();
      // the three products, small terms first
      pre[rt] = mfma16h(wl[s][1], b_c[0], pre[rt]);
      FENCE();
      task(3 * st);
      FENCE();
      pre[rt] = mfma16h(wl[s][0], b_c[1], pre[rt]);
      FENCE();
      task(3 * st + 1);
      FENCE();
      pre[rt] = mfma16h(wl[s][0], b_c[0], pre[rt]);
      FENCE();
      task(3 * st + 2);
      FENCE();
#pragma unroll
      for (int p = 0; p < 2; ++p) b_c[p] = b_n[p];
    }
  };
  // partial logits of rows 16 rt + li over this wave's features -> F_Z[zs]
  auto partial_rt = [&](const f32x4 &pre, const f32x4 &w3, int zs, int rt) {
    float zp = relu(pre[0]) * w3[0];
    zp = fmaf(relu(pre[1]), w3[1], zp);
    zp = fmaf(relu(pre[2]), w3[2], zp);
    zp = fmaf(relu(pre[3]), w3[3], zp);
    zp = sum_groups(zp);
    if (G == 0) lf[F_Z + zs * 512 + (16 * rt + li) * 8 + w] = zp;
  };
  auto partials = [&](const f32x4 (&pre)[4], const f32x4 &w3, int zs) {
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) partial_rt(pre[rt], w3, zs, rt);
  };
  auto no_task = [](int) {};

  // ---- pipeline prologue: groups 0 and 1 staged (group 2's rows loaded),
  // layer 1 and layer 2 of group 0 (its partial logits), layer 1 of group 1
  f32x4 pre_cur[4];
  if (w == 0) {
    stage_store(stage_load(0), 0);
    stage_store(stage_load(1), 1);
  }
  __syncthreads();
  layer1_all(0, stb0);
  __syncthreads();
  layer2(rdb0, pre_cur, no_task);
  partials(pre_cur, lds4v(lf + F_W3 + fo), 0);
  __syncthreads();
  layer1_all(1, stb0 + kH1Slot);
  __syncthreads();

  // dW2's accumulators are in units of 2^(14 - erun) S_H
  int erun = 0;
  for (int j = 0; j < J; ++j) {
    const int cs = j % 3, ns = (j + 2) % 3;  // slots of groups j and j + 2
    // H1 slots: group j+1's (layer 2 in X), group j's (dW2 in Y), group
    // j+2's (layer 1 in Y)
    const int h1n = ((j + 1) % 3) * kH1Slot, h1c = cs * kH1Slot, h1s = ns * kH1Slot;
    // per-lane absolute bases with the regions past the 16-bit ds offset
    // field folded in (the XOR'd bits 5-7 do not meet the region bits, so
    // (base + region) ^ x = (base ^ x) + region): rdb H1 slot j+1 rows; trg
    // dW2's A (g S_g M); trh dW2's B (H1 slot j, tile w); stg the mask
    // stores; sth the layer-1 stores (slot j+2); rdm dH1's A (0/1 mask)
    int rdb = rdb0 + h1n, trg0 = trm00 + L_GM, trg1 = trm10 + L_GM;
    int trh0 = (trm00 ^ (32 * w)) + L_H1 + h1c, trh1 = (trm10 ^ (32 * w)) + L_H1 + h1c;
    int stg = stb0 + L_GM, sth = stb0 + L_H1 + h1s, rdm = rdb0 + L_MASKH;
    asm volatile("" : "+v"(rdb), "+v"(trg0), "+v"(trg1), "+v"(stg), "+s"(gstep));
    asm volatile("" : "+v"(trh0), "+v"(trh1), "+v"(sth), "+v"(rdm));
    S8G_STAMP(a, j, w, l, 0);
    // (defined and used under w == 0 only: no value flows round the loop,
    // so nothing waits for the loads before the stores)
    Raw raw;
    if (w == 0) raw = stage_load(j + 2);
    const float *xim = lf + F_X + cs * 128;
    // T-layout constants of feature 16w + li (re-read: cheaper than holding)
    const float w1a = lf[F_W1T + 16 * w + li], w1b = lf[F_W1T + kH + 16 * w + li];

    // ================= X(j): layer 2 of group j+1 with group j's VALU ====
    // loads first (ahead of layer 2's operands): the partial logits, b3, the
    // record, the item flag
    const f32x4 z0 = lds4v(lf + F_Z + (j & 1) * 512 + 8 * l);
    const f32x4 z1 = lds4v(lf + F_Z + (j & 1) * 512 + 8 * l + 4);
    const float b3 = lf[F_B3];
    const f32x4 rec = lds4v(lf + F_REC + 4 * cs);
    const float itc = lf[F_IT + cs];
    float ex = 0.0f, se = 0.0f, gz = 0.0f;
    f32x4 gr4;
    // the group's dW2 scale S_g = 2^(14 - eg) (eg: max |g| < 2^eg, rounded up
    // to a multiple of 4) and g S_g of the lane's four C-layout rows as f16
    // pair bits
    int eg = 0;
    unsigned gh[4], gl[4];
    bool item_cur = false;
    float b1t = 0.0f;
    f32x4 w3;
    auto xtask = [&](int k) {
      if (k == 16) S8G_STAMP_X(a, j, w, l, 1);
      if (k == 32) S8G_STAMP_X(a, j, w, l, 2);
      if (k == 44) S8G_STAMP_X(a, j, w, l, 3);
      if (k == 46) S8G_STAMP_X(a, j, w, l, 4);
      if (k == 0) {
        const float zs = ((z0[0] + z0[1]) + (z0[2] + z0[3])) +
                         ((z1[0] + z1[1]) + (z1[2] + z1[3]));
        ex = __expf(zs + b3);
      } else if (k == 1) {
        se = seg_sum<64>(ex);
      } else if (k == 2) {
        const int cu = __builtin_amdgcn_readfirstlane(__float_as_int(rec[0]));
        const float po = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rec[1])));
        const float Ac = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rec[2])));
        const float p = ex * __builtin_amdgcn_rcpf(se);
        const float pc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), cu));
        if (a.algo == kPPO) {
          // clipped_gradient (rl.h:54-74) through softmax_layer::backward
          const float ratio = pc * __builtin_amdgcn_rcpf(po);
          float ce = a.clip_eps;  // the bounds computed here, not held
          asm volatile("" : "+s"(ce));
          const float clipped = fminf(fmaxf(ratio, 1.0f - ce), 1.0f + ce);
          const float ig = fminf(clipped * Ac, ratio * Ac) * -1.0f;
          const float gc = ig * __builtin_amdgcn_rcpf(pc);
          const float lin = l == cu ? p : 0.0f;
          gz = (lin - p * pc) * gc;
        } else {
          // softmax_gradient_log (rl.h:45-52) through softmax-xent
          gz = p * Ac;
          if (l == cu) gz -= Ac;
        }
      } else if (k == 3) {
        gw[l] = gz;
        gp[4 * (l & 15) + (l >> 4)] = gz;
        accB3 += gz;  // wave 0's is written out
        item_cur = __builtin_amdgcn_readfirstlane(__float_as_int(itc)) != 0;
        b1t = lf[F_B1F + (item_cur ? 0 : kH) + 16 * w + li];
      } else if (k == 4) {
        // max |g| over the group's 64 rows (every wave holds all of g; the
        // order of the magnitude bits is the order of the floats)
        unsigned gb = __float_as_uint(gz) & 0x7FFFFFFFu;
        gb = max(gb, (unsigned)__builtin_amdgcn_mov_dpp((int)gb, 0xB1, 0xF, 0xF, false));
        gb = max(gb, (unsigned)__builtin_amdgcn_mov_dpp((int)gb, 0x4E, 0xF, 0xF, false));
        gb = max(gb, (unsigned)__builtin_amdgcn_mov_dpp((int)gb, 0x141, 0xF, 0xF, false));
        gb = max(gb, (unsigned)__builtin_amdgcn_mov_dpp((int)gb, 0x140, 0xF, 0xF, false));
        const unsigned gm =
            max(max((unsigned)__builtin_amdgcn_readlane((int)gb, 0),
                    (unsigned)__builtin_amdgcn_readlane((int)gb, 16)),
                max((unsigned)__builtin_amdgcn_readlane((int)gb, 32),
                    (unsigned)__builtin_amdgcn_readlane((int)gb, 48)));
        // frexp exponent of max |g| (max |g| < 2^e), up to a multiple of 4,
        // within [-40, 40]
        const int e = (int)((gm >> 23) & 0xFFu) - 126;
        eg = min(max((e + 3) & ~3, -40), 40);
      } else if (k == 5) {
        gr4 = lds4v(gp + 4 * li);  // g of rows 16 rt + li
      } else if (k >= 11 && k < 15) {
        // dW3 / db2 of r-tile rt (pre-activations in units of S2: dW3 is
        // unscaled at the write-out)
        const int rt = k - 11;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float v = pre_cur[rt][jj];
          // relu'(v) as an integer clamp of v's bits (v_med3: no compare,
          // no VCC hazard)
          const float gm = gr4[rt] * (float)relu_bit(v);
          accW3[jj] = fmaf(gm, v, accW3[jj]);  // g relu(v)
          accB2[jj] += gm;                     // g M (w3 at the write-out)
        }
      } else if (k >= 16 && k < 20) {
        // g S_g of row 16 rt + li as an f16 pair (the bits, zero-extended)
        const int rt = k - 16;
        _Float16 h0, h1;
        split2h(gr4[rt] * __int_as_float((141 - eg) << 23), h0, h1);
        gh[rt] = __builtin_bit_cast(unsigned short, h0);
        gl[rt] = __builtin_bit_cast(unsigned short, h1);
      } else if (k >= 20 && k < 24) {
        // the relu masks of r-tile k - 20 (C layout) -> dW2's g S_g M images
        // (hi, lo) and dH1's 0/1 image, all f16
        const int rt = k - 20;
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        // 0 / 1 per value from the bits, two per dword
        unsigned m[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          m[jj] = (unsigned)relu_bit(pre_cur[rt][jj]);
        // times the f16 bits of g S_g's parts and of 1.0 by the full-rate
        // 24-bit multiply (the 32-bit one is quarter rate)
        const unsigned m01 = m[0] | (m[1] << 16), m23 = m[2] | (m[3] << 16);
        const u32x2 mh = {(unsigned)__umul24(m01, gh[rt]), (unsigned)__umul24(m23, gh[rt])};
        const u32x2 ml = {(unsigned)__umul24(m01, gl[rt]), (unsigned)__umul24(m23, gl[rt])};
        const u32x2 m1 = {(unsigned)__umul24(m01, 0x3C00u), (unsigned)__umul24(m23, 0x3C00u)};
        st4h(stg + 4096 * rt, __builtin_bit_cast(f16x4, mh));
        st4h(stg + kImg + 4096 * rt, __builtin_bit_cast(f16x4, ml));
        st4h(stg + (L_MASKH - L_GM) + 4096 * rt, __builtin_bit_cast(f16x4, m1));

      } else if (k == 36) {
        w3 = lds4v(lf + F_W3 + fo);  // for the partial logits after layer 2
      } else if (k == 44) {
        // wave 0: group j+2's rows (loaded at the start of X(j)) into slot ns
        if (w == 0) stage_store(raw, ns);
      }
    };
    f32x4 pre_nx[4];
    layer2(rdb, pre_nx, xtask);
    S8G_STAMP_Y(a, j, w, l, 1);
    S8G_STAMP_X(a, j, w, l, 5);
    partials(pre_nx, w3, (j + 1) & 1);
    S8G_STAMP_Y(a, j, w, l, 2);
    S8G_STAMP_X(a, j, w, l, 6);
    __syncthreads();
    S8G_STAMP_Y(a, j, w, l, 3);
    S8G_STAMP_X(a, j, w, l, 7);

    // ================= Y(j): dW2 / dH1 of group j with VALU of j, j+2 =====
    // 32 blocks: b < 16 dW2, three f16 MFMAs (ks = b / 8, ot = b % 8: S_g S_H
    // dW2 += (S_g g o M)^T (S_H H1), both from images), b >= 16 dH1, two f16
    // MFMAs (rt = (b - 16) / 4, s = (b - 16) % 4: S_D dH1 = M (S_D W2'), the
    // 0/1 image); A operands one block ahead
    {
      // the accumulators into this group's units (exact powers of two)
      if (eg != erun) {
        const float r = __int_as_float((127 + erun - eg) << 23);
#pragma unroll
        for (int ot = 0; ot < 8; ++ot) accW2[ot] *= r;
        erun = eg;
      }
      float sg = 0.0f;
      f32x4 wa, wb, bb, xp0, xp1, t1;
      float itn = 0.0f;
      f32x4 dx0, dx1, dgg;
      f32x4 dh[2];
      struct AOp {
        f16x8 h, l;
      };
      auto ldtrh = [&](int o0, int o1) { return __builtin_bit_cast(f16x8, ldtr(o0, o1)); };
      // B: this group's H1 columns 16 w .. 16 w + 15 by transposed reads
      f16x8 Bw[2][2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int p = 0; p < 2; ++p)
          Bw[ks][p] = ldtrh(trh0 + p * kImg + 8192 * ks, trh1 + p * kImg + 8192 * ks);
      // blocks alternate: even b dW2 block b / 2, odd b dH1 block (b - 1) / 2
      // (the LDS reads of the two kinds interleaved)
      auto load_ops = [&](int bb_, AOp &A) {
        if ((bb_ & 1) == 0) {
          const int b = bb_ >> 1;
          const int ks = b >> 3, ot = b & 7;
          A.h = ldtrh((trg0 ^ (32 * ot)) + 8192 * ks, (trg1 ^ (32 * ot)) + 8192 * ks);
          A.l = ldtrh((trg0 ^ (32 * ot)) + kImg + 8192 * ks,
                      (trg1 ^ (32 * ot)) + kImg + 8192 * ks);
        } else {
          const int b = bb_ >> 1;
          const int rt = b >> 2, s = b & 3;
          A.h = ld8h((rdm ^ (64 * s)) + 4096 * rt);
        }
      };
      // dW1 / db1 / item sums of value jj of r-tile rt (T layout)
      auto dw1 = [&](int jj, int rt) {
        const int q = rt & 1;
        const float tT = fmaf(dx1[jj], w1b, fmaf(dx0[jj], w1a, b1t));
        const float d = tT > 0.0f ? dh[q][jj] * dgg[jj] : 0.0f;
        sg += d;
        w0 = fmaf(d, dx0[jj], w0);
        w1 = fmaf(d, dx1[jj], w1);
      };
      // layer 1 of group j+2, r-tile rt of the feature block at store base
      // sb: half 0 the values, half 1 the split stores
      auto layer1_rt = [&](int rt, int half, int sb) {
        if (half == 0) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            t1[jj] = relu(fmaf(xp1[rt], wb[jj], fmaf(xp0[rt], wa[jj], bb[jj])));
        } else {
          store_h1(t1, sb, rt);
        }
      };
      auto ytask = [&](int b) {
        if (b == 0) {
          itn = lf[F_IT + ns];  // group j+2's item flag
        } else if (b == 4) {
          // group j+2's layer-1 operands (C layout)
          wa = lds4v(lf + F_W1T + fo);
          wb = lds4v(lf + F_W1T + kH + fo);
          xp0 = lds4v(lf + F_XP + ns * 128 + 4 * li);
          xp1 = lds4v(lf + F_XP + ns * 128 + 64 + 4 * li);
        } else if (b == 5) {
          const bool ia = __builtin_amdgcn_readfirstlane(__float_as_int(itn)) != 0;
          bb = lds4v(lf + F_B1F + (ia ? 0 : kH) + fo);
        } else if ((b & 1) == 0 && b >= 8 && b < 24) {
          // layer 1 of group j+2 in the dW2 blocks' slots, r-tile (b - 8) /
          // 4: values, then the split stores into its slot
          layer1_rt((b - 8) >> 2, (b >> 1) & 1, sth - L_H1);
        }
        if (b & 1) {
          const int rt = (b >> 1) >> 2, s = (b >> 1) & 3;
          if (rt > 0) dw1(s, rt - 1);
          if (s == 3) {
            // rows of r-tile rt (used in r-tile rt + 1's slots or the tail)
            const int r0 = 16 * rt + 4 * G;
            dx0 = lds4v(xim + r0);
            dx1 = lds4v(xim + 64 + r0);
            dgg = lds4v(gw + r0);
          }
        }
      };
      AOp A_c, A_n;
      load_ops(0, A_c);
#pragma unroll
      for (int b = 0; b < 32; ++b) {
        if (b + 1 < 32) load_ops(b + 1, A_n);
        FENCE();
        if ((b & 1) == 0) {
          const int ks = (b >> 1) >> 3, ot = (b >> 1) & 7;
          // the three products, small terms first
          accW2[ot] = mfma16h(A_c.l, Bw[ks][0], accW2[ot]);
          accW2[ot] = mfma16h(A_c.h, Bw[ks][1], accW2[ot]);
          accW2[ot] = mfma16h(A_c.h, Bw[ks][0], accW2[ot]);
        } else {
          const int rt = (b >> 1) >> 2, s = (b >> 1) & 3, q = rt & 1;
          if (s == 0) dh[q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
          dh[q] = mfma16h(A_c.h, wd[s][1], dh[q]);
          dh[q] = mfma16h(A_c.h, wd[s][0], dh[q]);
        }
        FENCE();
        ytask(b);
        FENCE();
        A_c = A_n;
      }
      S8G_STAMP_Y(a, j, w, l, 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) dw1(s, 3);
      if (item_cur)
        sa += sg;
      else
        sb += sg;
      S8G_STAMP_Y(a, j, w, l, 5);
    }
    __syncthreads();
    S8G_STAMP_Y(a, j, w, l, 6);
    S8G_STAMP_Y(a, j, w, l, 7);
    // rotate the pipeline
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) pre_cur[rt] = pre_nx[rt];
  }

  // ---------------------------------------------------- slab write-out ----
  // every entry has exactly one producing lane
  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
  const float *w3g = P + PL.ow3();
  // dW2's units 2^(14 - erun) S_H removed (powers of two: exact)
  const float u2 = __int_as_float((127 + erun - 14) << 23) * (1.0f / SH);
#pragma unroll
  for (int ot = 0; ot < 8; ++ot)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = 16 * ot + 4 * G + j;
      slab[PL.oW2() + o * kH + 16 * w + li] = (accW2[ot][j] * u2) * w3g[o];
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // dW3 / db2 of o = 16w + 4G + j: sums over the 16 lanes (rows) of group G
    const float s3 = seg_sum<16>(accW3[j]);
    const float s2 = seg_sum<16>(accB2[j]);
    const int o = 16 * w + 4 * G + j;
    if (li == 0) {
      slab[PL.ow3() + o] = s3 * (1.0f / S2);  // pre-activations were in units of S2
      slab[PL.ob2() + o] = s2 * w3g[o];
    }
  }
  if (w == 0) {
    const float v3 = seg_sum<64>(accB3);
    if (l == 0) slab[PL.ob3()] = v3;
  }
  {
    // dW1 / db1 of feature i = 16w + li: the four lane groups hold row subsets
    float tw0 = w0 + __shfl_xor(w0, 16, kWave);
    float tw1 = w1 + __shfl_xor(w1, 16, kWave);
    float va = sa + __shfl_xor(sa, 16, kWave);
    float vb = sb + __shfl_xor(sb, 16, kWave);
    tw0 += __shfl_xor(tw0, 32, kWave);
    tw1 += __shfl_xor(tw1, 32, kWave);
    va += __shfl_xor(va, 32, kWave);
    vb += __shfl_xor(vb, 32, kWave);
    // dH1 was in units of S_D
    tw0 *= 1.0f / SD;
    tw1 *= 1.0f / SD;
    va *= 1.0f / SD;
    vb *= 1.0f / SD;
    if (G == 0) {
      const int i = 16 * w + li;
      slab[PL.oW1() + i * kF0 + 0] = tw0;
      slab[PL.oW1() + i * kF0 + 1] = tw1;
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

}  // namespace s8g

hipError_t launch_policy_train_split8wg(const PolicyTrainArgs &a, int grid,
                                        hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s8g::policy_train_split8wg_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s8g::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s8g::policy_train_split8wg_kernel, dim3(grid),
                     dim3(s8g::kThreads), s8g::kLds, s, a);
  return hipGetLastError();
}

}  // namespace xh
