// policy_split8wh_kernels.hip -- the PPO / actor-critic train epoch of the
// 64-bin 2-D [128,128] policy (BASELINE configs 3 and 4): the pipelined
// 8-wave kernel of variants/policy_split8wp_kernels.hip with layer 2 and dH1 on the
// f16 matrix cores, each f32 operand scaled by a power of two and split
// EXACTLY into two f16 parts ("f16 pairs"):
//
//     S x = hi + lo + e,  hi = f16(S x), lo = f16(S x - hi),  |e| <= 2^-22 |S x|
//
// (11 significant bits per part, round to nearest; S x - hi is exact).  The
// scales are per launch, chosen from the operands' maxima so that |S x| <=
// 2^14 (f16's range ends at 65504): W2 and W2' = diag(w3) W2 from the
// parameters, H1 from the bound |H1[r][i]| <= |W1[i][0]| + |W1[i][1]| +
// |b1_item[i]| (|bins / 8| <= 1).  A product of two f16 values is exact in
// f32, so a dot product is
//
//     (S_a a).(S_b b) = hi.hi + hi.lo + lo.hi + d,  |d| <= 3 2^-22 sum|a_k b_k|
//
// (the dropped lo.lo and the two e terms): three MFMAs per K = 32 slice for
// layer 2 instead of the bf16 split's six, and two for dH1 (its mask operand
// is exact in f16) instead of three.  Results stay in scaled units where
// only signs matter (the relu masks) and are unscaled exactly (powers of two)
// in the partial logits (w3 / (S_W S_H)), in dW3 and in dW1 at the write-out.
// dW2's operand g (x) H1 has no bound known before the kernel (g ~ A / p_old),
// so dW2 keeps the exact three-part bf16 split.  MFMAs per wave per 64-row
// group: 192 -> 128.  Pipeline, layouts and swizzles as in
// variants/policy_split8wp_kernels.hip:
//
// Why: the two waves of a SIMD run the same phases in lockstep, so a VALU
// block and an MFMA block do not overlap, while VALU instructions issued
// between one wave's own MFMAs are nearly free (tools/probes/
// interleave_probe.hip: 96 v_mfma_f32_16x16x32_bf16 per wave at two waves
// per SIMD take 3083 cycles alone, 3200 with two independent v_fma_f32 after
// each MFMA, 4025 with the same VALU as a block after them).  A group's
// softmax, loss gradient, masks, dW3 / db2 sums, g (x) H1 splits, dW1 sums
// and layer 1 have no MFMA work of their own group to hide under, so the
// loop runs two groups at once:
//
//   X(j): MFMA  layer 2 of group j+1 (96 per wave)
//         VALU  softmax + loss gradient of group j, its relu masks (image),
//               dW3 / db2 sums, the first K-step's g (x) H1 fragments;
//               then group j+1's partial logits      -> barrier
//   Y(j): MFMA  dW2 and dH1 of group j (96 per wave)
//         VALU  the second K-step's g (x) H1 fragments, layer 1 of group
//               j+2 (-> H1 image), dW1 / db1 / item sums of group j
//                                                     -> barrier
//
// Waves issue in order, so a task must never wait: the VALU work is cut into
// slots of independent instructions after each block of three MFMAs
// (sched_barrier-fenced), and every LDS value a slot uses was loaded at
// least one slot earlier and before the next block's operand prefetch (LDS
// returns in order, so a consumer then waits for nothing younger).  The
// partial logits are summed over lane groups with v_permlane16/32_swap (no
// LDS round trip); each wave keeps its own copies of the rows' loss
// gradients, in row order and in the C layout's order, so no barrier
// separates producing and using them; the X rows are staged in both orders.
// Image addresses are plain integers (dynamic LDS starts at 0: this kernel
// has no static LDS) so the region and tile offsets fold into the ds_read /
// ds_write immediates.
//
// Layouts, swizzle and operand maps: "C layout" = the 16x16 MFMA result,
// lane column li = l & 15 (a row of the group), registers rows 4G + j (G =
// l >> 4; features); "T layout" = lane feature, registers rows.  Images are
// [64 rows][128 x bf16] with 16-byte chunks XOR-swizzled by swz2(row & 15)
// (conflict-free for the 16x16x32 row reads in the natural chunk order 4s +
// G, for ds_read_b64_tr_b16 and for the C-layout ds_write_b64 stores).
#include <cstdlib>

#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

// Built twice (Makefile): the PPO / actor-critic kernel (the benchmark's),
// and with XH_8WH_KL_TU=1 (policy_split8wh_kl_kernels.o) its KL-PPO form,
// policy_train_split8wh_kl_kernel.  The KL additions are preprocessor blocks
// so that the PPO object compiles from exactly its measured source (the
// kernel's register allocation moves with any change to it), and the KL
// object gets the higher full-unroll threshold its larger task lambdas need.
#ifndef XH_8WH_KL_TU
#define XH_8WH_KL_TU 0
#endif
#ifndef XH_8WH_XCD
#define XH_8WH_XCD 1
#endif
#if XH_8WH_KL_TU
#define KLTU(...) __VA_ARGS__
#else
#define KLTU(...)
#endif

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
#define S8H_STAMP(a, gi, w, lane, slot)                                         \
  do {                                                                        \
    if ((a).trace && blockIdx.x < kTraceBlocks && (gi) < kTraceGroups &&      \
        (lane) == 0)                                                          \
      (a).trace[((blockIdx.x * kTraceGroups + (gi)) * 8 + (w)) * kTraceSlots + \
                (slot)] = clock64();                                          \
  } while (0)
#else
#define S8H_STAMP(a, gi, w, lane, slot) \
  do {                                  \
  } while (0)
#endif

// XH_TRACE_X=1 (diagnostic trace builds only): the stamps 1-7 inside X
// instead (after tasks 15, 31, 43, 45, layer 2's end, the partial logits,
// the barrier)
#ifndef XH_TRACE_X
#define XH_TRACE_X 0
#endif
#define S8H_STAMP_Y(a, gi, w, lane, slot) \
  do {                                    \
    if (!XH_TRACE_X) S8H_STAMP(a, gi, w, lane, slot); \
  } while (0)
#define S8H_STAMP_X(a, gi, w, lane, slot) \
  do {                                    \
    if (XH_TRACE_X) S8H_STAMP(a, gi, w, lane, slot); \
  } while (0)

namespace xh {
namespace s8h {

constexpr int kB = 64, kD = 2, kF0 = 2 * kD, kH = 128;
// relu masks from the pre-activations' bits (relu_bit): 2.37 -> 2.28 ms per
// epoch against compare + select (the VCC hazard's s_nops)
#ifndef XH_8WH_IMASK
#define XH_8WH_IMASK 1
#endif
constexpr int kThreads = 512;
constexpr int kImg = 64 * kImgRow;  // one 64-row part image, 16 KB
// LDS carve (bytes): the H1 image (two f16 parts, scaled by S_H), the mask
// image as bf16 (dW2's A operand, transposed reads) and as f16 (dH1's A
// operand, row reads), then f32.  W2 / W2' live in registers as f16 pairs.
constexpr int L_H1 = 0;
constexpr int L_MASK = 2 * kImg;
// (3 * kImg: the f16 mask image before the one-image masks, unused)
constexpr int L_F = 4 * kImg;
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
#if XH_8WH_KL_TU
constexpr int F_Q = F_SC + 16;         // KL-PPO: [3 slots][64 bins] old distribution
constexpr int F_END = F_Q + 3 * 64;
#else
constexpr int F_END = F_SC + 16;
#endif
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
__device__ __forceinline__ void split4(const f32x4 &v, bf16x4 &ph, bf16x4 &pm,
                                       bf16x4 &pl) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    __bf16 a, b, c;
    split3(v[u], a, b, c);
    ph[u] = a;
    pm[u] = b;
    pl[u] = c;
  }
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

#if XH_8WH_KL_TU
// kl_ppo_learner's epoch (policy_gradient.h:310-335) over every row of its
// state matrix, as policy_train_kernel<S, true> (policy_kernels.hip): the T N
// transitions, then the open trajectories' end rows (slot T, q of step T - 1,
// valid unless step T - 1 ended), then the terminal end rows E_t of end_list
// (bins with the item taken back out of the chosen bin, rl.h:336-343); end
// rows have A = 0.  The loss head is kl_regulated_loss through
// softmax_layer::backward, and each workgroup sums KL(q || p) over its valid
// rows into kl_part.
__global__ __launch_bounds__(kThreads, 2) void policy_train_split8wh_kl_kernel(
    PolicyTrainArgs a) {
#else
__global__ __launch_bounds__(kThreads, 2) void policy_train_split8wh_kernel(
    PolicyTrainArgs a) {
#endif
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH, kH};
  const float *P = a.params;
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int l = tid & 63, G = l >> 4, li = l & 15;
#if XH_8WH_KL_TU
  const int NT = a.b.T * a.b.N;
  const int n_end = *a.n_end;
  const int ngroups = NT + a.b.N + n_end;
  const float beta = *a.beta;
#else
  const int ngroups = a.b.T * a.b.N;
#endif
  // this workgroup's groups: g_j = blockIdx.x + j gridDim.x, j < J; indices
  // past the end are clamped to the last group (their work is discarded)
#if XH_8WH_XCD
  // XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs
  // (XCD = blockIdx % 8), so workgroup b takes offset (b % 8) G / 8 + b / 8
  // of every run of G groups: the 32 adjacent groups whose records share a
  // 128-byte line of action / pold / adv / items are read by one XCD's L2,
  // not by all eight (config 3: 60.5 -> ≈43 MB of HBM traffic per launch)
  const int b0 = ((int)gridDim.x & 7) == 0
                     ? ((int)blockIdx.x & 7) * ((int)gridDim.x >> 3) + ((int)blockIdx.x >> 3)
                     : (int)blockIdx.x;
#else
  const int b0 = (int)blockIdx.x;
#endif
  const int J = b0 < ngroups ? (ngroups - b0 + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  if (J == 0) return;  // uniform over the workgroup
  // group g = t N + e is transition (t, e): its row of the [T][N] arrays
  int gstep = (int)gridDim.x;
  auto tindex = [&](int j) {
    return (size_t)(b0 + min(j, J - 1) * gstep);
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
  const int trm00 = trm_base(l, 0), trm10 = trm_base(l, 1);  // ^ 32 ot, + L_MASK
  const int stb0 = st_base(G, li) ^ (32 * w);  // + L_H1 / L_MASK + 4096 rt
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
#if XH_8WH_KL_TU
  double kl_acc = 0.0;  // sum of KL(q || p) over this wave's rows
#endif

  // wave 0 stages group j+2 during X(j): raw loads at its start (two
  // registers: the row's bins; lanes 0-3 the action, old probability,
  // advantage and the item's first two coordinates), the stores into slot s
  // (bins / 8 in row order and in the C layout's order, whether the item is
  // item_a, the record) late in the same phase, so the loads' latency hides
  // under layer 2
#if XH_8WH_KL_TU
  // (the old distribution goes straight to its LDS slot by an LDS-direct
  // load, and an open end row's done byte rides in lane 1's record word:
  // no registers held across layer 2 for either)
  struct Raw {
    int bi, rec;
  };
  // the row of the [T+1][N] arrays group g reads and the row of its old
  // distribution (kind 0 transition, 1 open end row, 2 terminal end row); g
  // is wave-uniform: scalar branches, and only terminal end rows wait for
  // their end_list entry
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
  auto stage_load = [&](int j) {
    size_t ti = tindex(j), qi = 0;
    kl_rows((int)ti, ti, qi);
    // (open end rows: the [T][N] record arrays end at slot T - 1; their
    // values are not used for end rows)
    const size_t ri = qi;
#else
  struct Raw {
    int bi, rec;
  };
  auto stage_load = [&](int j) {
    const size_t ti = tindex(j);
    const size_t ri = ti;
#endif
    int lo = l * kD;  // recomputed per use rather than held (register pressure)
    asm volatile("" : "+v"(lo));
    const int bins =
        *reinterpret_cast<const unsigned short *>(a.b.bins + ti * (kB * kD) + lo);
    // one branch-free load per lane (lanes 3.. the item's first two
    // coordinates), so nothing waits for it before its use
    // (the address chosen by selects, not branches)
    const unsigned long long p0 = (unsigned long long)(a.b.action + ri);
#if XH_8WH_KL_TU
    // lane 1: the aligned word holding done[qi] (an open end row's validity)
    const unsigned long long p1 =
        (unsigned long long)(a.b.done + (qi & ~(size_t)3));
#else
    const unsigned long long p1 = (unsigned long long)(a.b.pold + ri);
#endif
    const unsigned long long p2 = (unsigned long long)(a.adv + ri);
    const unsigned long long p3 = (unsigned long long)(a.b.items + ti * 4);
    unsigned long long pa = l >= 3 ? p3 : p2;
    pa = l == 1 ? p1 : pa;
    pa = l == 0 ? p0 : pa;
#if XH_8WH_KL_TU
    typedef __attribute__((address_space(1))) void gvoid;
    typedef __attribute__((address_space(3))) void lvoid;
    __builtin_amdgcn_global_load_lds((gvoid *)(a.qold + qi * kB + l),
                                     (lvoid *)(lf + F_Q + ((int)(j % 3)) * 64), 4, 0, 0);
    return Raw{bins, *reinterpret_cast<const int *>(pa)};
  };
  auto stage_store = [&](const Raw &r, int s, int j) {
    const int g = __builtin_amdgcn_readfirstlane((int)tindex(j));
    const int kind = g < NT ? 0 : g < NT + a.b.N ? 1 : 2;
    // the terminal view: the chosen bin without the item (rl.h:336-343)
    const int itm = __builtin_amdgcn_readlane(r.rec, 3);
    const bool sub = kind == 2 && l == __builtin_amdgcn_readfirstlane(r.rec);
    const int b0 = (signed char)(r.bi & 0xff) - (sub ? (signed char)(itm & 0xff) : 0);
    const int b1 = (signed char)((r.bi >> 8) & 0xff) - (sub ? (signed char)((itm >> 8) & 0xff) : 0);
    const float x0 = (float)b0 / (float)kCapacity;
    const float x1 = (float)b1 / (float)kCapacity;
    // the old distribution's LDS-direct load (issued with this group's
    // staging loads, long done): complete before the phase's barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
    return Raw{bins, *reinterpret_cast<const int *>(pa)};
  };
  auto stage_store = [&](const Raw &r, int s) {
    const float x0 = (float)(signed char)(r.bi & 0xff) / (float)kCapacity;
    const float x1 = (float)(signed char)((r.bi >> 8) & 0xff) / (float)kCapacity;
#endif
    const int pl = 4 * (l & 15) + (l >> 4);
    lf[F_X + s * 128 + l] = x0;
    lf[F_X + s * 128 + 64 + l] = x1;
    lf[F_XP + s * 128 + pl] = x0;
    lf[F_XP + s * 128 + 64 + pl] = x1;
    const int item = __builtin_amdgcn_readlane(r.rec, 3);
    const int i0 = (signed char)(item & 0xff), i1 = (signed char)((item >> 8) & 0xff);
    if (l == 0)
      lf[F_IT + s] = (i0 == a.env.item_a[0] && i1 == a.env.item_a[1]) ? 1.0f : 0.0f;
#if XH_8WH_KL_TU
    // the record: action (lane 0), advantage (lane 2, 0 for end rows), whether
    // the row counts (lane 3: not a terminal row past n_end, nor an open end
    // row whose env ended at step T - 1)
    const int dw = __builtin_amdgcn_readlane(r.rec, 1);
    const size_t qi1 = kind == 1 ? (size_t)(NT - a.b.N) + (g - NT) : 0;
    const int ended = (dw >> (8 * (int)(qi1 & 3))) & 0xff;
    const bool valid = kind == 0 || (kind == 1 ? ended == 0 : g - NT - a.b.N < n_end);
    if (l == 0 || l == 2) lf[F_REC + 4 * s + l] = kind == 0 ? __int_as_float(r.rec) : 0.0f;
    if (l == 3) lf[F_REC + 4 * s + 3] = valid ? 1.0f : 0.0f;
#else
    if (l < 3) lf[F_REC + 4 * s + l] = __int_as_float(r.rec);
#endif
  };
  // H1 values (C layout, r-tile rt) scaled by S_H -> the two f16 part images
  auto store_h1 = [&](const f32x4 &t, int sb, int rt) {
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    u32x2_t ph, pl;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      unsigned h2, l2;
      split2h_x2s(t[2 * u], t[2 * u + 1], SH, h2, l2);
      ph[u] = h2;
      pl[u] = l2;
    }
    st4h(sb + L_H1 + 4096 * rt, __builtin_bit_cast(f16x4, ph));
    st4h(sb + L_H1 + kImg + 4096 * rt, __builtin_bit_cast(f16x4, pl));
  };
  // layer 1 (C layout) of the group in slot s, all four r-tiles -> H1 image
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
    stage_store(stage_load(0), 0 KLTU(, 0));
    stage_store(stage_load(1), 1 KLTU(, 1));
  }
  __syncthreads();
  layer1_all(0, stb0);
  __syncthreads();
  layer2(rdb0, pre_cur, no_task);
  partials(pre_cur, lds4v(lf + F_W3 + fo), 0);
  __syncthreads();
  layer1_all(1, stb0);
  __syncthreads();

  for (int j = 0; j < J; ++j) {
    const int cs = j % 3, ns = (j + 2) % 3;  // slots of groups j and j + 2
    int rdb = rdb0, trm0 = trm00, trm1 = trm10, stb = stb0;
    asm volatile("" : "+v"(rdb), "+v"(trm0), "+v"(trm1), "+v"(stb), "+s"(gstep));
    S8H_STAMP(a, j, w, l, 0);
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
#if XH_8WH_KL_TU
    const float qv = lf[F_Q + cs * 64 + l];
    float kp = 0.0f, kg = 0.0f;
#endif
    f32x4 gx0[2], gx1[2];
    float ex = 0.0f, se = 0.0f, gz = 0.0f;
    f32x4 gr4, ggk[2], hT[2];
    bf16x8 bq0[3];
    bool item_cur = false;
    float b1t = 0.0f;
    f32x4 w3;
    auto xtask = [&](int k) {
      if (k == 16) S8H_STAMP_X(a, j, w, l, 1);
      if (k == 32) S8H_STAMP_X(a, j, w, l, 2);
      if (k == 44) S8H_STAMP_X(a, j, w, l, 3);
      if (k == 46) S8H_STAMP_X(a, j, w, l, 4);
      if (k == 0) {
        const float zs = ((z0[0] + z0[1]) + (z0[2] + z0[3])) +
                         ((z1[0] + z1[1]) + (z1[2] + z1[3]));
        ex = __expf(zs + b3);
      } else if (k == 1) {
        se = seg_sum<64>(ex);
#if XH_8WH_KL_TU
      } else if (k == 2) {
        // kl_regulated_loss (policy_gradient.h:41-85): softmax_gradient_log
        // + beta (p - q) as a probability-space gradient, through
        // softmax_layer::backward (nn.h:393-417) in the next slot; the KL sum
        // on one wave per group, in turn
        const int cu = __builtin_amdgcn_readfirstlane(__float_as_int(rec[0]));
        const float Ac = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rec[2])));
        const float p = ex * __builtin_amdgcn_rcpf(se);
        float gpv = fmaf(beta, p - qv, p * Ac);
        if (l == cu) gpv -= Ac;
        kp = p;
        kg = gpv;
        const bool vld = __builtin_amdgcn_readfirstlane(__float_as_int(rec[3])) != 0;
        if (vld && (j & 7) == w) kl_acc += (double)(qv * logf(qv / p));
#else
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
#endif
      } else if (k == 3) {
#if XH_8WH_KL_TU
        {
          const float sgv = seg_sum<64>(kp * kg);
          const bool vld = __builtin_amdgcn_readfirstlane(__float_as_int(rec[3])) != 0;
          gz = vld ? kp * (kg - sgv) : 0.0f;
        }
#endif
        gw[l] = gz;
        gp[4 * (l & 15) + (l >> 4)] = gz;
        accB3 += gz;  // wave 0's is written out
        item_cur = __builtin_amdgcn_readfirstlane(__float_as_int(itc)) != 0;
        b1t = lf[F_B1F + (item_cur ? 0 : kH) + 16 * w + li];
        // the rows of K-step 0 (T layout)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          gx0[h] = lds4v(xim + 16 * h + 4 * G);
          gx1[h] = lds4v(xim + 64 + 16 * h + 4 * G);
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
          hT[h][jj] = relu(fmaf(gx1[h][jj], w1b, fmaf(gx0[h][jj], w1a, b1t)));
      } else if (k >= 11 && k < 15) {
        // dW3 / db2 of r-tile rt (pre-activations in units of S2: dW3 is
        // unscaled at the write-out)
        const int rt = k - 11;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float v = pre_cur[rt][jj];
#if XH_8WH_IMASK
          // relu'(v) as an integer clamp of v's bits (v_med3: no compare,
          // no VCC hazard)
          const float gm = gr4[rt] * (float)relu_bit(v);
#else
          const float gm = v > 0.0f ? gr4[rt] : 0.0f;
#endif
          accW3[jj] = fmaf(gm, v, accW3[jj]);  // g relu(v)
          accB2[jj] += gm;                     // g M (w3 at the write-out)
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
        // the relu masks of r-tile k - 20 (C layout) -> the mask image (0 /
        // 0x4000: 2.0 as bf16 for dW2 and as f16 for dH1; the factor 2 is
        // taken back exactly at the write-outs)
        const int rt = k - 20;
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#if XH_8WH_IMASK
        // 0 / 1 per value from the bits, two per dword, times the 1.0 bits
        unsigned m[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          m[jj] = (unsigned)relu_bit(pre_cur[rt][jj]);
        // times the 2.0 bits by the full-rate 24-bit multiply (the 32-bit
        // one is quarter rate)
        const u32x2 mm = {(unsigned)__umul24(m[0] | (m[1] << 16), 0x4000u),
                          (unsigned)__umul24(m[2] | (m[3] << 16), 0x4000u)};
        st4(stb + L_MASK + 4096 * rt, __builtin_bit_cast(bf16x4, mm));
#else
        bf16x4 mk;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          mk[jj] = pre_cur[rt][jj] > 0.0f ? (__bf16)2.0f : (__bf16)0.0f;
        st4(stb + L_MASK + 4096 * rt, mk);
#endif
      } else if (k == 36) {
        w3 = lds4v(lf + F_W3 + fo);  // for the partial logits after layer 2
      } else if (k == 44) {
        // wave 0: group j+2's rows (loaded at the start of X(j)) into slot ns
        if (w == 0) stage_store(raw, ns KLTU(, j + 2));
      }
    };
    f32x4 pre_nx[4];
    layer2(rdb, pre_nx, xtask);
    S8H_STAMP_Y(a, j, w, l, 1);
    S8H_STAMP_X(a, j, w, l, 5);
    partials(pre_nx, w3, (j + 1) & 1);
    S8H_STAMP_Y(a, j, w, l, 2);
    S8H_STAMP_X(a, j, w, l, 6);
    __syncthreads();
    S8H_STAMP_Y(a, j, w, l, 3);
    S8H_STAMP_X(a, j, w, l, 7);

    // ================= Y(j): dW2 / dH1 of group j with VALU of j, j+2 =====
    // 32 blocks, alternating: even b dW2 block d = b / 2, three bf16 MFMAs
    // (ks = d / 8, ot = d % 8: dW2 += M^T (g (x) H1)), odd b dH1 block h =
    // b / 2, two f16 MFMAs (rt = h / 4, s = h % 4: S_D dH1 = M (S_D W2'), the
    // f16 mask image); operands one block ahead.  Alternating the two kinds
    // spreads their LDS reads and the layer-1 / dW1 VALU evenly over the
    // phase: 2.28 -> 2.21 ms per epoch against dW2 then dH1
    {
      float sg = 0.0f;
      bf16x8 bq1[3];
      f32x4 rx0[2], rx1[2], rgg[2], hT1[2];
      f32x4 wa, wb, bb, xp0, xp1, t1;
      float itn = 0.0f;
      f32x4 dx0, dx1, dgg;
      f32x4 dh[2];
      // blocks alternate: even bb_ dW2 block bb_ / 2, odd bb_ dH1 block
      // (bb_ - 1) / 2 (the two kinds' LDS reads and VALU interleaved)
      auto load_ops = [&](int bb_, bf16x8 &A) {
        const int b = bb_ >> 1;
        if ((bb_ & 1) == 0) {
          const int ks = b >> 3, ot = b & 7;
          A = ldtr((trm0 ^ (32 * ot)) + L_MASK + 8192 * ks,
                   (trm1 ^ (32 * ot)) + L_MASK + 8192 * ks);
        } else {
          const int rt = b >> 2, s = b & 3;
          A = ld8((rdb ^ (64 * s)) + L_MASK + 4096 * rt);  // read as f16
        }
      };
      // dW1 / db1 / item sums of value jj of r-tile rt (T layout)
      auto dw1 = [&](int jj, int rt) {
        const int q = rt & 1;
        const float tT = fmaf(dx1[jj], w1b, fmaf(dx0[jj], w1a, b1t));
#if XH_8WH_IMASK >= 2
        const float d = (dh[q][jj] * dgg[jj]) * (float)relu_bit(tT);
#else
        const float d = tT > 0.0f ? dh[q][jj] * dgg[jj] : 0.0f;
#endif
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
          // rows of K-step 1 (T-layout r-tiles 2, 3) and their g; group
          // j+2's item flag
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int r0 = 32 + 16 * h + 4 * G;
            rx0[h] = lds4v(xim + r0);
            rx1[h] = lds4v(xim + 64 + r0);
            rgg[h] = lds4v(gw + r0);
          }
          itn = lf[F_IT + ns];
        } else if (b == 2 || b == 3) {
          const int h = b - 2;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            hT1[h][jj] = relu(fmaf(rx1[h][jj], w1b, fmaf(rx0[h][jj], w1a, b1t)));
        } else if (b >= 4 && b < 8) {
          // g (x) H1 of K-step 1, two values per slot
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
            // group j+2's layer-1 operands (C layout)
            wa = lds4v(lf + F_W1T + fo);
            wb = lds4v(lf + F_W1T + kH + fo);
            xp0 = lds4v(lf + F_XP + ns * 128 + 4 * li);
            xp1 = lds4v(lf + F_XP + ns * 128 + 64 + 4 * li);
          } else if (b == 5) {
            const bool ia = __builtin_amdgcn_readfirstlane(__float_as_int(itn)) != 0;
            bb = lds4v(lf + F_B1F + (ia ? 0 : kH) + fo);
          }
        } else if ((b & 1) == 0 && b >= 8 && b < 24) {
          // layer 1 of group j+2 in the dW2 blocks' slots, r-tile (b - 8) /
          // 4: values, then the split stores
          layer1_rt((b - 8) >> 2, (b >> 1) & 1, stb);
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
      bf16x8 A_c, A_n;
      load_ops(0, A_c);
#pragma unroll
      for (int b = 0; b < 32; ++b) {
        if (b + 1 < 32) load_ops(b + 1, A_n);
        FENCE();
        if ((b & 1) == 0) {
          const int ot = (b >> 1) & 7;
          const bf16x8(&bq)[3] = (b >> 1) < 8 ? bq0 : bq1;
          accW2[ot] = mfma16(A_c, bq[2], accW2[ot]);
          accW2[ot] = mfma16(A_c, bq[1], accW2[ot]);
          accW2[ot] = mfma16(A_c, bq[0], accW2[ot]);
        } else {
          const int rt = (b >> 1) >> 2, s = (b >> 1) & 3, q = rt & 1;
          if (s == 0) dh[q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
          const f16x8 Ah = __builtin_bit_cast(f16x8, A_c);
          dh[q] = mfma16h(Ah, wd[s][1], dh[q]);
          dh[q] = mfma16h(Ah, wd[s][0], dh[q]);
        }
        FENCE();
        ytask(b);
        FENCE();
        A_c = A_n;
      }
      S8H_STAMP_Y(a, j, w, l, 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) dw1(s, 3);
      if (item_cur)
        sa += sg;
      else
        sb += sg;
      S8H_STAMP_Y(a, j, w, l, 5);
    }
    __syncthreads();
    S8H_STAMP_Y(a, j, w, l, 6);
    S8H_STAMP_Y(a, j, w, l, 7);
    // rotate the pipeline
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) pre_cur[rt] = pre_nx[rt];
  }

#if XH_8WH_KL_TU
  {
    // the workgroup's KL sum (the loop's last barrier is behind: F_Z is free)
    double v = kl_acc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o, kWave);
    double *kd = reinterpret_cast<double *>(lf + F_Z);
    if (l == 0) kd[w] = v;
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
  // every entry has exactly one producing lane
  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
  const float *w3g = P + PL.ow3();
#pragma unroll
  for (int ot = 0; ot < 8; ++ot)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = 16 * ot + 4 * G + j;
      slab[PL.oW2() + o * kH + 16 * w + li] = (accW2[ot][j] * 0.5f) * w3g[o];
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
    tw0 *= 0.5f / SD;  // (and the masks were 2.0)
    tw1 *= 0.5f / SD;
    va *= 0.5f / SD;
    vb *= 0.5f / SD;
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

}  // namespace s8h

#if XH_8WH_KL_TU
hipError_t launch_policy_train_split8wh_kl(const PolicyTrainArgs &a, int grid,
                                           hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s8h::policy_train_split8wh_kl_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s8h::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s8h::policy_train_split8wh_kl_kernel, dim3(grid),
                     dim3(s8h::kThreads), s8h::kLds, s, a);
  return hipGetLastError();
}
#else
hipError_t launch_policy_train_split8wh(const PolicyTrainArgs &a, int grid,
                                        hipStream_t s) {
  if (a.algo == kKLPPO) return launch_policy_train_split8wh_kl(a, grid, s);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s8h::policy_train_split8wh_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s8h::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s8h::policy_train_split8wh_kernel, dim3(grid),
                     dim3(s8h::kThreads), s8h::kLds, s, a);
  return hipGetLastError();
}
#endif

}  // namespace xh
