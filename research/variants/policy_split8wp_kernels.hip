// policy_split8wp_kernels.hip -- the PPO / actor-critic train epoch of the
// 64-bin 2-D [128,128] policy (BASELINE configs 3 and 4), software-pipelined
// over the row groups of a workgroup: the arithmetic of policy_split8w_kernels
// .hip (eight waves, two per SIMD, 16x16x32 bf16 MFMAs on exactly split f32
// operands, rank-1 backward; see xh_split.h), with every VALU phase of a
// group placed between the MFMAs of another group's GEMMs.
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
#define S8P_STAMP(a, gi, w, lane, slot)                                         \
  do {                                                                        \
    if ((a).trace && blockIdx.x < kTraceBlocks && (gi) < kTraceGroups &&      \
        (lane) == 0)                                                          \
      (a).trace[((blockIdx.x * kTraceGroups + (gi)) * 8 + (w)) * kTraceSlots + \
                (slot)] = clock64();                                          \
  } while (0)
#else
#define S8P_STAMP(a, gi, w, lane, slot) \
  do {                                  \
  } while (0)
#endif

namespace xh {
namespace s8p {

constexpr int kB = 64, kD = 2, kF0 = 2 * kD, kH = 128;
constexpr int kThreads = 512;
constexpr int kImg = 64 * kImgRow;  // one 64-row part image, 16 KB
// LDS carve (bytes): the H1 image (three parts), the mask image, the lo
// parts of W2 (layer 2's A operand) and of W2' (dH1's B operand), then f32
constexpr int L_H1 = 0;
constexpr int L_MASK = 3 * kImg;
constexpr int L_W2LO = 4 * kImg;
constexpr int L_WDLO = 6 * kImg;
constexpr int L_F = 8 * kImg;
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
constexpr int F_END = F_REC + 3 * 4;
constexpr size_t kLds = L_F + sizeof(float) * F_END;
static_assert(kLds <= 160 * 1024, "LDS");
static_assert(F_REC % 4 == 0 && F_GW % 4 == 0 && F_GP % 4 == 0 && F_X % 4 == 0 && F_XP % 4 == 0 &&
                  F_Z % 4 == 0 && F_W1T % 4 == 0 && F_B1F % 4 == 0,
              "16-byte aligned f32 vectors");

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x8 lbf16x8;
typedef __attribute__((address_space(3))) bf16x4 lbf16x4;
typedef __attribute__((address_space(3))) s16x4 ls16x4;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
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

__global__ __launch_bounds__(kThreads, 2) void policy_train_split8wp_kernel(
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

  // ---- prologue: small parameters into LDS, the split W2 / W2' fragments
  // of tile w into registers (hi / mid) and the lo images
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
    lf[F_B2 + i] = P[PL.ob2() + i];
    lf[F_W3 + i] = P[PL.ow3() + i];
  }
  if (tid == 0) lf[F_B3] = P[PL.ob3()];
  bf16x8 wl[4][2], wd[4][2];
  const int rdb0 = rd_base(G, li);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float4 *src = reinterpret_cast<const float4 *>(
        P + PL.oW2() + (16 * w + li) * kH + 32 * s + 8 * G);
    const float4 v0 = src[0], v1 = src[1];
    const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    bf16x8 lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 x0, x1, x2;
      split3(v[j], x0, x1, x2);
      wl[s][0][j] = x0;
      wl[s][1][j] = x1;
      lo[j] = x2;
    }
    *reinterpret_cast<bf16x8 *>(lds + L_W2LO + ((rdb0 ^ (64 * s)) + 4096 * w)) = lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = 32 * s + 8 * G + j, col = 16 * w + li;
      __bf16 x0, x1, x2;
      split3(P[PL.oW2() + o * kH + col] * P[PL.ow3() + o], x0, x1, x2);
      wd[s][0][j] = x0;
      wd[s][1][j] = x1;
      *reinterpret_cast<__bf16 *>(lds + L_WDLO + ioff2(o, col >> 3) + 2 * (col & 7)) =
          x2;
    }
  }
  // per-lane absolute LDS bases (the region offsets that exceed the 16-bit
  // immediate folded in)
  const int rdw0 = L_W2LO + 4096 * w + rdb0;  // ^ 64 s
  const int trm00 = trm_base(l, 0), trm10 = trm_base(l, 1);  // ^ 32 ot, + L_MASK
  const int trw00 = (trw_base(l, 0) ^ (32 * w)) + L_WDLO;    // + 8192 s
  const int trw10 = (trw_base(l, 1) ^ (32 * w)) + L_WDLO;
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
    const int *src = l == 0   ? a.b.action + ti
                     : l == 1 ? reinterpret_cast<const int *>(a.b.pold + ti)
                     : l == 2 ? reinterpret_cast<const int *>(a.adv + ti)
                              : reinterpret_cast<const int *>(a.b.items + ti * 4);
    return Raw{bins, *src};
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
      bf16x4 ph, pm, pl;
      split4(t, ph, pm, pl);
      st4(stb + L_H1 + 4096 * rt, ph);
      st4(stb + L_H1 + kImg + 4096 * rt, pm);
      st4(stb + L_H1 + 2 * kImg + 4096 * rt, pl);
    }
  };
  // layer 2 of the group whose H1 is in the image: 16 steps of 6 MFMAs (A =
  // W2 tile w, B = H1 rows 16 rt + li), pre = b2 + W2 . H1; task(k) runs
  // after each block of three (k = 0 .. 31)
  auto layer2 = [&](int rdb, int rdw, f32x4 (&pre)[4], auto &&task) {
    const f32x4 b2 = lds4v(lf + F_B2 + fo);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) pre[rt] = b2;
    bf16x8 b_c[3], b_n[3], lo_c = ld8(rdw), lo_n = lo_c;
#pragma unroll
    for (int p = 0; p < 3; ++p) b_c[p] = ld8(rdb + L_H1 + p * kImg);
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int s = st >> 2, rt = st & 3;
      if (st + 1 < 16) {
        const int s1 = (st + 1) >> 2, r1 = (st + 1) & 3;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          b_n[p] = ld8((rdb ^ (64 * s1)) + L_H1 + p * kImg + 4096 * r1);
        if (rt == 3) lo_n = ld8(rdw ^ (64 * s1));
      }
      FENCE();
      // the six products, small terms first (xh_split.h)
      pre[rt] = mfma16(wl[s][1], b_c[1], pre[rt]);
      pre[rt] = mfma16(wl[s][0], b_c[2], pre[rt]);
      pre[rt] = mfma16(lo_c, b_c[0], pre[rt]);
      FENCE();
      task(2 * st);
      FENCE();
      pre[rt] = mfma16(wl[s][0], b_c[1], pre[rt]);
      pre[rt] = mfma16(wl[s][1], b_c[0], pre[rt]);
      pre[rt] = mfma16(wl[s][0], b_c[0], pre[rt]);
      FENCE();
      task(2 * st + 1);
      FENCE();
#pragma unroll
      for (int p = 0; p < 3; ++p) b_c[p] = b_n[p];
      if (rt == 3) lo_c = lo_n;
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
  Raw raw = {0, 0};
  if (w == 0) {
    stage_store(stage_load(0), 0);
    stage_store(stage_load(1), 1);
  }
  __syncthreads();
  layer1_all(0, stb0);
  __syncthreads();
  layer2(rdb0, rdw0, pre_cur, no_task);
  partials(pre_cur, lds4v(lf + F_W3 + fo), 0);
  __syncthreads();
  layer1_all(1, stb0);
  __syncthreads();

  for (int j = 0; j < J; ++j) {
    const int cs = j % 3, ns = (j + 2) % 3;  // slots of groups j and j + 2
    int rdb = rdb0, rdw = rdw0, trm0 = trm00, trm1 = trm10, trw0 = trw00,
        trw1 = trw10, stb = stb0;
    asm volatile("" : "+v"(rdb), "+v"(rdw), "+v"(trm0), "+v"(trm1), "+v"(trw0),
                 "+v"(trw1), "+v"(stb), "+s"(gstep));
    S8P_STAMP(a, j, w, l, 0);
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
    f32x4 gx0[2], gx1[2];
    float ex = 0.0f, se = 0.0f, gz = 0.0f;
    f32x4 gr4, ggk[2], hT[2];
    bf16x8 bq0[3];
    bool item_cur = false;
    float b1t = 0.0f;
    f32x4 w3;
    auto xtask = [&](int k) {
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
        // the rows of K-step 0 (T layout)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          gx0[h] = lds4v(xim + 16 * h + 4 * G);
          gx1[h] = lds4v(xim + 64 + 16 * h + 4 * G);
        }
      } else if (k == 4) {
        gr4 = lds4v(gp + 4 * li);  // g of rows 16 rt + li
#pragma unroll
        for (int h = 0; h < 2; ++h) ggk[h] = lds4v(gw + 16 * h + 4 * G);
      } else if (k == 5 || k == 6) {
        // layer-1 values of K-step 0's rows (T layout), r-tile h
        const int h = k - 5;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          hT[h][jj] = relu(fmaf(gx1[h][jj], w1b, fmaf(gx0[h][jj], w1a, b1t)));
      } else if (k >= 8 && k < 12) {
        // dW3 / db2 of r-tile rt
        const int rt = k - 8;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float v = pre_cur[rt][jj];
          const float gm = v > 0.0f ? gr4[rt] : 0.0f;
          accW3[jj] = fmaf(gm, v, accW3[jj]);  // g relu(v)
          accB2[jj] += gm;                     // g M (w3 at the write-out)
        }
      } else if (k >= 12 && k < 16) {
        // g (x) H1 of K-step 0, two values per slot
        const int h = (k - 12) >> 1, j0 = 2 * ((k - 12) & 1);
#pragma unroll
        for (int jj = j0; jj < j0 + 2; ++jj) {
          __bf16 p0, p1, p2;
          split3(hT[h][jj] * ggk[h][jj], p0, p1, p2);
          bq0[0][4 * h + jj] = p0;
          bq0[1][4 * h + jj] = p1;
          bq0[2][4 * h + jj] = p2;
        }
      } else if (k == 24) {
        w3 = lds4v(lf + F_W3 + fo);  // for the partial logits after layer 2
      } else if (k == 30) {
        // wave 0: group j+2's rows (loaded at the start of X(j)) into slot ns
        if (w == 0) stage_store(raw, ns);
      }
      if (k < 4) {
        // the relu masks of r-tile k (C layout) -> mask image
        bf16x4 mk;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          mk[jj] = pre_cur[k][jj] > 0.0f ? (__bf16)1.0f : (__bf16)0.0f;
        st4(stb + L_MASK + 4096 * k, mk);
      }
    };
    f32x4 pre_nx[4];
    layer2(rdb, rdw, pre_nx, xtask);
    S8P_STAMP(a, j, w, l, 1);
    partials(pre_nx, w3, (j + 1) & 1);
    S8P_STAMP(a, j, w, l, 2);
    __syncthreads();
    S8P_STAMP(a, j, w, l, 3);

    // ================= Y(j): dW2 / dH1 of group j with VALU of j, j+2 =====
    // 32 blocks of three MFMAs: b < 16 dW2 (ks = b / 8, ot = b % 8: dW2 +=
    // M^T (g (x) H1)), b >= 16 dH1 (rt = (b - 16) / 4, s = (b - 16) % 4:
    // dH1 = M W2'); operands one block ahead
    {
      float sg = 0.0f;
      bf16x8 bq1[3];
      f32x4 rx0[2], rx1[2], rgg[2], hT1[2];
      f32x4 wa, wb, bb, xp0, xp1, t1;
      float itn = 0.0f;
      f32x4 dx0, dx1, dgg;
      f32x4 dh[2];
      auto load_ops = [&](int b, bf16x8 &A, bf16x8 &L) {
        if (b < 16) {
          const int ks = b >> 3, ot = b & 7;
          A = ldtr((trm0 ^ (32 * ot)) + L_MASK + 8192 * ks,
                   (trm1 ^ (32 * ot)) + L_MASK + 8192 * ks);
        } else {
          const int rt = (b - 16) >> 2, s = (b - 16) & 3;
          A = ld8((rdb ^ (64 * s)) + L_MASK + 4096 * rt);
          L = ldtr(trw0 + 8192 * s, trw1 + 8192 * s);
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
          bf16x4 ph, pm, pl;
          split4(t1, ph, pm, pl);
          st4(sb + L_H1 + 4096 * rt, ph);
          st4(sb + L_H1 + kImg + 4096 * rt, pm);
          st4(sb + L_H1 + 2 * kImg + 4096 * rt, pl);
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
        } else if (b >= 8 && b < 16) {
          // layer 1 of group j+2, r-tile (b - 8) / 2: values, then the
          // split stores
          layer1_rt((b - 8) >> 1, b & 1, stb);
        } else {
          const int rt = (b - 16) >> 2, s = (b - 16) & 3;
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
      bf16x8 A_c, L_c, A_n, L_n;
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
          dh[q] = mfma16(A_c, L_c, dh[q]);
          dh[q] = mfma16(A_c, wd[s][1], dh[q]);
          dh[q] = mfma16(A_c, wd[s][0], dh[q]);
        }
        FENCE();
        ytask(b);
        FENCE();
        A_c = A_n;
        L_c = L_n;
      }
      S8P_STAMP(a, j, w, l, 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) dw1(s, 3);
      if (item_cur)
        sa += sg;
      else
        sb += sg;
      S8P_STAMP(a, j, w, l, 5);
    }
    __syncthreads();
    S8P_STAMP(a, j, w, l, 6);
    S8P_STAMP(a, j, w, l, 7);
    // rotate the pipeline
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) pre_cur[rt] = pre_nx[rt];
  }

  // ---------------------------------------------------- slab write-out ----
  // every entry has exactly one producing lane
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
    // dW3 / db2 of o = 16w + 4G + j: sums over the 16 lanes (rows) of group G
    const float s3 = seg_sum<16>(accW3[j]);
    const float s2 = seg_sum<16>(accB2[j]);
    const int o = 16 * w + 4 * G + j;
    if (li == 0) {
      slab[PL.ow3() + o] = s3;
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

}  // namespace s8p

hipError_t launch_policy_train_split8wp(const PolicyTrainArgs &a, int grid,
                                        hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s8p::policy_train_split8wp_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s8p::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s8p::policy_train_split8wp_kernel, dim3(grid),
                     dim3(s8p::kThreads), s8p::kLds, s, a);
  return hipGetLastError();
}

}  // namespace xh
