// policy_split4p_kernels.hip -- the PPO / actor-critic train epoch of the
// 64-bin 2-D [128,128] policy (BASELINE configs 3 and 4): four waves, one per
// SIMD with up to 512 registers each, v_mfma_f32_32x32x16_bf16 on exactly
// split f32 operands (xh_split.h) with the rank-1 backward of
// policy_split_kernels.hip, software-pipelined over the row groups of a
// workgroup as policy_split8wp_kernels.hip is.
//
// Why this shape: the 8-wave kernel is bound by the issue port of its SIMDs
// (MI355X_MICROARCH.md: a v_mfma_f32_16x16x32_bf16 holds the SIMD's vector
// issue for 8 of its 16 cycles, a 32x32x16 for 8 of its 32) and by its two
// waves per SIMD running the same phases in lockstep (the older wave's VALU
// wins the arbitration; phase stamps: the younger half ends each phase
// 1.7-1.9k cycles after the older one).  Here one wave per SIMD issues its
// MFMAs back to back with about five VALU instructions hidden in each 32-cycle
// gap, and the 512-register budget holds two groups in flight:
//
//   X(j): MFMA  layer 2 of group j+1 (96 per wave)
//         VALU  softmax + loss gradient of group j, its relu masks (image),
//               dW3 / db2 sums, g (x) H1 of its first 32 rows (dW2's B
//               fragments, registers); then group j+1's partial logits
//                                                     -> barrier
//   Y(j): MFMA  dH1 of group j (48 per wave), then dW2 (48)
//         VALU  g (x) H1 of rows 32..63, layer 1 of group j+2 (-> H1 image),
//               dW1 / db1 / item sums of group j      -> barrier
//
// Wave q owns 32-wide tile q of every product (xh_split.h 32x32x16 maps):
//   layer 2  C[o][r]: lane = row r, registers = o in H2 tile q
//   dH1      C[r][i]: lane = i in H1 tile q, registers = rows ("T layout")
//   dW2      C[o][i] of tiles (n, q), n = 0..3, K = the 64 rows: A = M^T by
//            transposed reads of the mask image, B = g (x) H1 in registers
// dW2's K order follows the T layout: K-slice s = 2 rt + sg holds in lane
// half h the rows 32 rt + 16 sg + 4 h + e (e < 4) and + 8 + 4 h + e - 4
// (e >= 4), i.e. registers 8 sg + e of the T-layout tile rt; the mask's
// transposed reads supply the same rows (trp_base).
#include <cstdlib>

#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

// Phase stamps (trace build, -DXH_DIAG_TRACE=1, run with XH_PHASE_TRACE=1):
// lane 0 of every wave of the first kTraceBlocks workgroups records the cycle
// counter at 0 X start, 1 layer 2 (+ group j's VALU) done, 2 partial logits
// written, 3 after the X barrier, 4 dH1 / dW2 blocks done, 5 dW1 tail done,
// 6 after the Y barrier (7 = 6), for its first kTraceGroups groups.
#ifndef XH_DIAG_TRACE
#define XH_DIAG_TRACE 0
#endif
#if XH_DIAG_TRACE
#define S4P_STAMP(a, gi, w, lane, slot)                                         \
  do {                                                                        \
    if ((a).trace && blockIdx.x < kTraceBlocks && (gi) < kTraceGroups &&      \
        (lane) == 0)                                                          \
      (a).trace[((blockIdx.x * kTraceGroups + (gi)) * 8 + (w)) * kTraceSlots + \
                (slot)] = clock64();                                          \
  } while (0)
#else
#define S4P_STAMP(a, gi, w, lane, slot) \
  do {                                  \
  } while (0)
#endif

namespace xh {
namespace s4p {

constexpr int kB = 64, kD = 2, kF0 = 2 * kD, kH = 128;
constexpr int kThreads = 256;
constexpr int kImg = 64 * kImgRow;  // one 64-row part image, 16 KB
// LDS carve (bytes): the H1 image (three parts), the mask image, the lo parts
// of W2' (dH1's B operand) and of W2 (layer 2's A operand), then f32.  The
// prologue's W2 / W2' hi + mid images (2 x 32 KB) alias [0, 4 kImg).
constexpr int L_H1 = 0;
constexpr int L_MASK = 3 * kImg;
constexpr int L_WDLO = 4 * kImg;
constexpr int L_W2LO = 6 * kImg;
constexpr int L_F = 8 * kImg;
constexpr int F_W1T = 0;                // [2 k][128 i]: W1[i][k], the bin columns
constexpr int F_B1F = F_W1T + 2 * kH;   // [2 items][128]: b1 + the item's part
constexpr int F_B2 = F_B1F + 2 * kH;    // [128]
constexpr int F_W3 = F_B2 + kH;         // [128]
constexpr int F_B3 = F_W3 + kH;         // [4]
constexpr int F_Z = F_B3 + 4;           // [2 parity][4 waves][64 rows] partial logits
constexpr int F_GW = F_Z + 2 * 4 * 64;  // [4 waves][64 rows] g, row order
constexpr int F_X = F_GW + 4 * 64;      // [3 slots][2 dims][64 rows] bins / 8
constexpr int F_IT = F_X + 3 * kD * 64;  // [3 slots] the group's item is item_a
constexpr int F_REC = F_IT + 4;         // [3 slots][action bits, pold, adv, -]
constexpr int F_ACC = F_REC + 3 * 4;    // [4 waves][16 j][64 lanes] dW3 sums
constexpr int F_END = F_ACC + 4 * 16 * 64;
constexpr size_t kLds = L_F + sizeof(float) * F_END;
static_assert(kLds <= 160 * 1024, "LDS");
static_assert(F_REC % 4 == 0 && F_GW % 4 == 0 && F_X % 4 == 0 && F_Z % 4 == 0 &&
                  F_W3 % 4 == 0 && F_B1F % 4 == 0 && F_B2 % 4 == 0,
              "16-byte aligned f32 vectors");

// dW2's A operand (the mask image M[row][o], transposed reads) in the T
// layout's row order: read t of lane l (16-lane group g, index 4 qq + p)
// supplies row 8 t + 4 h + qq of the K-slice (+ 16 s rows: + 4096 s bytes),
// columns 4 p .. 4 p + 3 of chunk 2 (g & 1) + (p >> 1) of o-tile 0 (o-tile n:
// ^ 64 n).  Conflict-free: per 32-lane half four rows x four chunks.
__device__ __forceinline__ int trp_base(int l, int t) {
  const int g = l >> 4, li = l & 15, qq = li >> 2, p = li & 3, h = l >> 5;
  const int row = 8 * t + 4 * h + qq;
  const int ch = 2 * (g & 1) + (p >> 1);
  return kImgRow * row + 16 * (ch ^ img_swz(row)) + 8 * (p & 1);
}
__device__ __forceinline__ bf16x8 ldtr_at(const char *lds, int o0, int o1) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(lds + o0));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(lds + o1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, v);
}
using split::lds4;
using split::relu;
#define FENCE() __builtin_amdgcn_sched_barrier(0)

__global__ __launch_bounds__(kThreads, 1) void policy_train_split4p_kernel(
    PolicyTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH, kH};
  const float *P = a.params;
  const int tid = threadIdx.x;
  const int q = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int l = tid & 63, lr = l & 31, h = l >> 5;
  const int ngroups = a.b.T * a.b.N;
  // this workgroup's groups: g_j = blockIdx.x + j gridDim.x, j < J (the
  // host caps the grid at the group count); indices past the end are clamped
  // to the last group (layer 1 / layer 2 run ahead; their work is discarded)
  const int J = ((ngroups - (int)blockIdx.x) + (int)gridDim.x - 1) / (int)gridDim.x;
  if (J <= 0) return;  // uniform over the workgroup
  int gstep = (int)gridDim.x;
  auto tindex = [&](int j) {
    return (size_t)((int)blockIdx.x + min(j, J - 1) * gstep);
  };

  // ---- prologue: small parameters, the split W2 / W2' images, the
  // fragments of tile q into registers (hi / mid), the lo images
  for (int e = tid; e < kH * kH; e += kThreads) {
    const int o = e >> 7, i = e & 127;
    __bf16 x0, x1, x2;
    split3(P[PL.oW2() + e], x0, x1, x2);
    const int off = img_off(o, i >> 3) + 2 * (i & 7);
    *reinterpret_cast<__bf16 *>(lds + off) = x0;
    *reinterpret_cast<__bf16 *>(lds + 128 * kImgRow + off) = x1;
    *reinterpret_cast<__bf16 *>(lds + L_W2LO + off) = x2;
  }
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
  __syncthreads();
  // per-lane LDS bases (xh_split.h): rows lr / 32 + lr of the row images,
  // row 32 q + lr of W2's, the transposed reads of column tile q, the stores
  // (made opaque at every group, so the compiler recomputes the one XOR per
  // read instead of holding dozens of hoisted addresses)
  int rb0 = row_base(lr, h), rb1 = row_base(32 + lr, h);
  int rbw = row_base(q * 32 + lr, h);
  int tq0 = tr_base(l, 0) ^ (64 * q), tq1 = tr_base(l, 1) ^ (64 * q);
  int sb0 = st_base(lr, h), sb1 = st_base(32 + lr, h);
  int tp0 = trp_base(l, 0) + L_MASK, tp1 = trp_base(l, 1) + L_MASK;
  bf16x8 wl[8][2], wd[8][2];
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int p = 0; p < 2; ++p) wl[s][p] = ld_row(lds + p * 128 * kImgRow, rbw, s);
  __syncthreads();  // the W2 images' LDS becomes W2''s
  for (int e = tid; e < kH * kH; e += kThreads) {
    const int o = e >> 7, i = e & 127;
    __bf16 x0, x1, x2;
    split3(P[PL.oW2() + e] * P[PL.ow3() + o], x0, x1, x2);
    const int off = img_off(o, i >> 3) + 2 * (i & 7);
    *reinterpret_cast<__bf16 *>(lds + off) = x0;
    *reinterpret_cast<__bf16 *>(lds + 128 * kImgRow + off) = x1;
    *reinterpret_cast<__bf16 *>(lds + L_WDLO + off) = x2;
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int p = 0; p < 2; ++p) wd[s][p] = ld_tr(lds + p * 128 * kImgRow, tq0, tq1, s);
  __syncthreads();  // [0, 4 kImg) becomes the row images

  char *const h1i[3] = {lds + L_H1, lds + L_H1 + kImg, lds + L_H1 + 2 * kImg};
  float *const gw = lf + F_GW + 64 * q;  // this wave's copy of the rows' g

  f32x16 accW2[4];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
#pragma unroll
    for (int n = 0; n < 4; ++n) accW2[n][j] = 0.0f;
  }
  // dW3 / db2 per-lane partial sums in LDS (register pressure), read-
  // modify-written once per group: [j][lane] for this wave
  float *const accw3 = lf + F_ACC + q * 1024;
  float accB2[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    accw3[64 * j + l] = 0.0f;
    accB2[j] = 0.0f;
  }
  float accB3 = 0.0f, w0 = 0.0f, w1 = 0.0f, sa = 0.0f, sb = 0.0f;

  // wave 0 stages group j+2 during X(j): branch-free loads at its start
  // (lane = row: the row's two bins; lanes 0-2 the action, old probability
  // and advantage, the others the item's first two coordinates), the stores
  // into slot s (bins / 8, whether the item is item_a, the record) late in
  // the same phase, so the loads' latency hides under layer 2
  struct Raw {
    int bi, rec;
  };
  auto stage_load = [&](int j) {
    const size_t ti = tindex(j);
    int lo = l * kD;
    asm volatile("" : "+v"(lo));
    const int bins =
        *reinterpret_cast<const unsigned short *>(a.b.bins + ti * (kB * kD) + lo);
    const int *src = l == 0   ? a.b.action + ti
                     : l == 1 ? reinterpret_cast<const int *>(a.b.pold + ti)
                     : l == 2 ? reinterpret_cast<const int *>(a.adv + ti)
                              : reinterpret_cast<const int *>(a.b.items + ti * 4);
    return Raw{bins, *src};
  };
  auto stage_store = [&](const Raw &r, int s) {
    lf[F_X + s * 128 + l] = (float)(signed char)(r.bi & 0xff) / (float)kCapacity;
    lf[F_X + s * 128 + 64 + l] =
        (float)(signed char)((r.bi >> 8) & 0xff) / (float)kCapacity;
    const int item = __builtin_amdgcn_readlane(r.rec, 3);
    const int i0 = (signed char)(item & 0xff), i1 = (signed char)((item >> 8) & 0xff);
    if (l == 0)
      lf[F_IT + s] = (i0 == a.env.item_a[0] && i1 == a.env.item_a[1]) ? 1.0f : 0.0f;
    if (l < 3) lf[F_REC + 4 * s + l] = __int_as_float(r.rec);
  };
  // the layer-1 bias row of the group in slot s (item folded in)
  auto b1row = [&](int s) {
    const bool ia =
        __builtin_amdgcn_readfirstlane(__float_as_int(lf[F_IT + s])) != 0;
    return lf + F_B1F + (ia ? 0 : kH);
  };
  // layer 1 of the group in slot s, r-tile rt, C layout (lane = row, H1 tile
  // q in registers): one f32 MFMA over the two bin features
  auto layer1_c = [&](int s, int rt, const float *b1f) {
    f32x16 t = split::lds_acc16(b1f, q * 32, h);
    const float xb = lf[F_X + s * 128 + h * 64 + rt * 32 + lr];
    const float wa = lf[F_W1T + h * kH + q * 32 + lr];
    return mfma32(wa, xb, t);
  };
  // the same values transposed (lane = feature 32 q + lr, registers = rows
  // 32 rt + acc_row(j, h)): the same two products, bit-identical
  auto layer1_t = [&](int s, int rt, const float *b1f) {
    const float b1T = b1f[q * 32 + lr];
    f32x16 t;
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = b1T;
    const float xb = lf[F_X + s * 128 + h * 64 + rt * 32 + lr];
    const float wa = lf[F_W1T + h * kH + q * 32 + lr];
    return mfma32(xb, wa, t);
  };
  auto store_h1 = [&](const f32x16 &t, int rt) {
    f32x16 r;
#pragma unroll
    for (int j = 0; j < 16; ++j) r[j] = relu(t[j]);
    img_store_split_b(h1i[0], h1i[1], h1i[2], rt == 0 ? sb0 : sb1, q * 32, r);
  };
  // layer 2 of the group whose H1 is in the image: 16 steps (K-slice st / 2,
  // r-tile st % 2) of 6 MFMAs, task(k) after each block of three
  auto layer2 = [&](f32x16 (&pre)[2], auto &&task) {
    pre[0] = split::lds_acc16(lf + F_B2, q * 32, h);
    pre[1] = pre[0];
    bf16x8 lo_c = ld_row(lds + L_W2LO, rbw, 0), lo_n = lo_c, b_c[3], b_n[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) b_c[p] = ld_row(h1i[p], rb0, 0);
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int s = st >> 1, rt = st & 1;
      if (st + 1 < 16) {
        const int s1 = (st + 1) >> 1, r1 = (st + 1) & 1;
#pragma unroll
        for (int p = 0; p < 3; ++p) b_n[p] = ld_row(h1i[p], r1 ? rb1 : rb0, s1);
        if (r1 == 0) lo_n = ld_row(lds + L_W2LO, rbw, s1);
      }
      FENCE();
      // the six products, small terms first (xh_split.h)
      pre[rt] = mfma_bf16(wl[s][1], b_c[1], pre[rt]);
      pre[rt] = mfma_bf16(wl[s][0], b_c[2], pre[rt]);
      pre[rt] = mfma_bf16(lo_c, b_c[0], pre[rt]);
      FENCE();
      task(2 * st);
      FENCE();
      pre[rt] = mfma_bf16(wl[s][0], b_c[1], pre[rt]);
      pre[rt] = mfma_bf16(wl[s][1], b_c[0], pre[rt]);
      pre[rt] = mfma_bf16(wl[s][0], b_c[0], pre[rt]);
      FENCE();
      task(2 * st + 1);
      FENCE();
#pragma unroll
      for (int p = 0; p < 3; ++p) b_c[p] = b_n[p];
      if (rt == 1) lo_c = lo_n;
    }
  };
  // partial logits of rows 32 rt + lr over this wave's features -> F_Z[zs]
  auto partials = [&](const f32x16 (&pre)[2], int zs) {
    const f32x16 w3 = split::lds_acc16(lf + F_W3, q * 32, h);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      float zp = 0.0f;
#pragma unroll
      for (int j = 0; j < 16; ++j) zp = fmaf(relu(pre[rt][j]), w3[j], zp);
      zp += half_swap(zp);
      if (l < 32) lf[F_Z + zs * 256 + q * 64 + rt * 32 + lr] = zp;
    }
  };
  auto no_task = [](int) {};

  // ---- pipeline prologue: groups 0 and 1 staged, layer 1 and layer 2 of
  // group 0 (its partial logits), layer 1 of group 1
  f32x16 pre_cur[2];
  Raw raw = {0, 0};
  if (q == 0) {
    stage_store(stage_load(0), 0);
    stage_store(stage_load(1), 1);
  }
  __syncthreads();
  {
    const float *b1f = b1row(0);
    store_h1(layer1_c(0, 0, b1f), 0);
    store_h1(layer1_c(0, 1, b1f), 1);
  }
  __syncthreads();
  layer2(pre_cur, no_task);
  partials(pre_cur, 0);
  __syncthreads();
  {
    const float *b1f = b1row(1);
    store_h1(layer1_c(1, 0, b1f), 0);
    store_h1(layer1_c(1, 1, b1f), 1);
  }
  __syncthreads();

  for (int j = 0; j < J; ++j) {
    const int cs = j % 3, ns = (j + 2) % 3;  // slots of groups j and j + 2
    S4P_STAMP(a, j, q, l, 0);
    asm volatile("" : "+v"(rb0), "+v"(rb1), "+v"(rbw), "+v"(tq0), "+v"(tq1), "+v"(sb0),
                 "+v"(sb1), "+v"(tp0), "+v"(tp1), "+s"(gstep));
    if (q == 0) raw = stage_load(j + 2);
    const float *xim = lf + F_X + cs * 128;

    // ================= X(j): layer 2 of group j+1 with group j's VALU ====
    const float z0 = lf[F_Z + (j & 1) * 256 + l], z1 = lf[F_Z + (j & 1) * 256 + 64 + l];
    const float z2 = lf[F_Z + (j & 1) * 256 + 128 + l];
    const float z3 = lf[F_Z + (j & 1) * 256 + 192 + l];
    const float b3 = lf[F_B3];
    const float4 rec = lds4(lf + F_REC + 4 * cs);
    float ex = 0.0f, se = 0.0f, gz = 0.0f, sw = 0.0f;
    const float *b1c = nullptr;
    f32x16 tT;
    float4 ga[2], gb[2];
    bf16x8 bq[4][3];  // dW2's B fragments: K-slice, part
    float aw3[4];
    auto xtask = [&](int k) {
      if (k == 0) {
        ex = __expf((((z0 + z1) + z2) + z3) + b3);
      } else if (k == 1) {
        se = seg_sum<64>(ex);
      } else if (k == 2) {
        const int cu = __builtin_amdgcn_readfirstlane(__float_as_int(rec.x));
        const float po = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rec.y)));
        const float Ac = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rec.z)));
        const float p = ex * __builtin_amdgcn_rcpf(se);
        const float pc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), cu));
        if (a.algo == kPPO) {
          // clipped_gradient (rl.h:54-74) through softmax_layer::backward
          const float ratio = pc * __builtin_amdgcn_rcpf(po);
          float ce = a.clip_eps;
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
        sw = half_swap(gz);
        if (q == 0) accB3 += gz;
        b1c = b1row(cs);
      } else if (k == 4) {
        tT = layer1_t(cs, 0, b1c);  // rows 0..31, T layout (f32 MFMA)
      } else if (k >= 5 && k < 13) {
        // relu masks (-> image) of r-tile rt, registers 4 g4 .. 4 g4 + 3;
        // with r-tile 1 the dW3 / db2 sums of both r-tiles (LDS words read
        // in the previous slot)
        const int rt = (k - 5) >> 2, g4 = (k - 5) & 3;
        bf16x4 mk;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          mk[u] = pre_cur[rt][4 * g4 + u] > 0.0f ? (__bf16)1.0f : (__bf16)0.0f;
        if (rt == 1) {
#pragma unroll
          for (int r2 = 0; r2 < 2; ++r2) {
            const float gr = h == r2 ? gz : sw;  // the gradient of row 32 r2 + lr
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const float v = pre_cur[r2][4 * g4 + u];
              accB2[4 * g4 + u] += v > 0.0f ? gr : 0.0f;  // g M (w3 at the write-out)
              aw3[u] = fmaf(gr, relu(v), aw3[u]);
            }
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            accw3[64 * (4 * g4 + u) + l] = aw3[u];
          }
        }
        if (k >= 8 && k < 12) {  // the next slot's words
          const int g4n = k - 8;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            aw3[u] = accw3[64 * (4 * g4n + u) + l];
          }
        }
        *reinterpret_cast<bf16x4 *>(lds + L_MASK +
                                    ((rt == 0 ? sb0 : sb1) ^ (16 * (4 * q + g4)))) = mk;
      } else if (k == 13) {
        // the rows' g of dW2's K-slices 0, 1 (this wave's own copy)
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          ga[sg] = lds4(gw + 16 * sg + 4 * h);
          gb[sg] = lds4(gw + 16 * sg + 8 + 4 * h);
        }
      } else if (k >= 14 && k < 22) {
        // g (x) H1 of K-slices 0, 1: two values per slot
        const int sg = (k - 14) >> 2, e0 = 2 * ((k - 14) & 3);
#pragma unroll
        for (int e = e0; e < e0 + 2; ++e) {
          const float gv = e < 4 ? (&ga[sg].x)[e] : (&gb[sg].x)[e - 4];
          __bf16 p0, p1, p2;
          split3(relu(tT[8 * sg + e]) * gv, p0, p1, p2);
          bq[sg][0][e] = p0;
          bq[sg][1][e] = p1;
          bq[sg][2][e] = p2;
        }
      } else if (k == 26) {
        if (q == 0) stage_store(raw, ns);  // group j+2's rows
      }
    };
    f32x16 pre_nx[2];
    layer2(pre_nx, xtask);
    S4P_STAMP(a, j, q, l, 1);
    partials(pre_nx, (j + 1) & 1);
    S4P_STAMP(a, j, q, l, 2);
    __syncthreads();
    S4P_STAMP(a, j, q, l, 3);

    // ================= Y(j): dH1 and dW2 of group j =====================
    // 32 blocks of three MFMAs: dH1 r-tile 0 (b < 8, K-slice b: dH1 = M W2',
    // T layout), dW2 K-slices 0, 1 (b < 16: K-slice (b - 8) / 4, o-tile
    // (b - 8) % 4: dW2 += M^T (g (x) H1)), dH1 r-tile 1 (b < 24), dW2
    // K-slices 2, 3; operands one block ahead.  Each r-tile's dW1 runs in the
    // dW2 blocks after it, so one dH1 tile and two K-slices of dW2's B
    // fragments are live at a time.
    {
      float sg = 0.0f;
      f32x16 dh, tT1, t1;
      float4 ga1[2], gb1[2];
      const float *b1n = nullptr;
      auto load_ops = [&](int b, bf16x8 &A, bf16x8 &L) {
        if ((b & 8) == 0) {
          const int rt = b >> 4, s = b & 7;
          A = ld_row(lds + L_MASK, rt ? rb1 : rb0, s);
          L = ld_tr(lds + L_WDLO, tq0, tq1, s);
        } else {
          const int s = 2 * (b >> 4) + ((b & 7) >> 2), n = b & 3;
          A = ldtr_at(lds, (tp0 ^ (64 * n)) + 4096 * s, (tp1 ^ (64 * n)) + 4096 * s);
        }
      };
      // dW1 / db1 / item sums of registers 4 g4 .. 4 g4 + 3 of r-tile rt
      // (rows 32 rt + acc_row(j, h)): relu'(layer 1) gates g_r (M W2')[r][i]
      auto dw1 = [&](int rt, int g4, const f32x16 &tl) {
        const float4 x0 = lds4(xim + rt * 32 + 8 * g4 + 4 * h);
        const float4 x1 = lds4(xim + 64 + rt * 32 + 8 * g4 + 4 * h);
        const float4 gg = lds4(gw + rt * 32 + 8 * g4 + 4 * h);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int jj = 4 * g4 + u;
          const float d = tl[jj] > 0.0f ? dh[jj] * (&gg.x)[u] : 0.0f;
          sg += d;
          w0 = fmaf(d, (&x0.x)[u], w0);
          w1 = fmaf(d, (&x1.x)[u], w1);
        }
      };
      // relu, split, stores of layer 1 (group j+2), chunk g4 of r-tile rt
      auto store_l1 = [&](int rt, int g4) {
        bf16x4 ph, pm, pl;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          __bf16 x0, x1, x2;
          split3(relu(t1[4 * g4 + u]), x0, x1, x2);
          ph[u] = x0;
          pm[u] = x1;
          pl[u] = x2;
        }
        const int off = (rt ? sb1 : sb0) ^ (16 * (4 * q + g4));
        *reinterpret_cast<bf16x4 *>(h1i[0] + off) = ph;
        *reinterpret_cast<bf16x4 *>(h1i[1] + off) = pm;
        *reinterpret_cast<bf16x4 *>(h1i[2] + off) = pl;
      };
      auto ytask = [&](int b) {
        if (b == 0) {
          tT1 = layer1_t(cs, 1, b1c);  // rows 32..63, T layout
          b1n = b1row(ns);
        } else if (b == 1) {
          t1 = layer1_c(ns, 0, b1n);  // group j+2, rows 0..31
        } else if (b >= 2 && b < 6) {
          store_l1(0, b - 2);
        } else if (b == 6) {
          tT = layer1_t(cs, 0, b1c);  // rows 0..31 again, for relu' (dW1)
        } else if (b >= 8 && b < 12) {
          dw1(0, b - 8, tT);  // dH1 r-tile 0 completed in block 7
        } else if (b == 13) {
#pragma unroll
          for (int g2 = 0; g2 < 2; ++g2) {
            ga1[g2] = lds4(gw + 32 + 16 * g2 + 4 * h);
            gb1[g2] = lds4(gw + 32 + 16 * g2 + 8 + 4 * h);
          }
        } else if (b >= 14 && b < 22) {
          // g (x) H1 of K-slices 2, 3: two values per slot
          const int g2 = (b - 14) >> 2, e0 = 2 * ((b - 14) & 3);
#pragma unroll
          for (int e = e0; e < e0 + 2; ++e) {
            const float gv = e < 4 ? (&ga1[g2].x)[e] : (&gb1[g2].x)[e - 4];
            __bf16 p0, p1, p2;
            split3(relu(tT1[8 * g2 + e]) * gv, p0, p1, p2);
            bq[2 + g2][0][e] = p0;
            bq[2 + g2][1][e] = p1;
            bq[2 + g2][2][e] = p2;
          }
        } else if (b == 22) {
          t1 = layer1_c(ns, 1, b1n);  // group j+2, rows 32..63
        } else if (b >= 24 && b < 28) {
          store_l1(1, b - 24);
        } else if (b >= 28) {
          dw1(1, b - 28, tT1);  // dH1 r-tile 1 completed in block 23
        }
      };
      bf16x8 A_c, L_c, A_n, L_n;
      load_ops(0, A_c, L_c);
#pragma unroll
      for (int b = 0; b < 32; ++b) {
        if (b + 1 < 32) load_ops(b + 1, A_n, L_n);
        FENCE();
        if ((b & 8) == 0) {
          const int s = b & 7;
          if (s == 0) dh = zero16();
          dh = mfma_bf16(A_c, L_c, dh);
          dh = mfma_bf16(A_c, wd[s][1], dh);
          dh = mfma_bf16(A_c, wd[s][0], dh);
        } else {
          const int s = 2 * (b >> 4) + ((b & 7) >> 2), n = b & 3;
          accW2[n] = mfma_bf16(A_c, bq[s][2], accW2[n]);
          accW2[n] = mfma_bf16(A_c, bq[s][1], accW2[n]);
          accW2[n] = mfma_bf16(A_c, bq[s][0], accW2[n]);
        }
        FENCE();
        ytask(b);
        FENCE();
        A_c = A_n;
        L_c = L_n;
      }
      S4P_STAMP(a, j, q, l, 4);
      if (__builtin_amdgcn_readfirstlane(__float_as_int(lf[F_IT + cs])) != 0)
        sa += sg;
      else
        sb += sg;
      S4P_STAMP(a, j, q, l, 5);
    }
    __syncthreads();
    S4P_STAMP(a, j, q, l, 6);
    S4P_STAMP(a, j, q, l, 7);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) pre_cur[rt] = pre_nx[rt];
  }

  // ---------------------------------------------------- slab write-out ----
  // every entry has exactly one producing lane
  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
  const float *w3g = P + PL.ow3();
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int o = n * 32 + acc_row(j, h);
      slab[PL.oW2() + o * kH + q * 32 + lr] = accW2[n][j] * w3g[o];
    }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    // dW3 / db2 of o = 32 q + acc_row(j, h): sums over the 32 rows of each
    // lane half (valid in lr >= 16)
    const float s3 = half_sum32(accw3[64 * j + l]);
    const float s2 = half_sum32(accB2[j]);
    const int o = q * 32 + acc_row(j, h);
    if (lr == 31) {
      slab[PL.ow3() + o] = s3;
      slab[PL.ob2() + o] = s2 * w3g[o];
    }
  }
  if (q == 0) {
    const float v3 = seg_sum<64>(accB3);
    if (l == 0) slab[PL.ob3()] = v3;
  }
  {
    // dW1 / db1 of feature i = 32 q + lr: the two lane halves hold the two
    // row subsets
    const float tw0 = w0 + __shfl_xor(w0, 32, kWave);
    const float tw1 = w1 + __shfl_xor(w1, 32, kWave);
    const float va = sa + __shfl_xor(sa, 32, kWave);
    const float vb = sb + __shfl_xor(sb, 32, kWave);
    if (h == 0) {
      const int i = q * 32 + lr;
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

}  // namespace s4p

hipError_t launch_policy_train_split4p(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s4p::policy_train_split4p_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s4p::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s4p::policy_train_split4p_kernel, dim3(grid),
                     dim3(s4p::kThreads), s4p::kLds, s, a);
  return hipGetLastError();
}

}  // namespace xh
