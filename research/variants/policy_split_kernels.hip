// policy_split_kernels.hip -- the PPO / actor-critic train epoch of the
// 64-bin 2-D [128,128] policy (BASELINE configs 3 and 4) with its three
// 128x128 GEMMs on the bf16 matrix cores at f32 accuracy (xh_split.h: each
// f32 operand split exactly into three bf16 parts; six bf16 MFMAs per K = 16
// slice in place of eight f32 ones).  Round 2's config-3 kernel, superseded
// by policy_split8wh_kernels.hip: built only into the variant library
// (`make variants`, XH_TRAIN_KERNEL=split4w) for A/B runs; compiled with the
// VGPR form of the MFMAs (Makefile).
//
// Same math as policy_train8_kernel (policy_kernels.hip): per 64-row group
// (one env, its 64 bins) layer 1 (conv1d_1 F0 -> 128, item folded into the
// bias) -> relu -> layer 2 (128 -> 128) -> relu -> layer 3 -> softmax (no
// max shift, nn.h:382-392) -> clipped-surrogate (rl.h:54-74) or softmax-log
// (rl.h:45-52) gradient -> softmax Jacobian backward (nn.h:393-417) -> dA2 ->
// dW2 = dA2^T H1, dH1 = dA2 W2 -> dA1 -> dW1 / db1 (nn.h:149-186).  One
// gradient slab per workgroup, every entry written by exactly one wave.
//
// Rank-1 backward: layer 3 has one output per row, so
//     dA2[r][o] = g_r w3_o M[r][o],   M = relu'(A2) in {0, 1},
// and the two backward GEMMs run on the exact 0/1 image M (one bf16 part):
//     dW2 = diag(w3) M^T (g (x) H1),   dH1 = diag(g) M W2',  W2' = diag(w3) W2
// (g (x) H1 and W2' rounded once, split into three parts): three bf16 MFMAs
// per K = 16 slice (xh_split.h mfma_split3) instead of six; w3 is applied to
// dW2's tile at the write-out and g to dH1's rows in the dW1 sums.
//
// 4 waves (one per SIMD, 512 registers each), one workgroup per CU; wave q
// owns 32-wide tile q of every product:
//   layer 1: H1 tile q of both 32-row r-tiles -> split -> H1 image
//   layer 2: H2 tile q (W2 row fragments in registers, H1 image rows),
//            partial logits -> softmax + loss gradient (every wave, all rows)
//   dW3 / db2 partial sums; M tile q -> the mask image, g (x) H1 tile q ->
//            the H1 image (layer 2 has consumed it)
//   dW2 tiles (0..3, q) over the 64 rows (both operands by transposed image
//            reads; i-tile q of g (x) H1 held per K-half, the mask streamed)
//   dH1 tile q = M . W2'[:, tile q] (W2'^T fragments in registers, mask
//            image rows) -> relu' -> dW1 / db1 / item columns
// The W2 hi / mid fragments of layer 2 and the W2' ones of dH1 (8 K-slices
// x 2 parts each, 128 registers) are loaded once per launch from split
// images that the prologue builds in the LDS the row images use afterwards;
// the lo parts stay in LDS images (W2' lo in the mask region's spare parts).
#include <cstdlib>
#include <cstring>

#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

// Variant knobs (make variant VSRC=policy_split_kernels VFLAGS=...):
//   XH_SV_ABL  diagnostic timing builds only: bit0 skip the dW1 VALU, bit1
//              skip dW2, bit2 skip dH1, bit3 skip the layer-2 MFMAs (results
//              are wrong by design; the product build has 0)
#ifndef XH_SV_ABL
#define XH_SV_ABL 0
#endif

namespace xh {
namespace split {

constexpr int kB = 64, kD = 2, kF0 = 2 * kD, kH1 = 128, kH2 = 128;
constexpr int kThreads = 256;
// LDS carve (bytes): three part images of the 64-row H1 tile, the mask
// image + W2' lo ([row][feature], 256-byte swizzled rows), W2's lo-part
// image, then an f32 region.  The prologue's W2 hi / mid images (2 x 128 rows) alias the row
// images; their fragments live in registers, the lo part's are read per use.
constexpr int kImg = 64 * kImgRow;
constexpr int L_H1 = 0, L_DA = 3 * kImg, L_W2 = 0;
constexpr int L_W2LO = 6 * kImg;
constexpr int L_F = L_W2LO + 128 * kImgRow;
constexpr int F_W1 = 0;                    // [H1][F0]
constexpr int F_B2 = F_W1 + kH1 * kF0;     // [H2]
constexpr int F_W3 = F_B2 + kH2;           // [H2]
constexpr int F_B3 = F_W3 + kH2;           // [4]
constexpr int F_B1F = F_B3 + 4;            // [2][H1]: b1 + item part, per item
constexpr int F_Z = F_B1F + 2 * kH1;       // [4][64] partial logits
constexpr int F_X = F_Z + 4 * 64;          // [2 parity][2 dims][64 rows] bins/8
constexpr int F_G = F_X + 2 * kD * 64;     // [64] the rows' loss gradients
constexpr int F_END = F_G + 64;
// db2 / w3 partial sums per lane (g M summed over this lane's rows): [wave q][4]
// [64 lanes] float4, read-modify-written once per group
constexpr int L_B2A = L_F + sizeof(float) * F_END;
constexpr size_t kLds = L_B2A + 4 * 4 * 64 * 16;
static_assert(2 * 128 * kImgRow <= L_W2LO, "W2 images fit the row images");
static_assert(kLds <= 160 * 1024, "LDS");

__global__ __launch_bounds__(kThreads, 1) void policy_train_split_kernel(PolicyTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH1, kH2};
  const float *P = a.params;
  const int tid = threadIdx.x;
  // the wave index through readfirstlane: wave-uniform for the compiler
  const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, lr = lane & 31, h = lane >> 5;

  // ---- prologue: split W2 images [o][i], the small parameters, and the
  // layer-1 biases with either table item's contribution folded in
  for (int e = tid; e < kH2 * kH1; e += kThreads) {
    const int o = e >> 7, i = e & 127;
    __bf16 x0, x1, x2;
    split3(P[PL.oW2() + e], x0, x1, x2);
    const int off = img_off(o, i >> 3) + 2 * (i & 7);
    *reinterpret_cast<__bf16 *>(lds + L_W2 + off) = x0;
    *reinterpret_cast<__bf16 *>(lds + L_W2 + 128 * kImgRow + off) = x1;
    *reinterpret_cast<__bf16 *>(lds + L_W2LO + off) = x2;
  }
  for (int i = tid; i < kH1 * kF0; i += kThreads) lf[F_W1 + i] = P[PL.oW1() + i];
  for (int i = tid; i < kH2; i += kThreads) {
    lf[F_B2 + i] = P[PL.ob2() + i];
    lf[F_W3 + i] = P[PL.ow3() + i];
  }
  if (tid == 0) lf[F_B3] = P[PL.ob3()];
  for (int i = tid; i < 2 * kH1; i += kThreads) {
    const int e = i / kH1, u = i - e * kH1;
    const int *it = e == 0 ? a.env.item_a : a.env.item_b;
    float v = P[PL.ob1() + u];
#pragma unroll
    for (int d = 0; d < kD; ++d)
      v += P[PL.oW1() + u * kF0 + kD + d] * ((float)it[d] / (float)kCapacity);
    lf[F_B1F + i] = v;
  }
  __syncthreads();
  // W2 fragments of tile q: wl = the A operand of layer 2 (rows o, k = i),
  // wd = the A operand of dH1 (rows i, k = o: transposed reads)
  // per-lane LDS address bases (xh_split.h): rows rt*32 + lr of the row
  // images, row q*32 + lr of W2's, the transposed-read bases of column tile
  // q, stores of rows rt*32 + lr
  const int rb0_ = row_base(lr, h), rb1_ = row_base(32 + lr, h);
  const int rbw_ = row_base(q * 32 + lr, h);
  const int tb0_ = tr_base(lane, 0), tb1_ = tr_base(lane, 1);
  const int tq0_ = tb0_ ^ (64 * q), tq1_ = tb1_ ^ (64 * q);
  const int sb0 = st_base(lr, h), sb1 = st_base(32 + lr, h);
  bf16x8 wl[8][2], wd[8][2];
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const char *img = lds + L_W2 + p * 128 * kImgRow;
      wl[s][p] = ld_row(img, rbw_, s);
    }
  __syncthreads();  // the W2 images' LDS becomes the row images
  // W2' = diag(w3) W2 (rounded once), split: hi / mid images for dH1's
  // fragments (the same LDS again), its lo image in the dA2 region's parts
  // 1-2 (the mask needs one part)
  for (int e = tid; e < kH2 * kH1; e += kThreads) {
    const int o = e >> 7, i = e & 127;
    __bf16 x0, x1, x2;
    split3(P[PL.oW2() + e] * P[PL.ow3() + o], x0, x1, x2);
    const int off = img_off(o, i >> 3) + 2 * (i & 7);
    *reinterpret_cast<__bf16 *>(lds + L_W2 + off) = x0;
    *reinterpret_cast<__bf16 *>(lds + L_W2 + 128 * kImgRow + off) = x1;
    *reinterpret_cast<__bf16 *>(lds + L_DA + kImg + off) = x2;
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int p = 0; p < 2; ++p)
      wd[s][p] = ld_tr(lds + L_W2 + p * 128 * kImgRow, tq0_, tq1_, s);
  __syncthreads();

  char *h1i[3] = {lds + L_H1, lds + L_H1 + kImg, lds + L_H1 + 2 * kImg};
  char *mki = lds + L_DA;  // the 0/1 mask image M
  const char *w2lo = lds + L_W2LO;
  // the lo part of dH1's operand W2' = diag(w3) W2
  const char *w2dlo = lds + L_DA + kImg;
  const int N = a.b.N, T = a.b.T;
  const int ngroups = T * N;

  // dW2 tiles (n, q); dW3 partial sums (lane = row layout); dW1 of feature
  // i = q*32 + lr over this lane half's rows: bin columns w0 / w1 and the dA1
  // sums over rows holding item_a / item_b (the item columns and db1)
  f32x16s accW2[4];
  float accW3[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
#pragma unroll
    for (int n = 0; n < 4; ++n) accW2[n][j] = 0.0f;
    accW3[j] = 0.0f;
  }
  float accB3 = 0.0f, w0 = 0.0f, w1 = 0.0f, sa = 0.0f, sb = 0.0f;
  float4 *b2acc = reinterpret_cast<float4 *>(lds + L_B2A) + q * 4 * 64 + lane;
#pragma unroll
  for (int j4 = 0; j4 < 4; ++j4) b2acc[64 * j4] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  int par = 0;  // group parity: the X image double buffer

  // Software pipeline over the groups of this workgroup: iteration g runs
  // layer 2 .. dW2 of group g, then dH1 / dW1 of group g together with layer
  // 1 of group g+1 (independent work in one phase, which the scheduler
  // interleaves: the next H1 image is written while dH1's MFMAs run; the H1
  // image is free once dW2 has read it).  Per group: the rows' bins and item
  // (layer 1), the env's record (action, p_old, advantage: the loss).
  int bv[2][kD], iv[kD];
  bool item_a = true;  // of the group whose layer 1 ran last
  auto fetch_rows = [&](int g) {
    const int t = g / N, e = g - t * N;
    const size_t ti = (size_t)t * N + e;
    const int8_t *bp = a.b.bins + ti * (kB * kD);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int d = 0; d < kD; ++d) bv[rt][d] = bp[(rt * 32 + lr) * kD + d];
#pragma unroll
    for (int d = 0; d < kD; ++d) iv[d] = a.b.items[ti * 4 + d];
  };
  // ---- layer 1 of the fetched group: H1 tile q of both r-tiles -> relu ->
  // split -> image; the X image (bins / 8) of parity p.  The transposed tile
  // (lane = feature i, registers = rows) comes from the same two products
  // in the same order (bit-identical values): its relu mask gates dA1 in
  // dH1's transposed layout.
  auto layer1 = [&](int p) {
    item_a = true;
#pragma unroll
    for (int d = 0; d < kD; ++d) item_a &= iv[d] == a.env.item_a[d];
    float *xim = lf + F_X + p * (kD * 64);
    const float *b1f = lf + F_B1F + (item_a ? 0 : kH1);
    const float wa = lf[F_W1 + (q * 32 + lr) * kF0 + h];  // W1[i][k = h]
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      f32x16s t1 = lds_acc16(b1f, q * 32, h);
      // this lane's feature (k = h) as a register select, not an indexed
      // (scratch) array read
      int xv0 = bv[rt][0], xv1 = bv[rt][1];
      asm volatile("" : "+v"(xv0), "+v"(xv1));
      const float xb = (float)(h == 0 ? xv0 : xv1) / (float)kCapacity;
      if (q == 0) xim[h * 64 + rt * 32 + lr] = xb;
      t1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wa, xb, t1, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        t1[j] = relu(t1[j]);
      }
      img_store_split_b(h1i[0], h1i[1], h1i[2], rt == 0 ? sb0 : sb1, q * 32, t1);
    }
  };
  if ((int)blockIdx.x < ngroups) {
    fetch_rows(blockIdx.x);
    layer1(0);
  }
  __syncthreads();

  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int gn = g + gridDim.x;
    const bool has_next = gn < ngroups;
    int c;
    float po, A;
    {
      const int t = g / N, e = g - t * N;
      const size_t ti = (size_t)t * N + e;
      c = a.b.action[ti];
      po = a.b.pold[ti];
      A = a.adv[ti];
    }
    if (has_next) fetch_rows(gn);  // consumed by layer1() at the end
    const bool item_a_cur = item_a;
    const float *xim = lf + F_X + par * (kD * 64);

    // ---- layer 2 (H2 tile q, both r-tiles) + partial logits
    f32x16s pre[2];
    {
      const int rb0 = rb0_, rb1 = rb1_, rbw = rbw_;
      pre[0] = lds_acc16(lf + F_B2, q * 32, h);
      pre[1] = pre[0];
      // explicit one-step prefetch: step st = (K-slice st/2, r-tile st%2);
      // its operands are loaded while step st-1's MFMAs run
      bf16x8 lo_c = ld_row(w2lo, rbw, 0), lo_n = lo_c, b_c[3], b_n[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) b_c[p] = ld_row(h1i[p], rb0, 0);
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int s = st >> 1, rt = st & 1;
        if (st + 1 < 16) {
          const int s1 = (st + 1) >> 1, r1 = (st + 1) & 1;
#pragma unroll
          for (int p = 0; p < 3; ++p) b_n[p] = ld_row(h1i[p], r1 ? rb1 : rb0, s1);
          if (r1 == 0) lo_n = ld_row(w2lo, rbw, s1);
        }
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 wa[3] = {wl[s][0], wl[s][1], lo_c};
        if (!(XH_SV_ABL & 8)) pre[rt] = mfma_split6(wa, b_c, pre[rt]);
#pragma unroll
        for (int p = 0; p < 3; ++p) b_c[p] = b_n[p];
        if (rt == 1) lo_c = lo_n;
      }
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        float zp = 0.0f;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 ww = lds4(lf + F_W3 + q * 32 + 8 * g4 + 4 * h);
          zp += relu(pre[rt][4 * g4 + 0]) * ww.x;
          zp += relu(pre[rt][4 * g4 + 1]) * ww.y;
          zp += relu(pre[rt][4 * g4 + 2]) * ww.z;
          zp += relu(pre[rt][4 * g4 + 3]) * ww.w;
        }
        zp += half_swap(zp);
        if (lane < 32) lf[F_Z + q * 64 + rt * 32 + lr] = zp;
      }
    }
    __syncthreads();

    // ---- softmax -> loss gradient (lane = row = bin) -> dA2 tile q -> image
    {
      const float zs = ((lf[F_Z + lane] + lf[F_Z + 64 + lane]) + lf[F_Z + 128 + lane]) +
                       lf[F_Z + 192 + lane];
      const float z = zs + lf[F_B3];
      const float ex = __expf(z);
      const float se = seg_sum<64>(ex);
      const float p = ex * __builtin_amdgcn_rcpf(se);
      const int cu = __builtin_amdgcn_readfirstlane(c);
      const float pc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), cu));
      float gz;
      if (a.algo == kPPO) {
        // clipped_gradient (rl.h:54-74) through softmax_layer::backward
        const float ratio = pc * __builtin_amdgcn_rcpf(po);
        float clipped = ratio;
        if (ratio > 1.0f + a.clip_eps)
          clipped = 1.0f + a.clip_eps;
        else if (ratio < 1.0f - a.clip_eps)
          clipped = 1.0f - a.clip_eps;
        const float ig = fminf(clipped * A, ratio * A) * -1.0f;
        const float gc = ig * __builtin_amdgcn_rcpf(pc);
        const float lin = lane == cu ? p : 0.0f;
        gz = (lin - p * pc) * gc;
      } else {
        // softmax_gradient_log (rl.h:45-52) through softmax-xent
        gz = p * A;
        if (lane == cu) gz -= A;
      }
      if (q == 0) accB3 += gz;
      const float sw = half_swap(gz);
      float b2[16];  // db2 partial sums over this lane's rows (LDS between groups)
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const float4 v = b2acc[64 * j4];
        b2[4 * j4 + 0] = v.x;
        b2[4 * j4 + 1] = v.y;
        b2[4 * j4 + 2] = v.z;
        b2[4 * j4 + 3] = v.w;
      }
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        // row rt*32 + lr's gradient: own lane in half rt, else lane ^ 32
        const float gr = h == rt ? gz : sw;
        // dW3 partial sums; db2 / w3 = sum_r g_r M[r][o] (w3 applied at the
        // write-out, as dW2's)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const float v = pre[rt][j];
          accW3[j] += gr * relu(v);
          b2[j] += v > 0.0f ? gr : 0.0f;
        }
      }
      if (q == 0) lf[F_G + lane] = gz;
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4)
        b2acc[64 * j4] = make_float4(b2[4 * j4], b2[4 * j4 + 1], b2[4 * j4 + 2],
                                     b2[4 * j4 + 3]);
      // the backward GEMMs' operands: relu'(A2) as an exact 0/1 image (one
      // bf16 part) and g (x) H1 (the layer-1 tile again, bit-identical to
      // layer1()'s, times the row's gradient: three parts, over the H1 image,
      // which every wave's layer 2 has read before the logits barrier)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const float gr = h == rt ? gz : sw;
        const int sbb = rt == 0 ? sb0 : sb1;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          bf16x4 mk;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            mk[u] = pre[rt][4 * g4 + u] > 0.0f ? (__bf16)1.0f : (__bf16)0.0f;
          *reinterpret_cast<bf16x4 *>(mki + (sbb ^ (16 * (4 * q + g4)))) = mk;
        }
        const float *b1f = lf + F_B1F + (item_a_cur ? 0 : kH1);
        f32x16s t1 = lds_acc16(b1f, q * 32, h);
        t1 = __builtin_amdgcn_mfma_f32_32x32x2f32(
            lf[F_W1 + (q * 32 + lr) * kF0 + h], xim[h * 64 + rt * 32 + lr], t1, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 16; ++j) t1[j] = relu(t1[j]) * gr;
        img_store_split_b(h1i[0], h1i[1], h1i[2], sbb, q * 32, t1);
      }
    }
    __syncthreads();

    // ---- dW2 tiles (n, q) / w3, K = the 64 rows: M^T (g (x) H1).  Wave q's
    // B operand (i-tile q of g (x) H1, three parts) is loaded once per
    // K-half and reused over the four o-tiles of the mask (one part):
    // 28 KB of LDS reads per wave instead of 52
    {
      const int tb0 = tb0_, tb1 = tb1_, tq0 = tq0_, tq1 = tq1_;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        bf16x8 bq[2][3];
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
#pragma unroll
          for (int p = 0; p < 3; ++p) bq[ss][p] = ld_tr(h1i[p], tq0, tq1, 2 * kh + ss);
        bf16x8 m_c = ld_tr(mki, tb0, tb1, 2 * kh), m_n = m_c;
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const int n = st >> 1, ss = st & 1;
          if (st + 1 < 8) {
            const int n1 = (st + 1) >> 1, s1 = (st + 1) & 1;
            m_n = ld_tr(mki, tb0 ^ (64 * n1), tb1 ^ (64 * n1), 2 * kh + s1);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (!(XH_SV_ABL & 2)) accW2[n] = mfma_split3(m_c, bq[ss], accW2[n]);
          m_c = m_n;
        }
      }
    }
    __syncthreads();  // H1 image consumed: the next group's layer 1 may write

    // ---- dH1 tile q, transposed (lane = feature i, registers = rows: the
    // same products with the operands swapped) -> relu' -> dW1 / db1 / item
    // sums (four per-lane accumulators, the rows' bins/8 from the X image);
    // r-tile by r-tile, so r-tile 0's VALU overlaps r-tile 1's MFMAs.  Layer
    // 1 of the next group in the same phase.
    {
      const int rb0 = rb0_, rb1 = rb1_, tq0 = tq0_, tq1 = tq1_;
      float sg = 0.0f;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        f32x16s dh;
#pragma unroll
        for (int j = 0; j < 16; ++j) dh[j] = 0.0f;
        const int rb = rt == 0 ? rb0 : rb1;
        bf16x8 lo_c = ld_tr(w2dlo, tq0, tq1, 0), lo_n = lo_c;
        bf16x8 m_c = ld_row(mki, rb, 0), m_n = m_c;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          if (s + 1 < 8) {
            m_n = ld_row(mki, rb, s + 1);
            lo_n = ld_tr(w2dlo, tq0, tq1, s + 1);
          }
          __builtin_amdgcn_sched_barrier(0);
          const bf16x8 wa[3] = {wd[s][0], wd[s][1], lo_c};
          if (!(XH_SV_ABL & 4)) dh = mfma_split3(m_c, wa, dh);
          m_c = m_n;
          lo_c = lo_n;
        }
        if (XH_SV_ABL & 1) continue;
        // the transposed layer-1 tile again (the same two products as
        // layer1(): bit-identical), for relu' in this layout
        f32x16s tT;
        {
          const float *b1f = lf + F_B1F + (item_a_cur ? 0 : kH1);
          const float b1T = b1f[q * 32 + lr];
          const float wa1 = lf[F_W1 + (q * 32 + lr) * kF0 + h];
          const float xb = xim[h * 64 + rt * 32 + lr];
#pragma unroll
          for (int j = 0; j < 16; ++j) tT[j] = b1T;
          tT = __builtin_amdgcn_mfma_f32_32x32x2f32(xb, wa1, tT, 0, 0, 0);
        }
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          // dH1 = g_r (M W2')[r][i] (registers = rows rt*32 + acc_row(j, h)):
          // g_r is applied through the rows' g, g x0, g x1
          const float4 x0 = lds4(xim + rt * 32 + 8 * g4 + 4 * h);
          const float4 x1 = lds4(xim + 64 + rt * 32 + 8 * g4 + 4 * h);
          const float4 gg = lds4(lf + F_G + rt * 32 + 8 * g4 + 4 * h);
          const float gv[4] = {gg.x, gg.y, gg.z, gg.w};
          const float xa[4] = {x0.x, x0.y, x0.z, x0.w};
          const float xc[4] = {x1.x, x1.y, x1.z, x1.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = 4 * g4 + u;
            const float d = tT[j] > 0.0f ? dh[j] * gv[u] : 0.0f;
            sg += d;
            w0 = fmaf(d, xa[u], w0);
            w1 = fmaf(d, xc[u], w1);
          }
        }
      }
      if (item_a_cur)
        sa += sg;
      else
        sb += sg;
    }
    if (has_next) layer1(par ^ 1);
    par ^= 1;
    __syncthreads();  // dA2 image consumed; the next H1 / X images written
  }

  // ---------------------------------------------------- slab write-out ----
  // every entry has exactly one producing wave / lane
  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int j = 0; j < 16; ++j)
      slab[PL.oW2() + (n * 32 + acc_row(j, h)) * kH1 + q * 32 + lr] =
          accW2[n][j] * lf[F_W3 + n * 32 + acc_row(j, h)];
  {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      // db2: sums over the 32 rows of each lane half (valid in lr >= 16)
      const float s2 = half_sum32(b2acc[64 * (j >> 2)][j & 3]);
      if (lr == 31) slab[PL.ob2() + q * 32 + acc_row(j, h)] = s2 * lf[F_W3 + q * 32 + acc_row(j, h)];
    }
  }
  if (q == 0) {
    float v3 = accB3;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v3 += __shfl_xor(v3, o, kWave);
    if (lane == 0) slab[PL.ob3()] = v3;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    // dW3: sums over the 32 rows of each lane half (valid in lr >= 16)
    const float s3 = half_sum32(accW3[j]);
    if (lr == 31) slab[PL.ow3() + q * 32 + acc_row(j, h)] = s3;
  }
  {
    // dW1 / db1 of feature i: the two lane halves hold the two row subsets
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

}  // namespace split

// The variant library's entry point for this kernel (train_select.cpp,
// XH_TRAIN_KERNEL=split4w; `make variants`).
hipError_t launch_policy_train_split4w(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)split::policy_train_split_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)split::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(split::policy_train_split_kernel, dim3(grid),
                     dim3(split::kThreads), split::kLds, s, a);
  return hipGetLastError();
}

}  // namespace xh
