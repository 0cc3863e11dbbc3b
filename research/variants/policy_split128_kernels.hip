// policy_split128_kernels.hip -- the 128-bin 3-D train epoch (BASELINE
// config 5) with the rank-1 backward: the math and the image layout of
// policy_split_kernels.hip (see its header), one env of 128 rows per group,
// with layer 2 and dH1 on f16 pairs (xh_split.h: power-of-two scales chosen
// per launch from the parameters, three f16 MFMAs per K slice for layer 2
// instead of the bf16 split's six, two for dH1 instead of three; dW2 keeps
// the exact three-part bf16 split of g (x) H1, whose scale is not known
// before the kernel).  A file of its own so that each kernel is compiled
// with the flags measured best for it (Makefile).
#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

namespace xh {
namespace split {

// ============================== 128 bins, 3-D (BASELINE config 5), AC/PPO ==
// The same split GEMMs for one env of 128 rows per group = two 64-row
// half-groups through the 64-row images: layer 1 + layer 2 of half 0 and of
// half 1 (both halves' pre-activations kept in registers), the softmax over
// all 128 bins, the backward of half 1, then of half 0: the backward needs
// no H1 image of its own (dA2 writes g (x) H1 from the layer-1 tile
// recomputed from the bins, bit-identical), so only the X image is
// rewritten.  Layer 1 runs 2 k-steps (D = 3 bin features, the item folded
// into the bias).
namespace s128 {
constexpr int kB = 128, kD = 3, kF0 = 2 * kD, kH1 = 128, kH2 = 128, kS1 = 2;
constexpr int kThreads = 256;
constexpr int kImg = 64 * kImgRow;
// LDS: the row images (H1 as two f16 parts, then g (x) H1 as three bf16
// parts), the bf16 mask image (dW2's transposed reads) and its f16 copy
// (dH1's row reads), then f32
constexpr int L_H1 = 0, L_DA = 3 * kImg, L_MKH = 4 * kImg;
constexpr int L_F = 5 * kImg;
constexpr int F_W1 = 0;                  // [H1][F0]
constexpr int F_B2 = F_W1 + kH1 * kF0;   // [H2] b2 S_W S_H (layer 2's C input)
constexpr int F_W3 = F_B2 + kH2;         // [H2]
constexpr int F_B3 = F_W3 + kH2;         // [4]: b3, the scales S_W, S_D, S_H
constexpr int F_W3S = F_B3 + 4;          // [H2] w3 / (S_W S_H): the logits
constexpr int F_B1F = F_W3S + kH2;       // [2][H1]
constexpr int F_Z = F_B1F + 2 * kH1;     // [4][128] partial logits
constexpr int F_X = F_Z + 4 * 128;       // [3 dims][64 rows] of the current half
constexpr int F_G = F_X + kD * 64;       // [64] the half's row gradients
constexpr int F_SC = F_G + 64;           // [16] the scales' reduction
constexpr int F_END = F_SC + 16;
constexpr int L_B2A = L_F + sizeof(float) * F_END;
constexpr size_t kLds = L_B2A + 4 * 4 * 64 * 16;
static_assert(kLds <= 160 * 1024, "LDS");
}  // namespace s128

__global__ __launch_bounds__(s128::kThreads, 1) void policy_train_split128_kernel(PolicyTrainArgs a) {
  // this shape's constants (shadowing the 64-row kernel's)
  constexpr int kB = s128::kB, kD = s128::kD, kF0 = s128::kF0, kH1 = s128::kH1,
                kH2 = s128::kH2, kS1 = s128::kS1, kThreads = s128::kThreads,
                kImg = s128::kImg;
  constexpr int L_H1 = s128::L_H1, L_DA = s128::L_DA, L_MKH = s128::L_MKH,
                L_F = s128::L_F, L_B2A = s128::L_B2A;
  constexpr int F_W1 = s128::F_W1, F_B2 = s128::F_B2, F_W3 = s128::F_W3,
                F_B3 = s128::F_B3, F_W3S = s128::F_W3S, F_B1F = s128::F_B1F,
                F_Z = s128::F_Z, F_X = s128::F_X, F_G = s128::F_G, F_SC = s128::F_SC;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH1, kH2};
  const float *P = a.params;
  const int tid = threadIdx.x;
  const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, lr = lane & 31, h = lane >> 5;

  // the scales (maxima over the parameters; every workgroup the same): W2,
  // W2' = diag(w3) W2, and H1 <= |W1[i][0..2]| + |b1_item[i]| (|bins / 8| <= 1)
  {
    float mw = 0.0f, md = 0.0f, mh = 0.0f;
    for (int e = tid; e < kH2 * kH1; e += kThreads) {
      const float v = P[PL.oW2() + e];
      mw = fmaxf(mw, fabsf(v));
      md = fmaxf(md, fabsf(v * P[PL.ow3() + (e >> 7)]));
    }
    if (tid < kH1) {
      float ba = P[PL.ob1() + tid], bb = ba, wsum = 0.0f;
#pragma unroll
      for (int d = 0; d < kD; ++d) {
        const float wv = P[PL.oW1() + tid * kF0 + kD + d];
        ba += wv * ((float)a.env.item_a[d] / (float)kCapacity);
        bb += wv * ((float)a.env.item_b[d] / (float)kCapacity);
        wsum += fabsf(P[PL.oW1() + tid * kF0 + d]);
      }
      mh = wsum + fmaxf(fabsf(ba), fabsf(bb));
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      mw = fmaxf(mw, __shfl_xor(mw, o, kWave));
      md = fmaxf(md, __shfl_xor(md, o, kWave));
      mh = fmaxf(mh, __shfl_xor(mh, o, kWave));
    }
    if (lane == 0) {
      lf[F_SC + q] = mw;
      lf[F_SC + 4 + q] = md;
      lf[F_SC + 8 + q] = mh;
    }
    __syncthreads();
    if (tid == 0) {
      float MW = 0.0f, MD = 0.0f, MH = 0.0f;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        MW = fmaxf(MW, lf[F_SC + v]);
        MD = fmaxf(MD, lf[F_SC + 4 + v]);
        MH = fmaxf(MH, lf[F_SC + 8 + v]);
      }
      lf[F_B3 + 1] = f16_scale_for(MW);
      lf[F_B3 + 2] = f16_scale_for(MD);
      lf[F_B3 + 3] = f16_scale_for(MH);
    }
    __syncthreads();
  }
  const float SW = lf[F_B3 + 1], SD = lf[F_B3 + 2], SH = lf[F_B3 + 3];
  const float S2 = SW * SH;  // layer 2's pre-activations are in units of S2
  for (int i = tid; i < kH1 * kF0; i += kThreads) lf[F_W1 + i] = P[PL.oW1() + i];
  for (int i = tid; i < kH2; i += kThreads) {
    lf[F_B2 + i] = P[PL.ob2() + i] * S2;
    lf[F_W3 + i] = P[PL.ow3() + i];
    lf[F_W3S + i] = P[PL.ow3() + i] * (1.0f / S2);
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
  const int rb0_ = row_base(lr, h), rb1_ = row_base(32 + lr, h);
  const int tb0_ = tr_base(lane, 0), tb1_ = tr_base(lane, 1);
  const int tq0_ = tb0_ ^ (64 * q), tq1_ = tb1_ ^ (64 * q);
  const int sb0 = st_base(lr, h), sb1 = st_base(32 + lr, h);
  auto opq = [](int v) {
    asm volatile("" : "+v"(v));
    return v;
  };
  // f16-pair fragments of tile q: wl = layer 2's A operand (rows o = 32 q +
  // lr, k = i = 16 s + 8 h + j), wd = dH1's B operand (k = o = 16 s + 8 h +
  // j, column i = 32 q + lr), straight from the parameters
  f16x8 wl[8][2], wd[8][2];
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * h + j;
      _Float16 x0, x1;
      split2h(P[PL.oW2() + (q * 32 + lr) * kH1 + k] * SW, x0, x1);
      wl[s][0][j] = x0;
      wl[s][1][j] = x1;
      split2h((P[PL.oW2() + k * kH1 + q * 32 + lr] * P[PL.ow3() + k]) * SD, x0, x1);
      wd[s][0][j] = x0;
      wd[s][1][j] = x1;
    }

  char *h1i[3] = {lds + L_H1, lds + L_H1 + kImg, lds + L_H1 + 2 * kImg};
  char *mki = lds + L_DA;   // the 0/1 mask image M (bf16)
  char *mkh = lds + L_MKH;  // the same as f16
  float *xim = lf + F_X;
  const int N = a.b.N, T = a.b.T;
  const int ngroups = T * N;

  f32x16s accW2[4];
  float accW3[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
#pragma unroll
    for (int n = 0; n < 4; ++n) accW2[n][j] = 0.0f;
    accW3[j] = 0.0f;
  }
  float accB3 = 0.0f, wf0 = 0.0f, wf1 = 0.0f, wf2 = 0.0f, sa = 0.0f, sb = 0.0f;
  float4 *b2acc = reinterpret_cast<float4 *>(lds + L_B2A) + q * 4 * 64 + lane;
#pragma unroll
  for (int j4 = 0; j4 < 4; ++j4) b2acc[64 * j4] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);

  // rows hg*64 + rt*32 + lr of the current group: the D bins of a row packed
  // into one register (bytes 0..2, int8), fetched at the group's start
  int bh[2][2];
  auto fetch_half = [&](int g, int hg) {
    const int t = g / N, e = g - t * N;
    const size_t ti = (size_t)t * N + e;
    const int8_t *bp = a.b.bins + ti * (kB * kD);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int8_t *r = bp + (hg * 64 + rt * 32 + lr) * kD;
      bh[hg][rt] = (r[0] & 0xff) | ((r[1] & 0xff) << 8) | ((r[2] & 0xff) << 16);
    }
  };
  auto item_is_a = [&](int g) {
    const int t = g / N, e = g - t * N;
    const size_t ti = (size_t)t * N + e;
    bool ia = true;
#pragma unroll
    for (int d = 0; d < kD; ++d) ia &= a.b.items[ti * 4 + d] == a.env.item_a[d];
    return ia;
  };
  // layer-1 operand of this lane (k = 2 s + h < D) for r-tile rt of half hg
  auto xfeat = [&](int hg, int rt, int s1) {
    const int k = 2 * s1 + h;
    int v = __builtin_amdgcn_sbfe(bh[hg][rt], 8 * (k < kD ? k : 0), 8);
    asm volatile("" : "+v"(v));
    return k < kD ? (float)v / (float)kCapacity : 0.0f;
  };
  auto w1k = [&](int s1) {
    const int k = 2 * s1 + h;
    return k < kD ? lf[F_W1 + (q * 32 + lr) * kF0 + k] : 0.0f;
  };
  // ---- layer 1 of one half: H1 tile q -> relu -> split -> image; X image
  auto layer1 = [&](int hg, bool item_a) {
    const float *b1f = lf + F_B1F + (item_a ? 0 : kH1);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      f32x16s t1 = lds_acc16(b1f, q * 32, h);
#pragma unroll
      for (int s1 = 0; s1 < kS1; ++s1)
        t1 = __builtin_amdgcn_mfma_f32_32x32x2f32(w1k(s1), xfeat(hg, rt, s1), t1, 0, 0, 0);
      if (q == 0) {
        xim[h * 64 + rt * 32 + lr] = xfeat(hg, rt, 0);
        if (h == 0) xim[2 * 64 + rt * 32 + lr] = xfeat(hg, rt, 1);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) t1[j] = relu(t1[j]);
      img_store_h2(h1i[0], h1i[1], rt == 0 ? sb0 : sb1, q * 32, t1, SH);
    }
  };
  // ---- layer 2 of the imaged half (H2 tile q, both r-tiles)
  auto layer2 = [&](f32x16s (&pre)[2]) {
    const int rb0 = opq(rb0_), rb1 = opq(rb1_);
    pre[0] = lds_acc16(lf + F_B2, q * 32, h);
    pre[1] = pre[0];
    f16x8 b_c[2], b_n[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) b_c[p] = __builtin_bit_cast(f16x8, ld_row(h1i[p], rb0, 0));
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int s = st >> 1, rt = st & 1;
      if (st + 1 < 16) {
        const int s1 = (st + 1) >> 1, r1 = (st + 1) & 1;
#pragma unroll
        for (int p = 0; p < 2; ++p)
          b_n[p] = __builtin_bit_cast(f16x8, ld_row(h1i[p], r1 ? rb1 : rb0, s1));
      }
      __builtin_amdgcn_sched_barrier(0);
      // the three f16 products, small terms first
      pre[rt] = mfma_f16(wl[s][1], b_c[0], pre[rt]);
      pre[rt] = mfma_f16(wl[s][0], b_c[1], pre[rt]);
      pre[rt] = mfma_f16(wl[s][0], b_c[0], pre[rt]);
#pragma unroll
      for (int p = 0; p < 2; ++p) b_c[p] = b_n[p];
    }
  };
  auto logits = [&](const f32x16s (&pre)[2], int hg) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      float zp = 0.0f;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 ww = lds4(lf + F_W3S + q * 32 + 8 * g4 + 4 * h);
        zp += relu(pre[rt][4 * g4 + 0]) * ww.x;
        zp += relu(pre[rt][4 * g4 + 1]) * ww.y;
        zp += relu(pre[rt][4 * g4 + 2]) * ww.z;
        zp += relu(pre[rt][4 * g4 + 3]) * ww.w;
      }
      zp += half_swap(zp);
      if (lane < 32) lf[F_Z + q * 128 + hg * 64 + rt * 32 + lr] = zp;
    }
  };
  // ---- dA2 of one half (row gradients gz: lane = row of the half): dW3,
  // db2, and the backward GEMMs' operands (the 64-row kernel's rank-1 form):
  // the 0/1 relu'(A2) image and g (x) H1 over the H1 image of half hg
  auto dA2 = [&](const f32x16s (&pre)[2], float gz, int hg, bool item_a) {
    const float sw = half_swap(gz);
    float b2[16];
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
    const float *b1f = lf + F_B1F + (item_a ? 0 : kH1);
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
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<u32x2 *>(mkh + (sbb ^ (16 * (4 * q + g4)))) =
            __builtin_bit_cast(u32x2, mk) & 0x3C003C00u;
      }
      f32x16s t1 = lds_acc16(b1f, q * 32, h);
#pragma unroll
      for (int s1 = 0; s1 < kS1; ++s1)
        t1 = __builtin_amdgcn_mfma_f32_32x32x2f32(w1k(s1), xfeat(hg, rt, s1), t1, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 16; ++j) t1[j] = relu(t1[j]) * gr;
      img_store_split_b(h1i[0], h1i[1], h1i[2], sbb, q * 32, t1);
    }
  };
  // ---- dW2 tiles (q, n) / w3 over the imaged half's 64 rows: M^T (g (x) H1)
  // (the 64-row kernel's (n, q) tiling measured 0.8% slower here)
  auto dW2 = [&]() {
    const int tb0 = opq(tb0_), tb1 = opq(tb1_), tq0 = opq(tq0_), tq1 = opq(tq1_);
    bf16x8 m_c = ld_tr(mki, tq0, tq1, 0), m_n = m_c, b_c[3], b_n[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) b_c[p] = ld_tr(h1i[p], tb0, tb1, 0);
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int n = st & 3;
      if (st + 1 < 16) {
        const int s1 = (st + 1) >> 2, n1 = (st + 1) & 3;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          b_n[p] = ld_tr(h1i[p], tb0 ^ (64 * n1), tb1 ^ (64 * n1), s1);
        if (n1 == 0) m_n = ld_tr(mki, tq0, tq1, s1);
      }
      __builtin_amdgcn_sched_barrier(0);
      accW2[n] = mfma_split3(m_c, b_c, accW2[n]);
#pragma unroll
      for (int p = 0; p < 3; ++p) b_c[p] = b_n[p];
      if (n == 3) m_c = m_n;
    }
  };
  // ---- dH1 tile q of the half (transposed) -> relu' -> dW1 / db1 / items
  auto dH1 = [&](bool item_a) {
    const int rb0 = opq(rb0_), rb1 = opq(rb1_);
    const float *b1f = lf + F_B1F + (item_a ? 0 : kH1);
    const float b1T = b1f[q * 32 + lr];
    float sg = 0.0f;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      f32x16s dh;
#pragma unroll
      for (int j = 0; j < 16; ++j) dh[j] = 0.0f;
      const int rb = rt == 0 ? rb0 : rb1;
      f16x8 m_c = __builtin_bit_cast(f16x8, ld_row(mkh, rb, 0)), m_n = m_c;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        if (s + 1 < 8) m_n = __builtin_bit_cast(f16x8, ld_row(mkh, rb, s + 1));
        __builtin_amdgcn_sched_barrier(0);
        // S_D dH1 = M (S_D W2'): the mask is exact in f16
        dh = mfma_f16(m_c, wd[s][1], dh);
        dh = mfma_f16(m_c, wd[s][0], dh);
        m_c = m_n;
      }
      // the transposed layer-1 tile (the same two-step chain as layer1())
      f32x16s tT;
#pragma unroll
      for (int j = 0; j < 16; ++j) tT[j] = b1T;
#pragma unroll
      for (int s1 = 0; s1 < kS1; ++s1) {
        const int k = 2 * s1 + h;
        const float xk = k < kD ? xim[k * 64 + rt * 32 + lr] : 0.0f;
        tT = __builtin_amdgcn_mfma_f32_32x32x2f32(xk, w1k(s1), tT, 0, 0, 0);
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 x0 = lds4(xim + rt * 32 + 8 * g4 + 4 * h);
        const float4 x1 = lds4(xim + 64 + rt * 32 + 8 * g4 + 4 * h);
        const float4 x2 = lds4(xim + 128 + rt * 32 + 8 * g4 + 4 * h);
        const float xa[4] = {x0.x, x0.y, x0.z, x0.w};
        const float xc[4] = {x1.x, x1.y, x1.z, x1.w};
        const float xe[4] = {x2.x, x2.y, x2.z, x2.w};
        // dH1 = g_r (M W2')[r][i]: registers are rows rt*32 + acc_row(j, h)
        const float4 gg = lds4(lf + F_G + rt * 32 + 8 * g4 + 4 * h);
        const float gv[4] = {gg.x, gg.y, gg.z, gg.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = 4 * g4 + u;
          const float d = tT[j] > 0.0f ? dh[j] * gv[u] : 0.0f;
          sg += d;
          wf0 = fmaf(d, xa[u], wf0);
          wf1 = fmaf(d, xc[u], wf1);
          wf2 = fmaf(d, xe[u], wf2);
        }
      }
    }
    if (item_a)
      sa += sg;
    else
      sb += sg;
  };

  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    fetch_half(g, 0);
    fetch_half(g, 1);
    const bool item_a = item_is_a(g);
    int c;
    float po, A;
    {
      const int t = g / N, e = g - t * N;
      const size_t ti = (size_t)t * N + e;
      c = a.b.action[ti];
      po = a.b.pold[ti];
      A = a.adv[ti];
    }

    // ---- forward: half 0 (logits only), half 1 (pre kept)
    f32x16s pre[2], pre0[2];
#pragma unroll 1
    for (int hg = 0; hg < 2; ++hg) {
      layer1(hg, item_a);
      __syncthreads();
      layer2(pre);
      logits(pre, hg);
      if (hg == 0) {
        pre0[0] = pre[0];
        pre0[1] = pre[1];
      }
      __syncthreads();
    }

    // ---- softmax over the 128 bins (lane holds bins lane, 64 + lane)
    float gz0, gz1;
    {
      float z[2], ex[2];
      float se = 0.0f;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int r = k * 64 + lane;
        z[k] = (((lf[F_Z + r] + lf[F_Z + 128 + r]) + lf[F_Z + 256 + r]) +
                lf[F_Z + 384 + r]) + lf[F_B3];
        ex[k] = __expf(z[k]);
        se += ex[k];
      }
      se = seg_sum<64>(se);
      const float rse = __builtin_amdgcn_rcpf(se);
      const float p0 = ex[0] * rse, p1 = ex[1] * rse;
      const int cu = __builtin_amdgcn_readfirstlane(c);
      const float pcv = cu < 64 ? p0 : p1;
      const float pc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pcv), cu & 63));
      float g2[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const float pk = k == 0 ? p0 : p1;
        const int bin = k * 64 + lane;
        float gz;
        if (a.algo == kPPO) {
          const float ratio = pc * __builtin_amdgcn_rcpf(po);
          float clipped = ratio;
          if (ratio > 1.0f + a.clip_eps)
            clipped = 1.0f + a.clip_eps;
          else if (ratio < 1.0f - a.clip_eps)
            clipped = 1.0f - a.clip_eps;
          const float ig = fminf(clipped * A, ratio * A) * -1.0f;
          const float gc = ig * __builtin_amdgcn_rcpf(pc);
          const float lin = bin == cu ? pk : 0.0f;
          gz = (lin - pk * pc) * gc;
        } else {
          gz = pk * A;
          if (bin == cu) gz -= A;
        }
        g2[k] = gz;
        if (q == 0) accB3 += gz;
      }
      gz0 = g2[0];
      gz1 = g2[1];
    }

    // ---- backward of half 1 (its H1 image and pre-activations are live),
    // then of half 0 after its layer 1 and layer 2 again
#pragma unroll 1
    for (int hb = 0; hb < 2; ++hb) {
      if (hb == 1) {
        // half 0's pre-activations were kept; dA2 rebuilds its g (x) H1
        // image from the bins, dH1 reads its X image
        pre[0] = pre0[0];
        pre[1] = pre0[1];
        if (q == 0) {
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) {
            xim[h * 64 + rt * 32 + lr] = xfeat(0, rt, 0);
            if (h == 0) xim[2 * 64 + rt * 32 + lr] = xfeat(0, rt, 1);
          }
        }
      }
      dA2(pre, hb == 0 ? gz1 : gz0, hb == 0 ? 1 : 0, item_a);
      __syncthreads();
      dW2();
      __syncthreads();
      dH1(item_a);
      __syncthreads();
    }
  }

  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int j = 0; j < 16; ++j)
      slab[PL.oW2() + (q * 32 + acc_row(j, h)) * kH1 + n * 32 + lr] =
          accW2[n][j] * lf[F_W3 + q * 32 + acc_row(j, h)];
  if (q == 0) {
    float v3 = accB3;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v3 += __shfl_xor(v3, o, kWave);
    if (lane == 0) slab[PL.ob3()] = v3;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float s2 = half_sum32(b2acc[64 * (j >> 2)][j & 3]);
    const float s3 = half_sum32(accW3[j]);
    if (lr == 31) {
      slab[PL.ob2() + q * 32 + acc_row(j, h)] = s2 * lf[F_W3 + q * 32 + acc_row(j, h)];
      slab[PL.ow3() + q * 32 + acc_row(j, h)] = s3 * (1.0f / S2);
    }
  }
  {
    // dH1 was in units of S_D
    const float t0 = (wf0 + __shfl_xor(wf0, 32, kWave)) * (1.0f / SD);
    const float t1 = (wf1 + __shfl_xor(wf1, 32, kWave)) * (1.0f / SD);
    const float t2 = (wf2 + __shfl_xor(wf2, 32, kWave)) * (1.0f / SD);
    const float va = (sa + __shfl_xor(sa, 32, kWave)) * (1.0f / SD);
    const float vb = (sb + __shfl_xor(sb, 32, kWave)) * (1.0f / SD);
    if (h == 0) {
      const int i = q * 32 + lr;
      slab[PL.oW1() + i * kF0 + 0] = t0;
      slab[PL.oW1() + i * kF0 + 1] = t1;
      slab[PL.oW1() + i * kF0 + 2] = t2;
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

hipError_t launch_policy_train_split128(const PolicyTrainArgs &a, int grid,
                                        hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)split::policy_train_split128_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)split::s128::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(split::policy_train_split128_kernel, dim3(grid),
                     dim3(split::s128::kThreads), split::s128::kLds, s, a);
  return hipGetLastError();
}

}  // namespace xh
