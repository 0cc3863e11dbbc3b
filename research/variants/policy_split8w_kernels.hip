// policy_split8w_kernels.hip -- the PPO / actor-critic train epoch of the
// 64-bin 2-D [128,128] policy (BASELINE configs 3 and 4): the math of
// policy_split_kernels.hip (three 128x128 GEMMs on the bf16 matrix cores at
// f32 accuracy, rank-1 backward; see its header and xh_split.h), laid out for
// EIGHT waves, two per SIMD, on v_mfma_f32_16x16x32_bf16.
//
// Why: with one 512-register wave per SIMD (policy_split_kernels.hip) the
// serial VALU phases of a group (operand splits, softmax, loss gradient, dW3
// / db2, dW1) cannot overlap the matrix pipe: 0.37 of the MFMA peak.  Wave w
// here owns the 16-wide feature tile w of every product, so its W2 / W2'
// fragments (all three split parts, 96 registers) and accumulators fit in
// 256 registers, and the two waves of a SIMD issue VALU and MFMA work side
// by side.
//
// Per 64-row group (one env, its 64 bins), wave w, lane l (G = l >> 4, li =
// l & 15); "C layout" = the 16x16 MFMA result: column l & 15, rows 4G + j:
//   layer 1 (VALU fma, bit-identical in both orientations): H1[r][16w..+15]
//     for rows r = li + 16 rt -> relu -> split -> H1 image (3 parts)
//   layer 2: pre[o][r] = W2[o][:] . H1[r][:], o in tile w (A = W2 fragments
//     in registers, B = H1 image rows) -> partial logits -> barrier
//   softmax + loss gradient g (lane = row, every wave) -> dW3 / db2 partial
//     sums, the 0/1 mask image M = relu'(pre), g (x) H1 over the H1 image
//     (layer 2 has consumed it) -> barrier
//   dW2[:, tile w] = M^T (g (x) H1) (both operands by transposed image reads,
//     K = rows); dH1[r][tile w] = M[r][:] . W2'[:, tile w] (A = mask image
//     rows, B = W2' fragments) -> relu' -> dW1 / db1 / item sums (lane =
//     feature); layer 1 of the next group into the other image set -> barrier
//
// LDS images: [64 rows][128 x bf16], 16-byte chunks XOR-swizzled (xh_split.h
// img_off, cdna_hip_programming.md T10 layout (b)).  The row reads of the
// 16x16x32 operand take K-step s's chunk s + 8 (G & 1) + 4 (G >> 1) in lane
// group G (a permutation of the K order shared by both operands of the
// product): with it the ds_read_b128 row reads, the ds_read_b64_tr_b16
// transposed reads and the ds_write_b64 stores are all bank-conflict-free
// (in the natural chunk order 4s + G the row reads are 2-way).
#include <cstdlib>

#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

// Phase stamps (trace build: this file and policy_kernels.hip compiled with
// -DXH_DIAG_TRACE=1, run with XH_PHASE_TRACE=1): lane 0 of every wave of the
// first kTraceBlocks workgroups records the cycle counter at these phase
// boundaries of its first kTraceGroups groups: 0 group start, 1 layer 2 +
// logits done, 2 after barrier 1, 3 softmax / masks / g (x) H1 done, 4 dW2
// done, 5 after its barrier, 6 dH1 / dW1 done, 7 layer 1 (next) done.
#ifndef XH_DIAG_TRACE
#define XH_DIAG_TRACE 0
#endif
#if XH_DIAG_TRACE
#define S8_STAMP(a, gi, w, lane, slot)                                          \
  do {                                                                        \
    if ((a).trace && blockIdx.x < kTraceBlocks && (gi) < kTraceGroups &&      \
        (lane) == 0)                                                          \
      (a).trace[((blockIdx.x * kTraceGroups + (gi)) * 8 + (w)) * kTraceSlots + \
                (slot)] = clock64();                                          \
  } while (0)
#else
#define S8_STAMP(a, gi, w, lane, slot) \
  do {                                 \
  } while (0)
#endif

namespace xh {
namespace s8w {

constexpr int kB = 64, kD = 2, kF0 = 2 * kD, kH = 128;
constexpr int kThreads = 512;
constexpr int kImg = 64 * kImgRow;  // one part image, 16 KB
// LDS carve (bytes): one image set of three parts (H1, then g (x) H1), the
// mask image, the lo parts of W2 ([o][i], 128 rows: layer 2's A operand) and
// of W2' (128 rows in dH1's transposed-read order: dH1's B operand), both
// read per use, then an f32 region
constexpr int L_IMG = 0;
constexpr int L_MASK = 3 * kImg;
constexpr int L_W2LO = 4 * kImg;
constexpr int L_WDLO = 6 * kImg;
constexpr int L_F = 8 * kImg;
constexpr int F_W1T = 0;             // [2 k][128 i]: W1[i][k], the bin columns
constexpr int F_B1F = F_W1T + 2 * kH;  // [2 items][128]: b1 + the item's part
constexpr int F_B2 = F_B1F + 2 * kH;   // [128]
constexpr int F_W3 = F_B2 + kH;        // [128]
constexpr int F_B3 = F_W3 + kH;        // [4]
constexpr int F_Z = F_B3 + 4;          // [64 rows][8 waves] partial logits
constexpr int F_G = F_Z + 64 * 8;      // [64] the rows' loss gradients
constexpr int F_X = F_G + 64;          // [2 parity][2 dims][64 rows] bins / 8
constexpr int F_IT = F_X + 2 * kD * 64;  // [2 parity] the group's item is item_a
constexpr int F_END = F_IT + 4;
constexpr size_t kLds = L_F + sizeof(float) * F_END;
static_assert(kLds <= 160 * 1024, "LDS");
static_assert((L_F + 4 * F_Z) % 16 == 0 && (L_F + 4 * F_X) % 16 == 0 &&
                  (L_F + 4 * F_G) % 16 == 0,
              "16-byte aligned f32 vectors");

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// the six products of two split operands, small terms first (xh_split.h)
__device__ __forceinline__ f32x4 split6(const bf16x8 (&a)[3], const bf16x8 (&b)[3],
                                        f32x4 c) {
  c = mfma16(a[1], b[1], c);
  c = mfma16(a[0], b[2], c);
  c = mfma16(a[2], b[0], c);
  c = mfma16(a[0], b[1], c);
  c = mfma16(a[1], b[0], c);
  c = mfma16(a[0], b[0], c);
  return c;
}
// an operand exact in one bf16 part (the 0/1 mask) times a split one
__device__ __forceinline__ f32x4 split3a(bf16x8 a, const bf16x8 (&b)[3], f32x4 c) {
  c = mfma16(a, b[2], c);
  c = mfma16(a, b[1], c);
  c = mfma16(a, b[0], c);
  return c;
}
__device__ __forceinline__ f32x4 split3b(const bf16x8 (&a)[3], bf16x8 b, f32x4 c) {
  c = mfma16(a[2], b, c);
  c = mfma16(a[1], b, c);
  c = mfma16(a[0], b, c);
  return c;
}

// chunk of K-step s (0..3) read by lane group G (the permuted K order)
__device__ __forceinline__ constexpr int kchunk(int s, int G) {
  return s + 8 * (G & 1) + 4 * (G >> 1);
}
// Row reads: lane (G, li) reads row 16 rt + li, chunk kchunk(s, G) at
// rd_base ^ (16 s) + 4096 rt.
__device__ __forceinline__ int rd_base(int G, int li) {
  return kImgRow * li + 16 * (kchunk(0, G) ^ img_swz(li));
}
__device__ __forceinline__ bf16x8 ld_rd(const char *img, int base, int s, int rt) {
  return *reinterpret_cast<const bf16x8 *>(img + ((base ^ (16 * s)) + 4096 * rt));
}
// Transposed reads of a 16x16x32 operand whose k runs down the image rows:
// lane (G, li) gets column 16 ct + li of rows 32 ks + 8G .. +7 (element j =
// row 32 ks + 8G + j).  Two ds_read_b64_tr_b16: in read t, lane 4q + p of
// the group supplies row 32 ks + 8G + 4t + q, columns 16 ct + 4p .. +3, at
// tr16_base(l, t) ^ (32 ct) + 8192 ks.  EXEC must be full.
__device__ __forceinline__ int tr16_base(int l, int t) {
  const int G = l >> 4, li = l & 15, q = li >> 2, p = li & 3;
  const int row = 8 * G + 4 * t + q;
  return kImgRow * row + 16 * ((p >> 1) ^ img_swz(row)) + 8 * (p & 1);
}
__device__ __forceinline__ bf16x8 ld_tr16(const char *img, int b0, int b1, int ct,
                                          int ks) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4 *)(img + ((b0 ^ (32 * ct)) + 8192 * ks)));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4 *)(img + ((b1 ^ (32 * ct)) + 8192 * ks)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// Stores from the C layout (lane row 16 rt + li, features 16 ft + 4G .. +3):
// 8 bytes at st16_base ^ (32 ft) + 4096 rt.
__device__ __forceinline__ int st16_base(int G, int li) {
  return kImgRow * li + 16 * ((G >> 1) ^ img_swz(li)) + 8 * (G & 1);
}
__device__ __forceinline__ void st_split(char *img, int off, const f32x4 &v) {
  bf16x4 ph, pm, pl;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    __bf16 a, b, c;
    split3(v[u], a, b, c);
    ph[u] = a;
    pm[u] = b;
    pl[u] = c;
  }
  *reinterpret_cast<bf16x4 *>(img + off) = ph;
  *reinterpret_cast<bf16x4 *>(img + kImg + off) = pm;
  *reinterpret_cast<bf16x4 *>(img + 2 * kImg + off) = pl;
}
__device__ __forceinline__ f32x4 lds4v(const float *p) {
  return *reinterpret_cast<const f32x4 *>(p);
}
__device__ __forceinline__ float relu(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}

__global__ __launch_bounds__(kThreads, 2) void policy_train_split8w_kernel(
    PolicyTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH, kH};
  const float *P = a.params;
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int l = tid & 63, G = l >> 4, li = l & 15;

  // ---- prologue: small parameters into LDS, the split W2 / W2' fragments
  // of tile w into registers
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
  // wl: layer 2's A operand, W2[o = 16w + li][i = 8 kchunk(s, G) + j]: the
  // hi / mid parts in registers, the lo part into the W2-lo image (the
  // layout of the row reads, tile w at image rows 16w .. 16w + 15);
  // wd: dH1's B operand, W2'[o = 8 kchunk(s, G) + j][i = 16w + li],
  // W2' = diag(w3) W2 rounded once (xh_split.h)
  bf16x8 wl[4][2], wd[4][2];
  const int rdb0 = rd_base(G, li);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int c8 = 8 * kchunk(s, G);
    const float4 *src =
        reinterpret_cast<const float4 *>(P + PL.oW2() + (16 * w + li) * kH + c8);
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
    *reinterpret_cast<bf16x8 *>(lds + L_W2LO + ((rdb0 ^ (16 * s)) + 4096 * w)) = lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = c8 + j;
      __bf16 x0, x1, x2;
      split3(P[PL.oW2() + o * kH + 16 * w + li] * P[PL.ow3() + o], x0, x1, x2);
      wd[s][0][j] = x0;
      wd[s][1][j] = x1;
      // lo: W2' row o at image row 32 s + 8 G + j (the rows ld_tr16 reads
      // for K-step s in lane group G), column 16 w + li
      const int row = 32 * s + 8 * G + j, col = 16 * w + li;
      *reinterpret_cast<__bf16 *>(lds + L_WDLO + img_off(row, col >> 3) +
                                  2 * (col & 7)) = x2;
    }
  }
  // per-lane LDS address bases
  const int trb00 = tr16_base(l, 0), trb10 = tr16_base(l, 1);
  const int stb0 = st16_base(G, li) ^ (32 * w);
  const int fo0 = 16 * w + 4 * G;  // this lane's 4 features in the C layout
  char *mski = lds + L_MASK;
  const int N = a.b.N, T = a.b.T;
  const int ngroups = T * N;
  __syncthreads();

  // accumulators: dW2 (o-tile ot, i-tile w; C layout o = 16 ot + 4G + j,
  // i = 16w + li); dW3 / db2 partial sums for o = 16w + 4G + j over this
  // lane's rows; dW1 / db1 / item sums of feature i = 16w + li over this
  // lane group's rows; b3 (wave 0, lane = row)
  f32x4 accW2[8];
#pragma unroll
  for (int ot = 0; ot < 8; ++ot)
#pragma unroll
    for (int j = 0; j < 4; ++j) accW2[ot][j] = 0.0f;
  float accW3[4] = {0.0f, 0.0f, 0.0f, 0.0f}, accB2[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float accB3 = 0.0f, w0 = 0.0f, w1 = 0.0f, sa = 0.0f, sb = 0.0f;

  // Group g's rows into the X image of parity p (bins / 8, lane = row) and
  // whether its item is item_a (one wave: 128 bytes of bins, 2 of item)
  auto stage_rows = [&](int g, int p) {
    const int t = g / N, e = g - t * N;
    const size_t ti = (size_t)t * N + e;
    const char2 v = *reinterpret_cast<const char2 *>(a.b.bins + ti * (kB * kD) + l * kD);
    lf[F_X + p * 128 + l] = (float)v.x / (float)kCapacity;
    lf[F_X + p * 128 + 64 + l] = (float)v.y / (float)kCapacity;
    if (l == 0) {
      const char2 iv = *reinterpret_cast<const char2 *>(a.b.items + ti * 4);
      lf[F_IT + p] = (iv.x == a.env.item_a[0] && iv.y == a.env.item_a[1]) ? 1.0f : 0.0f;
    }
  };
  // layer 1 of the group staged in parity p: H1[r][16w + 4G + j] (C layout,
  // rows r = 16 rt + li) -> relu -> split -> image set p
  auto layer1 = [&](int p, int stb, int fi) {
    char *img = lds + L_IMG;
    const bool ia = lf[F_IT + p] != 0.0f;
    const f32x4 wa = lds4v(lf + F_W1T + fi), wb = lds4v(lf + F_W1T + kH + fi);
    const f32x4 bb = lds4v(lf + F_B1F + (ia ? 0 : kH) + fi);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      const float x0 = lf[F_X + p * 128 + 16 * rt + li];
      const float x1 = lf[F_X + p * 128 + 64 + 16 * rt + li];
      f32x4 t;
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = relu(fmaf(x1, wb[j], fmaf(x0, wa[j], bb[j])));
      st_split(img, stb + 4096 * rt, t);
    }
  };
  if ((int)blockIdx.x < ngroups && w == 0) stage_rows(blockIdx.x, 0);
  __syncthreads();
  if ((int)blockIdx.x < ngroups) layer1(0, stb0, fo0);
  __syncthreads();

  int par = 0, gi = 0;
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x, ++gi) {
    S8_STAMP(a, gi, w, l, 0);
    const int gn = g + gridDim.x;
    const bool has_next = gn < ngroups;
    // opaque copies of the per-lane LDS bases and of the f32 vector offset:
    // the compiler recomputes each read address (one v_xor / v_add) in
    // place instead of hoisting dozens of them out of the loop (spills)
    int rdb = rdb0, trb0 = trb00, trb1 = trb10, stb = stb0, fo = fo0;
    asm volatile("" : "+v"(rdb), "+v"(trb0), "+v"(trb1), "+v"(stb), "+v"(fo));
    int c;
    float po, A;
    {
      const int t = g / N, e = g - t * N;
      const size_t ti = (size_t)t * N + e;
      c = a.b.action[ti];
      po = a.b.pold[ti];
      A = a.adv[ti];
    }
    const bool item_cur = lf[F_IT + par] != 0.0f;
    char *img = lds + L_IMG;
    const float *xim = lf + F_X + par * 128;

    // ---- layer 2: pre[rt] = W2[tile w] . H1[rows 16 rt + li]^T + b2
    f32x4 pre[4];
    {
      const f32x4 b2 = lds4v(lf + F_B2 + fo);
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) pre[rt] = b2;
      // explicit one-step operand prefetch: step st = (K-step st / 4,
      // r-tile st % 4); the lo part of W2 (A) once per K-step
      const char *w2lo = lds + L_W2LO + 4096 * w;
      bf16x8 b_c[3], b_n[3], lo_c = ld_rd(w2lo, rdb, 0, 0), lo_n = lo_c;
#pragma unroll
      for (int p = 0; p < 3; ++p) b_c[p] = ld_rd(img + p * kImg, rdb, 0, 0);
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int s = st >> 2, rt = st & 3;
        if (st + 1 < 16) {
#pragma unroll
          for (int p = 0; p < 3; ++p)
            b_n[p] = ld_rd(img + p * kImg, rdb, (st + 1) >> 2, (st + 1) & 3);
          if (rt == 3) lo_n = ld_rd(w2lo, rdb, s + 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 wa[3] = {wl[s][0], wl[s][1], lo_c};
        pre[rt] = split6(wa, b_c, pre[rt]);
#pragma unroll
        for (int p = 0; p < 3; ++p) b_c[p] = b_n[p];
        if (rt == 3) lo_c = lo_n;
      }
      // partial logits of rows 16 rt + li over this wave's 16 features
      const f32x4 w3 = lds4v(lf + F_W3 + fo);
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
        float zp = relu(pre[rt][0]) * w3[0];
        zp = fmaf(relu(pre[rt][1]), w3[1], zp);
        zp = fmaf(relu(pre[rt][2]), w3[2], zp);
        zp = fmaf(relu(pre[rt][3]), w3[3], zp);
        zp += __shfl_xor(zp, 16, kWave);
        zp += __shfl_xor(zp, 32, kWave);
        if (G == 0) lf[F_Z + (16 * rt + li) * 8 + w] = zp;
      }
    }
    S8_STAMP(a, gi, w, l, 1);
    __syncthreads();
    S8_STAMP(a, gi, w, l, 2);

    // ---- softmax -> loss gradient g (lane = row = bin, every wave) ->
    // dW3 / db2 sums, the mask image, g (x) H1 over the H1 image; wave 0
    // stages the next group's rows (read by layer 1 after the barrier)
    if (has_next && w == 0) stage_rows(gn, par ^ 1);
    {
      const f32x4 z0 = lds4v(lf + F_Z + 8 * l), z1 = lds4v(lf + F_Z + 8 * l + 4);
      const float zs = ((z0[0] + z0[1]) + (z0[2] + z0[3])) +
                       ((z1[0] + z1[1]) + (z1[2] + z1[3]));
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
        const float lin = l == cu ? p : 0.0f;
        gz = (lin - p * pc) * gc;
      } else {
        // softmax_gradient_log (rl.h:45-52) through softmax-xent
        gz = p * A;
        if (l == cu) gz -= A;
      }
      if (w == 0) {
        accB3 += gz;
        lf[F_G + l] = gz;
      }
      const f32x4 wa = lds4v(lf + F_W1T + fo), wb = lds4v(lf + F_W1T + kH + fo);
      const f32x4 bb = lds4v(lf + F_B1F + (item_cur ? 0 : kH) + fo);
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
        const float gr = __shfl(gz, 16 * rt + li, kWave);
        bf16x4 mk;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = pre[rt][j];
          const bool on = v > 0.0f;
          const float gm = on ? gr : 0.0f;
          accW3[j] = fmaf(gm, v, accW3[j]);  // g relu(v)
          accB2[j] += gm;                    // g M (w3 at the write-out)
          mk[j] = on ? (__bf16)1.0f : (__bf16)0.0f;
        }
        *reinterpret_cast<bf16x4 *>(mski + stb + 4096 * rt) = mk;
        // g (x) H1: the layer-1 values again (the same two fma: bit-identical)
        const float x0 = xim[16 * rt + li], x1 = xim[64 + 16 * rt + li];
        f32x4 t;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          t[j] = relu(fmaf(x1, wb[j], fmaf(x0, wa[j], bb[j]))) * gr;
        st_split(img, stb + 4096 * rt, t);
      }
    }
    S8_STAMP(a, gi, w, l, 3);
    __syncthreads();

    // ---- dW2[:, tile w] += M^T (g (x) H1): K = the 64 rows (two K-steps);
    // the g (x) H1 fragments of tile w held per K-step, the mask streamed
    {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 bq[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) bq[p] = ld_tr16(img + p * kImg, trb0, trb1, w, ks);
        bf16x8 m_c = ld_tr16(mski, trb0, trb1, 0, ks), m_n = m_c;
#pragma unroll
        for (int ot = 0; ot < 8; ++ot) {
          if (ot + 1 < 8) m_n = ld_tr16(mski, trb0, trb1, ot + 1, ks);
          __builtin_amdgcn_sched_barrier(0);
          accW2[ot] = split3a(m_c, bq, accW2[ot]);
          m_c = m_n;
        }
      }
    }
    S8_STAMP(a, gi, w, l, 4);
    __syncthreads();  // g (x) H1 consumed: the next group's layer 1 may write
    S8_STAMP(a, gi, w, l, 5);
    // ---- dH1[rows 16 rt + 4G + j][i = 16w + li] = M . W2' -> relu' -> dW1 /
    // db1 / item sums, r-tile by r-tile; layer 1 of the next group in the
    // same phase
    {
      float sg = 0.0f;
      const float w1a = lf[F_W1T + 16 * w + li], w1b = lf[F_W1T + kH + 16 * w + li];
      const float b1t = lf[F_B1F + (item_cur ? 0 : kH) + 16 * w + li];
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
        f32x4 dh = {0.0f, 0.0f, 0.0f, 0.0f};
        const char *wdlo = lds + L_WDLO;
        bf16x8 m_c = ld_rd(mski, rdb, 0, rt), m_n = m_c;
        bf16x8 l_c = ld_tr16(wdlo, trb0, trb1, w, 0), l_n = l_c;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if (s + 1 < 4) {
            m_n = ld_rd(mski, rdb, s + 1, rt);
            l_n = ld_tr16(wdlo, trb0, trb1, w, s + 1);
          }
          __builtin_amdgcn_sched_barrier(0);
          const bf16x8 wb3[3] = {wd[s][0], wd[s][1], l_c};
          dh = split3a(m_c, wb3, dh);
          m_c = m_n;
          l_c = l_n;
        }
        const int r0 = 16 * rt + 4 * G;
        const f32x4 x0 = lds4v(xim + r0), x1 = lds4v(xim + 64 + r0);
        const f32x4 gg = lds4v(lf + F_G + r0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float tT = fmaf(x1[j], w1b, fmaf(x0[j], w1a, b1t));
          const float d = tT > 0.0f ? dh[j] * gg[j] : 0.0f;
          sg += d;
          w0 = fmaf(d, x0[j], w0);
          w1 = fmaf(d, x1[j], w1);
        }
      }
      if (item_cur)
        sa += sg;
      else
        sb += sg;
    }
    S8_STAMP(a, gi, w, l, 6);
    if (has_next) layer1(par ^ 1, stb, fo);
    S8_STAMP(a, gi, w, l, 7);
    par ^= 1;
    __syncthreads();  // mask / g (x) H1 consumed; the next images written
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

}  // namespace s8w

hipError_t launch_policy_train_split8w(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s8w::policy_train_split8w_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s8w::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s8w::policy_train_split8w_kernel, dim3(grid),
                     dim3(s8w::kThreads), s8w::kLds, s, a);
  return hipGetLastError();
}

}  // namespace xh
