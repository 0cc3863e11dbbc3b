// value_net_kernels.hip -- the learners' value net (full_layer Fin -> 64 ->
// 32 -> 1, relu between; the value_h1 / value_h2 defaults of
// ppo_training.cc:19-26) for update_value_model and calculate_advantage
// (policy_gradient.h:196-281) as two gfx950 kernels: a persistent forward and
// one fused backward (TD targets, data gradients, all weight gradients).
//
// Layer 0 runs on the bf16 matrix cores with f32 accuracy.  The observation
// features are integers over kCapacity (observation::to_vector,
// bin_packing.h:31-40; bins minus the item for a terminal view): every such
// integer (|v| <= 255) is exact in bf16, and the 1/kCapacity scale moves onto
// the weights exactly (a power of two).  W0 / kCapacity splits exactly into
// three bf16 parts (round-to-nearest hi, mid of the residual, and the last
// residual, which has at most 8 significant bits), so
//   x . W0/8 = x . hi + x . mid + x . lo
// with every product exact and f32 accumulation: the accuracy of the f32
// MFMA at 3/16 of its matrix-core time.  The backward's dW0 = g0^T [x | 1]
// takes the same exact split on the f32 data gradient g0, x exact.  Layers 1
// and 2 (a 64 x 32 and a 32 x 1 matrix) and their gradients stay on the f32
// MFMA / VALU.
//
// Observation layout: the reduced feature vector of dense_kernels.hip's
// ObsRedRows (the B*D bin features, then the D item features once, their B
// copies' weights summed), so layer 0's K = B*D + D.
#include <cstdlib>

#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {
namespace vnet {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int V1 = 64, V2 = 32;  // hidden widths
constexpr int TM = 64;           // rows per tile / chunk

__device__ __forceinline__ f32x16 mfma_bf(const bf16x8 &a, const bf16x8 &b, const f32x16 &c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// D = A(16x4) B(4x16) + C: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15];
// C/D: row 4 (l>>4) + r, column l&15
__device__ __forceinline__ f32x4 mfma16(float a, float b, const f32x4 &c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ unsigned pk(float a, float b) {  // v_cvt_pk_bf16_f32
  return __builtin_bit_cast(unsigned, bf16x2{(__bf16)a, (__bf16)b});
}
// v = hi + mid + lo exactly, each part a bf16 (returned as f32)
__device__ __forceinline__ void split3(float v, float &hi, float &mid, float &lo) {
  hi = (float)(__bf16)v;
  const float r = v - hi;  // exact
  mid = (float)(__bf16)r;
  lo = r - mid;            // exact, and exact in bf16
}
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.0f, 0.0f, 0.0f, 0.0f}; }
__device__ __forceinline__ float sbyte(unsigned w, int b) {
  return (float)(int)(int8_t)(w >> (8 * b));
}

// ---------------------------------------------------------------- W0 prep --
// The item columns of W0 on the reduced observation: isum[n][c] = sum over
// bins of W0[n][b 2D + D + c] (reduce_w0_kernel's sum, here in a fixed tree
// order), one workgroup per (n, c): one round of loads instead of B
// dependent ones per lane.
__global__ __launch_bounds__(256) void w0_item_kernel(const float *W0, int in, int B,
                                                      int D, float *isum) {
  __shared__ float ws[4];
  const int n = blockIdx.x / D, c = blockIdx.x - n * D;
  const float *col = W0 + (size_t)n * in + D + c;
  float v = 0.0f;
  for (int b = threadIdx.x; b < B; b += 256) v += col[b * 2 * D];
  v = seg_sum<64>(v);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) isum[blockIdx.x] = (ws[0] + ws[1]) + (ws[2] + ws[3]);
}
// W0 / kCapacity on the reduced observation, three exact bf16 parts, in the
// forward's B-fragment order: frag[(p * 2 + cb) * nkb + kb][lane] = part p
// of [n = 32 cb + (lane & 31)][k = 16 kb + 8 (lane >> 5) + j], j = 0..7
// (k >= K: zero).
// isum[n][c] for B <= 64 inside one lane, in w0_item_kernel's order: its
// seg_sum<64> is the balanced pairwise tree over the 64 lanes (zeros past B),
// then + 0 for the empty waves, so the bits are the same
__device__ __forceinline__ float item_sum_tree(const float *col, int D, int B) {
  float r[4];
#pragma unroll
  for (int row = 0; row < 4; ++row) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int b = 16 * row + i;
      v[i] = b < B ? col[b * 2 * D] : 0.0f;
    }
#pragma unroll
    for (int w = 1; w < 16; w <<= 1)
#pragma unroll
      for (int i = 0; i < 16; i += 2 * w) v[i] = v[i] + v[i + w];
    r[row] = v[0];
  }
  const float s = (r[0] + r[1]) + (r[2] + r[3]);
  return (s + 0.0f) + (0.0f + 0.0f);
}
// The three parts of fragment (cb, kb) of one lane (isum == nullptr, B <=
// 64: the item sums computed here)
__device__ __forceinline__ void w0_frag_parts(const float *W0, const float *isum, int in,
                                              int B, int D, int cb, int kb, int lane,
                                              bf16x8 (&out)[3]) {
  const int n = 32 * cb + (lane & 31), k0 = 16 * kb + 8 * (lane >> 5);
  const int BD = B * D, K = BD + D;
  const float *Wn = W0 + (size_t)n * in;
  float hi[8], mid[8], lo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k0 + j;
    float w = 0.0f;
    if (k < BD)
      w = Wn[(k / D) * 2 * D + k % D];
    else if (k < K)
      w = isum ? isum[n * D + (k - BD)] : item_sum_tree(Wn + D + (k - BD), D, B);
    split3(w * (1.0f / (float)kCapacity), hi[j], mid[j], lo[j]);
  }
  out[0] = __builtin_bit_cast(bf16x8, u32x4{pk(hi[0], hi[1]), pk(hi[2], hi[3]),
                                            pk(hi[4], hi[5]), pk(hi[6], hi[7])});
  out[1] = __builtin_bit_cast(bf16x8, u32x4{pk(mid[0], mid[1]), pk(mid[2], mid[3]),
                                            pk(mid[4], mid[5]), pk(mid[6], mid[7])});
  out[2] = __builtin_bit_cast(bf16x8, u32x4{pk(lo[0], lo[1]), pk(lo[2], lo[3]),
                                            pk(lo[4], lo[5]), pk(lo[6], lo[7])});
}
__global__ void w0_frag_kernel(const float *W0, const float *isum, int in, int B, int D,
                               int nkb, bf16x8 *frag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * nkb * 64) return;
  const int lane = i & 63, kb = (i >> 6) % nkb, cb = (i >> 6) / nkb;
  bf16x8 v[3];
  w0_frag_parts(W0, isum, in, B, D, cb, kb, lane, v);
  const size_t f = ((size_t)cb * nkb + kb) * 64 + lane, ps = (size_t)2 * nkb * 64;
  frag[f] = v[0];
  frag[f + ps] = v[1];
  frag[f + 2 * ps] = v[2];
}

// ---------------------------------------------------------------- forward --
struct FwdArgs {
  const int8_t *bins, *items;
  int BD, D;
  // rows >= term_from are terminal views E_t (rl.h:336-343): transition
  // q = term_list[row - term_from], state S_t with bins[action[q]] -= item
  const int32_t *action;
  int term_from;
  const int *term_list;
  const int *rows;  // device row count (nullptr: max_rows)
  int max_rows;
  const bf16x8 *w0f;
  int nkb;
  // w0src != nullptr (up to 64 bins, fresh parameters): every wave splits its
  // own fragments from W0 (w0_frag_kernel's values, its launch saved) and
  // workgroup 0 stores them to w0f_out for the next forward
  const float *w0src;
  bf16x8 *w0f_out;
  int in, B;
  const float *b0, *W1, *b1, *W2, *b2;
  float *act0, *act1;  // layer outputs of rows < act_rows (the backward's)
  int act_rows;
  float *out;
  float *v_term;  // non-null: V of row term_from + j also to v_term[term_list[j]]
};

// The observation bytes of one 64-row tile move HBM -> registers (one tile
// ahead, coalesced 16-byte loads) -> LDS as bf16 (each byte converted once)
// -> the MFMA A operand (ds_read_b128).  A thread's chunk: 16 bytes
// (features 16 q .. 16 q + 15 of tile row r), and for a terminal view E_t
// (rl.h:336-343: transition q = term_list[row - term_from], the state S_t
// with bins[action[q]] -= item) its item dword and the action bin's first
// feature relative to the chunk.  Rows past M read row M - 1 (their outputs
// are never stored).
struct FwdChunk {
  u32x4 v;
  unsigned it;
  int sk;
};
constexpr int kNoTerm = -(1 << 20);
__device__ __forceinline__ int fwd_idx(const FwdArgs &o, int m, int &sub) {
  sub = -1;
  if (o.action && m >= o.term_from) {
    const int qi = o.term_list ? o.term_list[m - o.term_from] : m - o.term_from;
    sub = o.action[qi];
    return qi;
  }
  return m;
}

// One 64-row tile per iteration of a persistent workgroup.  Layer 0: wave w
// = (column block cb = w & 1, k half kh = w >> 1) holds its W0 fragments in
// registers for the whole launch and sums its k half for both 32-row blocks
// from the bf16 tile in LDS; the k halves meet in LDS (wave (cb, kh)
// finishes row block kh).  Layer 1 (16x16x4 f32 MFMA, wave w: rows
// 16w..16w+15) and layer 2 (a 16-lane DPP sum) from the H1 tile in LDS.
// Per tile: K loop | barrier | stage tile + 1, load tile + 2 | H1 | barrier |
// layers 1, 2.
// SPLIT: the W0 split inside (o.w0src; instantiated up to NKH 3 -- beyond, the
// item sums' unrolled loads spill the kernel)
template <int NKH, bool SPLIT>  // >= k blocks per half
__global__ __launch_bounds__(256, 1) void vnet_forward_kernel(FwdArgs o) {
  constexpr int XP = 32 * NKH + 8;          // bf16 row stride (848 B at NKH 13)
  constexpr int NCH = (2 * NKH + 3) / 4;    // 16-byte chunks per thread and tile
  __shared__ __attribute__((aligned(16))) __bf16 xs[TM][XP];
  __shared__ float red[2][2][16][64];  // [cb][row block][acc reg][lane]
  __shared__ __attribute__((aligned(16))) float h1s[TM][V1 + 4];
  __shared__ __attribute__((aligned(16))) float w1s[V2][V1 + 4];
  const int M = o.rows ? min(o.max_rows, *o.rows) : o.max_rows;
  const int ntiles = (M + TM - 1) / TM;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5, l15 = lane & 15, q = lane >> 4;
  const int cb = w & 1, kh = w >> 1;
  const int nkb = 2 * NKH, kbase = NKH * kh;  // o.nkb == 2 NKH (zero-padded)
  const int BD = o.BD, D = o.D, K = BD + D, ncpr = BD / 16;
  bf16x8 wf[NKH][3];
  const size_t ps = (size_t)2 * nkb * 64;
  // the fragments from W0; workgroup 0 stores them (with or without a tile)
  auto split_w0 = [&]() {
#pragma unroll
    for (int kb = 0; kb < NKH; ++kb)
      w0_frag_parts(o.w0src, nullptr, o.in, o.B, D, cb, kbase + kb, lane, wf[kb]);
    if (blockIdx.x == 0) {
#pragma unroll
      for (int kb = 0; kb < NKH; ++kb) {
        const size_t f = ((size_t)cb * nkb + kbase + kb) * 64 + lane;
#pragma unroll
        for (int p = 0; p < 3; ++p) o.w0f_out[f + p * ps] = wf[kb][p];
      }
    }
  };
  if ((int)blockIdx.x >= ntiles) {  // uniform
    if constexpr (SPLIT)
      if (blockIdx.x == 0) split_w0();
    return;
  }
  for (int i = tid; i < V2 * V1; i += 256) w1s[i / V1][i % V1] = o.W1[i];
  // features K .. 16 nkb - 1 meet zero weights: finite zeros, once
  for (int i = tid; i < TM * (16 * nkb - K); i += 256)
    xs[i / (16 * nkb - K)][K + i % (16 * nkb - K)] = (__bf16)0.0f;
  if constexpr (SPLIT) {
    split_w0();
  } else {
#pragma unroll
    for (int kb = 0; kb < NKH; ++kb) {
      const size_t f = ((size_t)cb * nkb + kbase + kb) * 64 + lane;
#pragma unroll
      for (int p = 0; p < 3; ++p) wf[kb][p] = o.w0f[f + p * ps];
    }
  }
  const float bias0 = o.b0[32 * cb + l31];
  const float b1a = o.b1[l15], b1b = o.b1[16 + l15];
  const float w2a = o.W2[l15], w2b = o.W2[16 + l15], b2 = o.b2[0];

  // this thread's chunks (fixed for the launch) and its tile row's item
  int cr[NCH], cq[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = tid + 256 * i;
    cr[i] = c / ncpr;
    cq[i] = c - cr[i] * ncpr;
  }
  FwdChunk ch[NCH];
  unsigned rit = 0u;
  // (the tile-uniform fast path has no branch on a loaded value: such a
  // branch makes the compiler wait for every load before it -- 7 HBM
  // latencies in a row per tile)
  auto fetch = [&](int t) {
    const int m0 = t * TM;
    if (!(o.action && m0 + TM > o.term_from)) {  // no terminal view in the tile
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int m = min(m0 + min(cr[i], TM - 1), M - 1);
        ch[i].v = *(const u32x4 *)(o.bins + (size_t)m * BD + 16 * cq[i]);
        ch[i].sk = kNoTerm;
      }
      rit = *(const unsigned *)(o.items + (size_t)min(m0 + (tid & (TM - 1)), M - 1) * 4);
      return;
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      int sub;
      const int idx = fwd_idx(o, min(m0 + min(cr[i], TM - 1), M - 1), sub);
      ch[i].v = *(const u32x4 *)(o.bins + (size_t)idx * BD + 16 * cq[i]);
      ch[i].it = *(const unsigned *)(o.items + (size_t)idx * 4);
      ch[i].sk = sub >= 0 ? sub * D - 16 * cq[i] : kNoTerm;
    }
    int sub;
    const int idx = fwd_idx(o, min(m0 + (tid & (TM - 1)), M - 1), sub);
    rit = *(const unsigned *)(o.items + (size_t)idx * 4);
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (cr[i] < TM) {
        float f[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) f[b] = sbyte(ch[i].v[b >> 2], b & 3);
        const int d = ch[i].sk;
        if (d > -D && d < 16) {  // terminal view: bins[action] -= item
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int c = j - d;
            if (c >= 0 && c < D) f[j] -= sbyte(ch[i].it, c);
          }
        }
        *(u32x4 *)&xs[cr[i]][16 * cq[i]] =
            u32x4{pk(f[0], f[1]), pk(f[2], f[3]), pk(f[4], f[5]), pk(f[6], f[7])};
        *(u32x4 *)&xs[cr[i]][16 * cq[i] + 8] =
            u32x4{pk(f[8], f[9]), pk(f[10], f[11]), pk(f[12], f[13]), pk(f[14], f[15])};
      }
    }
    if (tid < TM)
      for (int c = 0; c < D; ++c) xs[tid][BD + c] = (__bf16)sbyte(rit, c);
  };

  int tile = blockIdx.x;
  fetch(tile);
  stage();
  if (tile + (int)gridDim.x < ntiles) fetch(tile + gridDim.x);
  __syncthreads();
  for (; tile < ntiles; tile += gridDim.x) {
    const int nxt = tile + gridDim.x;
    f32x16 acc[2] = {zero16(), zero16()};
    // (no branch while the accumulators live: a conditional MFMA block
    // makes the compiler copy them between AGPRs and VGPRs around it)
#pragma unroll
    for (int kb = 0; kb < NKH; ++kb) {
      const int k0 = 16 * (kbase + kb) + 8 * h;
      const bf16x8 A0 = *(const bf16x8 *)&xs[l31][k0];
      const bf16x8 A1 = *(const bf16x8 *)&xs[32 + l31][k0];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        acc[0] = mfma_bf(A0, wf[kb][p], acc[0]);
        acc[1] = mfma_bf(A1, wf[kb][p], acc[1]);
      }
    }
    // the k halves: wave (cb, kh) hands row block 1 - kh to its partner
#pragma unroll
    for (int r = 0; r < 16; ++r) red[cb][1 - kh][r][lane] = kh ? acc[0][r] : acc[1][r];
    __syncthreads();
    float hv1[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      hv1[r] = fmaxf((kh ? acc[1][r] : acc[0][r]) + red[cb][kh][r][lane] + bias0, 0.0f);
    if (nxt < ntiles) stage();  // every K-loop read of this tile is done
    const int m0 = tile * TM;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = 32 * kh + acc_row(r, h), m = m0 + i;
      h1s[i][32 * cb + l31] = hv1[r];
      if (m < o.act_rows && m < M) o.act0[(size_t)m * V1 + 32 * cb + l31] = hv1[r];
    }
    __syncthreads();
    // layer 1: rows 16w + (l & 15), k = 16 q + s
    f32x4 c1[2] = {zero4(), zero4()};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const f32x4 hv = *(const f32x4 *)&h1s[16 * w + l15][16 * q + 4 * s4];
      const f32x4 wa = *(const f32x4 *)&w1s[l15][16 * q + 4 * s4];
      const f32x4 wb = *(const f32x4 *)&w1s[16 + l15][16 * q + 4 * s4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        c1[0] = mfma16(hv[e], wa[e], c1[0]);
        c1[1] = mfma16(hv[e], wb[e], c1[1]);
      }
    }
    // H2 and layer 2: row 16w + 4q + r, columns l & 15 and 16 + (l & 15)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 16 * w + 4 * q + r;
      const float ha = fmaxf(c1[0][r] + b1a, 0.0f), hb = fmaxf(c1[1][r] + b1b, 0.0f);
      if (m < o.act_rows && m < M) {
        o.act1[(size_t)m * V2 + l15] = ha;
        o.act1[(size_t)m * V2 + 16 + l15] = hb;
      }
      const float pv = seg_sum<16>(ha * w2a + hb * w2b);
      if (l15 == 0 && m < M) {
        const float v = pv + b2;
        o.out[m] = v;
        if (o.v_term && m >= o.term_from) o.v_term[o.term_list[m - o.term_from]] = v;
      }
    }
    // tile + 2's bytes, after this tile's stores: in flight over the next
    // tile's K loop
    if (nxt + (int)gridDim.x < ntiles) fetch(nxt + gridDim.x);
  }
}

// --------------------------------------------------------------- backward --
struct BwdArgs {
  const int8_t *bins, *items;
  int BD, D;
  int M, N;  // transition rows (row q = slot t * N + env), envs
  const uint8_t *done;
  const float *v_state, *v_term;  // V(S_0..S_T) of the forward, V(E_t) by row
  float gamma;
  float *targets, *row_g;
  const float *act0, *act1, *W1, *W2;
  float *slab;
  int stride, splits, in;  // slab stride, workgroups, Fin
  int o1, o2;              // flat offsets of layers 1 and 2
};

// value_targets_kernel's arithmetic (TD(0) target, square_loss_grad,
// nn.h:548-550), uncontracted, on values loaded beforehand (no branch on a
// loaded value in the prefetch: the compiler would wait for every load)
__device__ __forceinline__ float td_grad(float gamma, unsigned done, float v, float vnext,
                                         float vterm, float &target) {
#pragma clang fp contract(off)
  const float reward = done ? 0.0f : 1.0f;
  const float vn = done ? vterm : vnext;
  target = reward + gamma * vn;
  return v - target;
}

// Workgroup z sums rows [z kper, (z + 1) kper) in 64-row chunks into its
// slab (the flat parameter layout; the reduced layer 0 writes bin 0's item
// columns only, SlabAlias): per chunk
//   g2 = V - target; g1 = (g2 W2) [H2 > 0]; dW2 += g2^T H2, db1 += sum g1 (VALU)
//   g0 = (g1 W1) [H1 > 0] (16x16x4 f32 MFMA), split into three bf16 parts
//   dW1 += g1^T H1 (32x32x2 f32 MFMA; wave w: columns 32 (w & 1), rows half w >> 1)
//   [dW0 | db0] += g0^T [x | 1] (32x32x16 bf16 MFMA; wave w: row block w & 1
//   of dW0, column blocks (w >> 1) + 2i; x^T staged as bf16 in LDS)
// with the next chunk's loads in flight during the MFMAs.
template <int NKC>  // >= 32-wide column blocks of [x | 1]
__global__ __launch_bounds__(256, 1) void vnet_backward_kernel(BwdArgs o) {
  constexpr int XS = TM + 8;                  // bf16 row stride: 144 B
  constexpr int NT0 = (NKC + 1) / 2;          // dW0 tiles per wave
  constexpr int NW = (2 * 32 * NKC + 255) / 256;  // obs dword columns x 8 rows per thread
  // [x | 1]^T; rows K + 1 .. stay zero (wave pair 1's last tile when NKC is
  // odd reads zeros: no conditional MFMA)
  __shared__ __attribute__((aligned(16))) __bf16 xt[64 * NT0][XS];
  __shared__ __attribute__((aligned(16))) __bf16 g0t[3][V1][XS];    // g0^T parts
  __shared__ __attribute__((aligned(16))) float a0s[TM][V1 + 4];
  __shared__ float a1s[TM][V2 + 1];
  __shared__ __attribute__((aligned(16))) float g1s[TM][V2 + 4];
  __shared__ float g2s[TM];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5, l15 = lane & 15, q = lane >> 4;
  const int z = blockIdx.x;
  const int kper = (o.M + o.splits - 1) / o.splits;
  const int r0 = min(o.M, z * kper), r1 = min(o.M, r0 + kper);
  const int BD = o.BD, K = BD + o.D, ncol4 = BD / 4;
  // rows K+1 .. 64 NT0 - 1 of x^T stay zero
  for (int i = tid; i < (64 * NT0 - (K + 1)) * TM; i += 256)
    xt[K + 1 + i / TM][i % TM] = (__bf16)0.0f;
  // W1 as the B operand of g0 = g1 W1: [n = 8q + s][j = 16t + (l & 15)]
  float w1r[4][8];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int s = 0; s < 8; ++s) w1r[t][s] = o.W1[(8 * q + s) * V1 + 16 * t + l15];
  const int vn = tid & 31, vg = tid >> 5;  // VALU sums: unit n, rows 8 vg..8 vg+7
  const float w2n = o.W2[vn];
  float db1p = 0.0f, dw2p = 0.0f, db2p = 0.0f;
  const int jb = w & 1, kc0 = w >> 1;
  f32x16 accW0[NT0];
#pragma unroll
  for (int i = 0; i < NT0; ++i) accW0[i] = zero16();
  f32x16 accW1 = zero16();

  // ---- the loads of one chunk into registers
  unsigned xb[NW][8];
  f32x4 pa0[4], pa1[2];
  unsigned pit = 0, pdone = 0;
  float pv = 0.0f, pvn = 0.0f, pvt = 0.0f;
  int plast = 0;
  // rows past the chunk's n read its last row (finite values): their g2,
  // hence g1 and g0, and their ones column are zero, so they add nothing
  auto fetch = [&](int c0) {
    const int last = min(TM, r1 - c0) - 1;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int wi = min(tid + 256 * i, 8 * ncol4 - 1), rg = wi / ncol4, dc = wi - rg * ncol4;
      const int8_t *p = o.bins + (size_t)c0 * BD + 4 * dc;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        xb[i][e] = *(const unsigned *)(p + (size_t)min(8 * rg + e, last) * BD);
    }
    const int ar = min(tid >> 2, last), ac = tid & 3;
#pragma unroll
    for (int v = 0; v < 4; ++v)
      pa0[v] = *(const f32x4 *)(o.act0 + (size_t)(c0 + ar) * V1 + 16 * ac + 4 * v);
#pragma unroll
    for (int v = 0; v < 2; ++v)
      pa1[v] = *(const f32x4 *)(o.act1 + (size_t)(c0 + ar) * V2 + 8 * ac + 4 * v);
    {
      const int q = c0 + min(tid & (TM - 1), last);
      pit = *(const unsigned *)(o.items + (size_t)q * 4);
      pdone = o.done[q];
      pv = o.v_state[q];
      pvn = o.v_state[q + o.N];
      pvt = o.v_term[q];
      plast = last;
    }
  };

  if (r0 < r1) fetch(r0);
  for (int c0 = r0; c0 < r1; c0 += TM) {
    const int n = min(TM, r1 - c0);
    __syncthreads();  // the previous chunk's readers are done
    // ---- stage: x^T (bins, items, ones), H1, H2, g2
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int wi = tid + 256 * i, rg = wi / ncol4, dc = wi - rg * ncol4;
      if (rg < 8) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const u32x4 v{pk(sbyte(xb[i][0], b), sbyte(xb[i][1], b)),
                        pk(sbyte(xb[i][2], b), sbyte(xb[i][3], b)),
                        pk(sbyte(xb[i][4], b), sbyte(xb[i][5], b)),
                        pk(sbyte(xb[i][6], b), sbyte(xb[i][7], b))};
          *(u32x4 *)&xt[4 * dc + b][8 * rg] = v;
        }
      }
    }
    if (tid < TM) {
      float tg;
      const float g = tid <= plast ? td_grad(o.gamma, pdone, pv, pvn, pvt, tg) : 0.0f;
      for (int c = 0; c < o.D; ++c) xt[BD + c][tid] = (__bf16)sbyte(pit, c);
      xt[K][tid] = (__bf16)(tid < n ? 1.0f : 0.0f);
      g2s[tid] = g;
      if (tid < n) {
        o.targets[c0 + tid] = tg;
        o.row_g[c0 + tid] = g;
      }
    }
    {
      const int ar = tid >> 2, ac = tid & 3;
#pragma unroll
      for (int v = 0; v < 4; ++v) *(f32x4 *)&a0s[ar][16 * ac + 4 * v] = pa0[v];
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int e = 0; e < 4; ++e) a1s[ar][8 * ac + 4 * v + e] = pa1[v][e];
    }
    __syncthreads();
    fetch(c0 + TM < r1 ? c0 + TM : c0);  // (the last chunk re-reads itself)
    // ---- g1 = (g2 W2) [H2 > 0]; dW2, db1, db2 partial sums
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int r = 8 * vg + e;
      const float g2 = g2s[r], a1 = a1s[r][vn];
      const float g1 = a1 > 0.0f ? g2 * w2n : 0.0f;
      g1s[r][vn] = g1;
      db1p += g1;
      dw2p += g2 * a1;
      db2p += g2;
    }
    __syncthreads();
    // ---- g0 = (g1 W1) [H1 > 0]: rows 16w + 4q + r, columns 16t + (l & 15)
    {
      f32x4 c[4] = {zero4(), zero4(), zero4(), zero4()};
      const f32x4 ga = *(const f32x4 *)&g1s[16 * w + l15][8 * q];
      const f32x4 gb = *(const f32x4 *)&g1s[16 * w + l15][8 * q + 4];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const float a = s < 4 ? ga[s] : gb[s - 4];
#pragma unroll
        for (int t = 0; t < 4; ++t) c[t] = mfma16(a, w1r[t][s], c[t]);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float hi[4], mid[4], lo[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float g = a0s[16 * w + 4 * q + r][16 * t + l15] > 0.0f ? c[t][r] : 0.0f;
          split3(g, hi[r], mid[r], lo[r]);
        }
        const int j = 16 * t + l15, rr = 16 * w + 4 * q;
        *(u32x2 *)&g0t[0][j][rr] = u32x2{pk(hi[0], hi[1]), pk(hi[2], hi[3])};
        *(u32x2 *)&g0t[1][j][rr] = u32x2{pk(mid[0], mid[1]), pk(mid[2], mid[3])};
        *(u32x2 *)&g0t[2][j][rr] = u32x2{pk(lo[0], lo[1]), pk(lo[2], lo[3])};
      }
    }
    // ---- dW1 += g1^T H1: A[n = l31][k = h] = g1[r][n], B[k][j] = H1[r][j]
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int r = 32 * kc0 + 2 * s + h;
      accW1 = mfma32(g1s[r][l31], a0s[r][32 * jb + l31], accW1);
    }
    __syncthreads();
    // ---- [dW0 | db0] += g0^T [x | 1]
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 A[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) A[p] = *(const bf16x8 *)&g0t[p][32 * jb + l31][16 * s + 8 * h];
#pragma unroll
      for (int i = 0; i < NT0; ++i) {
        const int kc = kc0 + 2 * i;
        const bf16x8 B = *(const bf16x8 *)&xt[32 * kc + l31][16 * s + 8 * h];
#pragma unroll
        for (int p = 0; p < 3; ++p) accW0[i] = mfma_bf(A[p], B, accW0[i]);
      }
    }
  }

  // ---- the slab of split z
  float *S = o.slab + (size_t)z * o.stride;
  const int D = o.D, in = o.in;
#pragma unroll
  for (int i = 0; i < NT0; ++i) {
    const int kc = kc0 + 2 * i;
    {
      const int f = 32 * kc + l31;  // reduced feature (K: the ones column)
      int col = -1;
      if (f < BD)
        col = (f / D) * 2 * D + f % D;
      else if (f < K)
        col = D + (f - BD);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = 32 * jb + acc_row(r, h);
        if (col >= 0)  // x^T held the integers: the 1/kCapacity (exact)
          S[(size_t)j * in + col] = accW0[i][r] * (1.0f / (float)kCapacity);
        else if (f == K)
          S[(size_t)V1 * in + j] = accW0[i][r];
      }
    }
  }
  __syncthreads();  // LDS reuse below
  float *red = &a0s[0][0];  // [jb][16 regs][64 lanes] of the rows-half 1 waves
  if (kc0 == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(jb * 16 + r) * 64 + lane] = accW1[r];
  }
  float *vs = &g1s[0][0];  // [3][8][32] VALU partial sums
  vs[(0 * 8 + vg) * 32 + vn] = db1p;
  vs[(1 * 8 + vg) * 32 + vn] = dw2p;
  vs[(2 * 8 + vg) * 32 + vn] = db2p;
  __syncthreads();
  if (kc0 == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int nrow = acc_row(r, h);
      S[o.o1 + nrow * V1 + 32 * jb + l31] = accW1[r] + red[(jb * 16 + r) * 64 + lane];
    }
  }
  if (tid < V2) {
    float a = 0.0f, b = 0.0f;
    for (int g = 0; g < 8; ++g) {
      a += vs[(0 * 8 + g) * 32 + tid];
      b += vs[(1 * 8 + g) * 32 + tid];
    }
    S[o.o1 + V2 * V1 + tid] = a;
    S[o.o2 + tid] = b;
    if (tid == 0) {
      float c = 0.0f;
      for (int g = 0; g < 8; ++g) c += vs[(2 * 8 + g) * 32];
      S[o.o2 + V2] = c;
    }
  }
}

}  // namespace vnet

// ------------------------------------------------------------------ host --
// layer 0's k blocks per half (the forward's template bound, exact: nkb is
// padded to 2 NKH with zero-weight blocks)
static int vnet_nkh(const EnvDesc &e) {
  const int h = ((e.B * e.D + e.D + 15) / 16 + 1) / 2;
  static const int bucket[] = {1, 2, 3, 4, 5, 6, 8, 10, 13};
  for (int b : bucket)
    if (h <= b) return b;
  return 0;
}
static int vnet_nkb(const EnvDesc &e) { return 2 * vnet_nkh(e); }
// [x | 1]'s 32-wide column blocks (the backward's template bound, exact)
static int vnet_nkc(const EnvDesc &e) {
  const int c = (e.B * e.D + e.D + 1 + 31) / 32;
  static const int bucket[] = {2, 3, 4, 5, 6, 8, 10, 13};
  for (int b : bucket)
    if (c <= b) return b;
  return 0;
}

// W0's fragments, then the item-column sums [64][D]
static size_t vnet_frag_only(const EnvDesc &e) { return (size_t)3 * 2 * vnet_nkb(e) * 64 * 16; }
size_t vnet_frag_bytes(const EnvDesc &e) { return vnet_frag_only(e) + 64 * 3 * 4; }

bool vnet_shape_ok(const MlpArgs &a) {
  const int BD = a.env.B * a.env.D;
  return a.nlayers == 3 && a.w[1] == vnet::V1 && a.w[2] == vnet::V2 && a.w[3] == 1 &&
         a.env.D >= 1 && a.env.D <= 3 && BD % 16 == 0 && a.w[0] == 2 * BD &&
         vnet_nkh(a.env) > 0 && vnet_nkc(a.env) > 0 && a.w0frag != nullptr;
}

static int layer_off(const int *w, int l) {
  int off = 0;
  for (int i = 0; i < l; ++i) off += w[i + 1] * w[i] + w[i + 1];
  return off;
}

hipError_t vnet_forward(const MlpArgs &a, hipStream_t s) {
  using namespace vnet;
  const int nkb = vnet_nkb(a.env);
  const int in = a.w[0];
  bf16x8 *frag = (bf16x8 *)a.w0frag;
  float *isum = (float *)((char *)a.w0frag + vnet_frag_only(a.env));
  // up to 64 bins the forward splits W0 itself, item sums included (config
  // 2: two launches fewer per forward than the item kernel + the fragment
  // kernel); at 128 bins the serial sums cost more.  XH_W0_FUSE=0: the item
  // kernel and the fragment kernel; =1: the fragment kernel with the item
  // sums (tests compare the three)
  static const int fuse_mode = [] {
    const char *e = std::getenv("XH_W0_FUSE");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : 2;
  }();
  const bool fuse = fuse_mode >= 1 && a.env.B <= 64;
  const bool in_fwd = fuse_mode == 2 && a.env.B <= 64 && vnet_nkh(a.env) <= 3 &&
                      !a.w0frag_ready;
  if (!a.w0frag_ready && !in_fwd) {
    if (!fuse)
      hipLaunchKernelGGL(w0_item_kernel, dim3(V1 * a.env.D), dim3(256), 0, s, a.params, in,
                         a.env.B, a.env.D, isum);
    hipLaunchKernelGGL(w0_frag_kernel, dim3((2 * nkb * 64 + 255) / 256), dim3(256), 0, s,
                       a.params, fuse ? nullptr : (const float *)isum, in, a.env.B, a.env.D,
                       nkb, frag);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int o1 = layer_off(a.w, 1), o2 = layer_off(a.w, 2);
  FwdArgs o{};
  o.bins = a.bins;
  o.items = a.items;
  o.BD = a.env.B * a.env.D;
  o.D = a.env.D;
  o.action = a.action;
  o.term_from = a.term_from;
  o.term_list = a.term_list;
  o.rows = a.rows;
  o.max_rows = a.max_rows;
  o.w0f = frag;
  o.nkb = nkb;
  o.w0src = in_fwd ? a.params : nullptr;
  o.w0f_out = frag;
  o.in = in;
  o.B = a.env.B;
  o.b0 = a.params + (size_t)V1 * in;
  o.W1 = a.params + o1;
  o.b1 = a.params + o1 + V2 * V1;
  o.W2 = a.params + o2;
  o.b2 = a.params + o2 + V2;
  o.act0 = a.act[0];
  o.act1 = a.act[1];
  // MlpArgs::act_rows (xh_kernels.h): 0 = every row, < 0 = none
  o.act_rows = a.act_rows < 0 ? 0 : a.act_rows == 0 ? a.max_rows : a.act_rows;
  o.out = a.act[2];
  o.v_term = a.v_term && a.term_list ? a.v_term : nullptr;
  const int tiles = (a.max_rows + TM - 1) / TM;
  // up to 512 workgroups (two per CU) where the kernel's registers allow two
  // waves per SIMD (NKH <= 6: configs 2 / 3, value phase 0.055 -> 0.053 and
  // 0.156 -> 0.133 ms per iteration); one tile each, so its prefetch idles
  const int gcap = vnet_nkh(a.env) <= 6 ? 512 : 256;
  const dim3 grid(tiles < gcap ? (tiles < 1 ? 1 : tiles) : gcap);
  switch (vnet_nkh(a.env)) {
#define XH_VNET_FWD(n)                                                          \
  case n:                                                                       \
    if constexpr (n <= 3) {                                                     \
      if (in_fwd) {                                                             \
        hipLaunchKernelGGL((vnet_forward_kernel<n, true>), grid, dim3(256), 0, s, o); \
        break;                                                                  \
      }                                                                         \
    }                                                                           \
    hipLaunchKernelGGL((vnet_forward_kernel<n, false>), grid, dim3(256), 0, s, o); \
    break;
    XH_VNET_FWD(1) XH_VNET_FWD(2) XH_VNET_FWD(3) XH_VNET_FWD(4) XH_VNET_FWD(5)
    XH_VNET_FWD(6) XH_VNET_FWD(8) XH_VNET_FWD(10) XH_VNET_FWD(13)
#undef XH_VNET_FWD
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t vnet_backward(const MlpArgs &a, const ValueArgs &va, float gamma,
                         float *targets, float *slab, int stride, int splits,
                         hipStream_t s) {
  using namespace vnet;
  BwdArgs o{};
  o.bins = a.bins;
  o.items = a.items;
  o.BD = a.env.B * a.env.D;
  o.D = a.env.D;
  o.M = a.max_rows;
  o.N = va.b.N;
  o.done = va.b.done;
  o.v_state = va.v_state;
  o.v_term = va.v_term;
  o.gamma = gamma;
  o.targets = targets;
  o.row_g = a.grad[2];
  o.act0 = a.act[0];
  o.act1 = a.act[1];
  o.o1 = layer_off(a.w, 1);
  o.o2 = layer_off(a.w, 2);
  o.W1 = a.params + o.o1;
  o.W2 = a.params + o.o2;
  o.slab = slab;
  o.stride = stride;
  o.splits = splits < 1 ? 1 : splits;
  o.in = a.w[0];
  const dim3 grid(o.splits);
  switch (vnet_nkc(a.env)) {
#define XH_VNET_BWD(n)                                                          \
  case n:                                                                       \
    hipLaunchKernelGGL(vnet_backward_kernel<n>, grid, dim3(256), 0, s, o);      \
    break;
    XH_VNET_BWD(2) XH_VNET_BWD(3) XH_VNET_BWD(4) XH_VNET_BWD(5) XH_VNET_BWD(6)
    XH_VNET_BWD(8) XH_VNET_BWD(10) XH_VNET_BWD(13)
#undef XH_VNET_BWD
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace xh
