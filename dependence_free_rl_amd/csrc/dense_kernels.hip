// dense_kernels.hip -- full_layer (nn.h:60-110) forward / backward as one
// f32 MFMA GEMM template for gfx950, plus the row-gathering loaders that let
// a layer read observations straight from the int8 env states.
//
// C(m, n) = sum_k A(m, k) B(k, n), 64x64 output tile per 256-thread
// workgroup (4 waves in a 2x2 grid of 32x32 v_mfma_f32_32x32x2_f32 tiles),
// K staged through LDS in slices of 16 with a register prefetch of the next
// slice.  The operand loaders and the epilogue are template functors:
//   forward      Y = act(X W^T + b)           A = X rows, B = W^T
//   data grad    dX = (dY W) * [H > 0]        A = dY, B = W, relu mask of H
//   weight grad  [dW | db] = dY^T [X | 1]     A = dY^T, B = [X | 1], split-K
//                                             over rows into per-split slabs
// One dimension may be a device-side row count (rows of this learn() batch),
// so a launch needs no host synchronisation.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {
namespace dense {

// K slice depth (make variant VSRC=dense_kernels VFLAGS=-DXH_DENSE_BK=..):
// 32 and 64 measured slower than 16 on the value net (config 5: +0.5%, +2.7%
// per iteration) -- the obs-gathering loader, not the barriers, sets the pace
#ifndef XH_DENSE_BK
#define XH_DENSE_BK 16
#endif
constexpr int BM = 64, BN = 64, BK = XH_DENSE_BK, PAD = 4;
constexpr int NJ = BM * BK / 256;  // slice elements per thread per operand
static_assert(BK == 16 || BK == 32 || BK == 64, "BK");

// ------------------------------------------------------------- loaders ----
// Each loader returns element (i, k) of its operand viewed as [I x K]; for A
// i = m, for B i = n.  kKContig: consecutive k are adjacent in memory (pick
// the thread -> element order that coalesces).
struct RowMajor {  // p[i * ld + k]
  const float *p;
  int ld;
  static constexpr bool kKContig = true;
  static constexpr bool kRowCtx = false;
  __device__ float operator()(int i, int k) const { return p[(size_t)i * ld + k]; }
};
struct ColMajor {  // p[k * ld + i]
  const float *p;
  int ld;
  static constexpr bool kKContig = false;
  static constexpr bool kRowCtx = false;
  __device__ float operator()(int i, int k) const { return p[(size_t)k * ld + i]; }
};
// [X | 1] as the B operand of a weight gradient: element (n, k=row) =
// X[row][n] for n < ncol, 1 for n == ncol (the bias column).
struct RowsOnes {
  const float *p;
  int ld, ncol;
  static constexpr bool kKContig = false;
  static constexpr bool kRowCtx = false;
  __device__ float operator()(int n, int r) const {
    return n < ncol ? p[(size_t)r * ld + n] : 1.0f;
  }
};
// observation::to_vector (bin_packing.h:31-40, generalised to D dims) of
// row r: feature k = bin (k / 2D), c = k % 2D: c < D -> bins[bin][c] / 8,
// else item[c - D] / 8.  Row r is slot s, env e with s * N + e = list[r]
// (list == nullptr: slot `slot`, env r).  With `action`, rows r >= term_from
// are the terminal views E_t of transition q = r - term_from (or q =
// term_list[r - term_from]): the state of slot t with bins[action[q]] -=
// item, taken before the reset (rl.h:336-343).
template <int DC>  // dims, compile time: the feature -> (bin, c) split is
struct ObsRows {   // a constant division
  EnvDesc E;
  const int8_t *bins, *items;
  const int *list;
  int N, slot;
  const int32_t *action;
  int term_from;
  const int *term_list;
  // (slot*N + env, terminal action or -1) of row r: resolved once per row
  struct RowCtx {
    int idx, sub;
  };
  __device__ RowCtx ctx(int r) const {
    RowCtx c{0, -1};
    if (action && r >= term_from) {
      c.idx = term_list ? term_list[r - term_from] : r - term_from;
      c.sub = action[c.idx];
    } else {
      c.idx = list ? list[r] : slot * N + r;
    }
    return c;
  }
  __device__ float feature_at(RowCtx rc, int k) const {
    const int bin = k / (2 * DC), c = k - bin * 2 * DC;
    int v = c < DC ? bins[(size_t)rc.idx * E.B * DC + bin * DC + c]
                   : items[(size_t)rc.idx * 4 + c - DC];
    if (c < DC && bin == rc.sub) v -= items[(size_t)rc.idx * 4 + c];
    return (float)v * (1.0f / (float)kCapacity);
  }
  __device__ float feature(int r, int k) const { return feature_at(ctx(r), k); }
};
template <int DC>
struct ObsA : ObsRows<DC> {  // A operand: (m = row, k = feature)
  using RowCtx = typename ObsRows<DC>::RowCtx;
  static constexpr bool kKContig = true;
  // a thread's rows are fixed for the whole K loop: the GEMM resolves them
  // once per tile (ctx) instead of once per K slice
  static constexpr bool kRowCtx = true;
  __device__ float operator()(int r, int k) const { return this->feature(r, k); }
  __device__ float at(RowCtx rc, int k) const { return this->feature_at(rc, k); }
};
template <int DC>
struct ObsOnesB : ObsRows<DC> {  // B operand of dW1: (n = feature | 1, k = row)
  int ncol;
  static constexpr bool kKContig = false;
  static constexpr bool kRowCtx = false;
  __device__ float operator()(int n, int r) const {
    return n < ncol ? this->feature(r, n) : 1.0f;
  }
};
// The reduced observation of a row: the B*D bin features, then the D item
// features once (to_vector repeats the item in every bin's row; layer 0's
// weights for those copies are pre-summed, reduce_w0_kernel).  Feature k < BD:
// bin k / DC, dim k % DC; k >= BD: item dim k - BD.
template <int DC>
struct ObsRedRows : ObsRows<DC> {
  using RowCtx = typename ObsRows<DC>::RowCtx;
  __device__ float red_at(RowCtx rc, int k) const {
    const int BD = this->E.B * DC;
    int v;
    if (k < BD) {
      const int bin = k / DC, c = k - bin * DC;
      v = this->bins[(size_t)rc.idx * BD + k];
      if (bin == rc.sub) v -= this->items[(size_t)rc.idx * 4 + c];
    } else {
      v = this->items[(size_t)rc.idx * 4 + (k - BD)];
    }
    return (float)v * (1.0f / (float)kCapacity);
  }
};
template <int DC>
struct ObsRedA : ObsRedRows<DC> {  // A operand: (m = row, k = reduced feature)
  using RowCtx = typename ObsRows<DC>::RowCtx;
  static constexpr bool kKContig = true;
  static constexpr bool kRowCtx = true;
  __device__ float operator()(int r, int k) const {
    return this->red_at(this->ctx(r), k);
  }
  __device__ float at(RowCtx rc, int k) const { return this->red_at(rc, k); }
};
template <int DC>
struct ObsRedOnesB : ObsRedRows<DC> {  // B of dW1: (n = reduced feature | 1, k = row)
  int ncol;  // B*D + D
  static constexpr bool kKContig = false;
  static constexpr bool kRowCtx = false;
  __device__ float operator()(int n, int r) const {
    return n < ncol ? this->red_at(this->ctx(r), n) : 1.0f;
  }
};

// the observation loaders of MlpArgs a, for D = DC
template <class L>
__host__ L obs_loader(const MlpArgs &a) {
  L l;
  l.E = a.env;
  l.bins = a.bins;
  l.items = a.items;
  l.list = a.list;
  l.N = a.N;
  l.slot = a.slot;
  l.action = a.action;
  l.term_from = a.term_from;
  l.term_list = a.term_list;
  return l;
}

// ----------------------------------------------------------- epilogues ----
struct EpBiasAct {  // Y[m][n] = act(c + b[n])
  float *y;
  int ld;
  const float *bias;
  int relu;
  __device__ void operator()(int m, int n, int, float c) const {
    float v = c + bias[n];
    if (relu) v = v > 0.0f ? v : 0.0f;
    y[(size_t)m * ld + n] = v;
  }
};
struct EpReluMask {  // dX[m][n] = H[m][n] > 0 ? c : 0 (relu backward, nn.h:364-376)
  float *dx;
  int ld;
  const float *h;
  __device__ void operator()(int m, int n, int, float c) const {
    dx[(size_t)m * ld + n] = h[(size_t)m * ld + n] > 0.0f ? c : 0.0f;
  }
};
// Layer-0 weight gradient over reduced features n (see ObsRedRows): bin
// feature (b, c) -> column b*2D + c; item feature c -> bin 0's item column
// D + c only (the other bins' item columns hold the same row sum: the slab
// reduce reads them from bin 0's, SlabAlias); n == B*D + D -> bias.
struct EpSlabRed {
  float *slab;
  int stride, oW, oB, in, B, D;
  __device__ void operator()(int m, int n, int split, float c) const {
    float *s = slab + (size_t)split * stride;
    const int BD = B * D;
    if (n < BD)
      s[oW + m * in + (n / D) * 2 * D + n % D] = c;
    else if (n < BD + D)
      s[oW + m * in + D + (n - BD)] = c;
    else
      s[oB + m] = c;
  }
};
struct EpSlab {  // weight-gradient slab: [A(out x in), b(out)] of one layer
  float *slab;
  int stride, oW, oB, in;
  __device__ void operator()(int m, int n, int split, float c) const {
    float *s = slab + (size_t)split * stride;
    if (n < in)
      s[oW + m * in + n] = c;
    else
      s[oB + m] = c;
  }
};

// ---------------------------------------------------------------- GEMM ----
namespace detail {
template <class L, bool = L::kRowCtx>
struct CtxOf {
  using type = int;
};
template <class L>
struct CtxOf<L, true> {
  using type = typename L::RowCtx;
};
}  // namespace detail

// One 64x64 output tile (rows bm.., columns bn..) over K range [k0, k1):
// the waves' 32x32 accumulators (wave w: rows 32 (w & 1), columns 32 (w >> 1)).
// Every caller that needs the GEMM's bits runs this exact chain.
template <class LA, class LB>
__device__ __forceinline__ f32x16 gemm_tile(const LA &la, const LB &lb, int M,
                                            int N, int bm, int bn, int k0, int k1,
                                            float (&As)[BK][BM + PAD],
                                            float (&Bs)[BK][BN + PAD]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 31, h = lane >> 5, wm = w & 1, wn = w >> 1;
  f32x16 acc = zero16();

  // this thread's NJ (i, kk) positions in a BM x BK (or BN x BK) slice
  auto pos = [&](bool kcontig, int j, int &i, int &kk) {
    if (kcontig) {
      kk = tid & (BK - 1);
      i = tid / BK + (256 / BK) * j;
    } else {
      i = tid & 63;
      kk = (tid >> 6) + 4 * j;
    }
  };
  float ra[NJ], rb[NJ];
  // row contexts of this thread's four A rows (kKContig: i does not depend
  // on the K slice), for loaders that gather rows
  struct NoCtx {};
  using Ctx = std::conditional_t<LA::kRowCtx, typename detail::CtxOf<LA>::type, NoCtx>;
  Ctx rc[NJ];
  if constexpr (LA::kRowCtx) {
    static_assert(LA::kKContig, "row contexts need fixed rows per thread");
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      int i, kk;
      pos(true, j, i, kk);
      const int m = bm + i;
      rc[j] = la.ctx(m < M ? m : 0);
    }
  }
  auto fetch = [&](int kb) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      int i, kk;
      pos(LA::kKContig, j, i, kk);
      const int m = bm + i, k = kb + kk;
      if constexpr (LA::kRowCtx)
        ra[j] = (m < M && k < k1) ? la.at(rc[j], k) : 0.0f;
      else
        ra[j] = (m < M && k < k1) ? la(m, k) : 0.0f;
      pos(LB::kKContig, j, i, kk);
      const int n = bn + i;
      rb[j] = (n < N && kb + kk < k1) ? lb(n, kb + kk) : 0.0f;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      int i, kk;
      pos(LA::kKContig, j, i, kk);
      As[kk][i] = ra[j];
      pos(LB::kKContig, j, i, kk);
      Bs[kk][i] = rb[j];
    }
  };

  if (k0 < k1) fetch(k0);
  for (int kb = k0; kb < k1; kb += BK) {
    __syncthreads();
    stash();
    __syncthreads();
    if (kb + BK < k1) fetch(kb + BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2)
      acc = mfma32(As[kk + h][wm * 32 + lr], Bs[kk + h][wn * 32 + lr], acc);
  }
  return acc;
}

// dyn: 0 = static sizes, 1 = M is *rows, 2 = K is *rows (each <= the static
// bound).  Split-K: blockIdx.z takes K range [z*kper, (z+1)*kper).
template <class LA, class LB, class EP>
__global__ __launch_bounds__(256) void gemm_kernel(LA la, LB lb, EP ep, int M,
                                                   int N, int K, const int *rows,
                                                   int dyn) {
  __shared__ float As[BK][BM + PAD];
  __shared__ float Bs[BK][BN + PAD];
  if (dyn == 1) M = min(M, *rows);
  if (dyn == 2) K = min(K, *rows);
  const int bm = blockIdx.x * BM, bn = blockIdx.y * BN;
  if (bm >= M && dyn == 1) return;  // no rows for this tile (uniform exit)
  const int splits = gridDim.z;
  int kper = (K + splits - 1) / splits;
  kper = (kper + BK - 1) / BK * BK;
  const int k0 = blockIdx.z * kper, k1 = min(K, k0 + kper);
  const f32x16 acc = gemm_tile(la, lb, M, N, bm, bn, k0, k1, As, Bs);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lr = lane & 31, h = lane >> 5, wm = w & 1, wn = w >> 1;
  const int n = bn + wn * 32 + lr;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = bm + wm * 32 + acc_row(r, h);
    if (m < M && n < N) ep(m, n, blockIdx.z, acc[r]);
  }
}

// ---------------------------------------------- the value MLP, fused ----
// The value net of the learners (full Fin -> 64 -> 32 -> 1 with relu between,
// the value_h1 / value_h2 defaults; ppo_training.cc:19-26) in three launches
// per update instead of nine, every output bit-identical to the layer-by-
// layer GEMMs above: each fused phase feeds the MFMA the operand values of
// the corresponding gemm_kernel launch in the same k order (gemm_tile itself
// for the observation-gathering layer 0, the LDS-resident hidden tiles for
// the others), and the same epilogue arithmetic.
constexpr int kFV1 = 64, kFV2 = 32;
constexpr int kHS = kFV1 + 2;  // LDS row stride of the hidden tiles: lanes
                               // (lr, h) read row lr, column k + h -> banks
                               // 2 lr + h, conflict-free
struct Mlp3Fwd {
  const float *b0, *W1, *b1, *W2, *b2;
  float *act0, *act1, *out;
  const int *term_list;  // non-null: rows >= term_from also write V to
  int term_from;         // v_term[term_list[row - term_from]]
  float *v_term;
};

// Forward, one 64-row tile per workgroup: layer 0 (gemm_tile), layer 1 and
// layer 2 from the tile in LDS.  act0 / act1 are written for the backward.
template <class LA, class LB>
__global__ __launch_bounds__(256) void mlp3_forward_kernel(LA la, LB w0, Mlp3Fwd o,
                                                           int M, int K0,
                                                           const int *rows) {
  __shared__ float As[BK][BM + PAD];
  __shared__ float Bs[BK][BN + PAD];
  __shared__ float Hs[BM][kHS];        // H1, then H2 in columns 0..31
  __shared__ float W1s[kFV2][kHS];     // W1 [out][in]
  __shared__ float W2s[kFV2];
  if (rows) M = min(M, *rows);
  const int bm = blockIdx.x * BM;
  if (bm >= M) return;  // uniform
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 31, h = lane >> 5, wm = w & 1, wn = w >> 1;
  for (int i = tid; i < kFV2 * kFV1; i += 256) W1s[i / kFV1][i % kFV1] = o.W1[i];
  if (tid < kFV2) W2s[tid] = o.W2[tid];
  // layer 0: mlp_forward's first GEMM tile (its barriers also order the
  // staging above before the reads below)
  const f32x16 acc = gemm_tile(la, w0, M, kFV1, bm, 0, 0, K0, As, Bs);
  {
    const int n = wn * 32 + lr;
    const float b = o.b0[n];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = wm * 32 + acc_row(r, h), m = bm + i;
      float v = acc[r] + b;
      v = v > 0.0f ? v : 0.0f;
      Hs[i][n] = v;
      if (m < M) o.act0[(size_t)m * kFV1 + n] = v;
    }
  }
  __syncthreads();
  // layer 1 (64 -> 32): the waves of output columns 0..31
  f32x16 acc1 = zero16();
  if (wn == 0) {
#pragma unroll
    for (int k = 0; k < kFV1; k += 2)
      acc1 = mfma32(Hs[wm * 32 + lr][k + h], W1s[lr][k + h], acc1);
  }
  __syncthreads();  // every read of H1 done before H2 replaces it
  if (wn == 0) {
    const float b = o.b1[lr];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = wm * 32 + acc_row(r, h), m = bm + i;
      float v = acc1[r] + b;
      v = v > 0.0f ? v : 0.0f;
      Hs[i][lr] = v;
      if (m < M) o.act1[(size_t)m * kFV2 + lr] = v;
    }
  }
  __syncthreads();
  // layer 2 (32 -> 1): output column 0 (lanes lr == 0)
  if (wn == 0) {
    f32x16 acc2 = zero16();
#pragma unroll
    for (int k = 0; k < kFV2; k += 2)
      acc2 = mfma32(Hs[wm * 32 + lr][k + h], lr == 0 ? W2s[k + h] : 0.0f, acc2);
    if (lr == 0) {
      const float b = o.b2[0];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = bm + wm * 32 + acc_row(r, h);
        if (m < M) {
          const float v = acc2[r] + b;
          o.out[m] = v;
          if (o.term_list && m >= o.term_from) o.v_term[o.term_list[m - o.term_from]] = v;
        }
      }
    }
  }
}

// Backward through the data path for one 64-row tile of transition rows:
// value_targets_kernel's TD targets and dL/dV = V - target (square_loss_grad,
// nn.h:548-550), then dX2 = (dV W2) * [H2 > 0] and dX1 = (dX2 W1) * [H1 > 0]
// (the two EpReluMask GEMMs of mlp_backward, their chains: K = 1 and K = 32).
struct Mlp3Bwd {
  ValueArgs va;
  float gamma;
  float *targets;
  const float *W1, *W2, *act0, *act1;
  float *g2, *g1, *g0;  // dV [rows], dX2 [rows][32], dX1 [rows][64]
};
__global__ __launch_bounds__(256) void mlp3_backward_data_kernel(Mlp3Bwd o, int M) {
#pragma clang fp contract(off)
  __shared__ float G2[BM][kHS];      // dX2 tile (columns 0..31)
  __shared__ float W1s[kFV2][kHS];   // W1 [out k][in n]
  __shared__ float rg[BM];
  const int bm = blockIdx.x * BM;
  if (bm >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 31, h = lane >> 5, wm = w & 1, wn = w >> 1;
  for (int i = tid; i < kFV2 * kFV1; i += 256) W1s[i / kFV1][i % kFV1] = o.W1[i];
  if (tid < BM) {
    const int q = bm + tid;
    float g = 0.0f;
    if (q < M) {
      const int N = o.va.b.N;
      const int done = o.va.b.done[q];
      const float reward = done ? 0.0f : 1.0f;
      const float vn = done ? o.va.v_term[q] : o.va.v_state[q + N];
      const float target = reward + o.gamma * vn;
      o.targets[q] = target;
      g = o.va.v_state[q] - target;
      o.g2[q] = g;
    }
    rg[tid] = g;
  }
  __syncthreads();
  // dX2: K = 1 (k = 0 in lane half 0 of the first step; the rest of the
  // gemm's BK = 16 slice is its zero pad, kept so the bits match)
  if (wn == 0) {
    const float ga = h == 0 ? rg[wm * 32 + lr] : 0.0f, gb = h == 0 ? o.W2[lr] : 0.0f;
    f32x16 acc = mfma32(ga, gb, zero16());
#pragma unroll
    for (int kk = 2; kk < BK; kk += 2) acc = mfma32(0.0f, 0.0f, acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = wm * 32 + acc_row(r, h), m = bm + i;
      float v = 0.0f;
      if (m < M) {
        v = o.act1[(size_t)m * kFV2 + lr] > 0.0f ? acc[r] : 0.0f;
        o.g1[(size_t)m * kFV2 + lr] = v;
      }
      G2[i][lr] = v;
    }
  }
  __syncthreads();
  // dX1: K = 32, every wave (64 x 64)
  f32x16 acc = zero16();
#pragma unroll
  for (int k = 0; k < kFV2; k += 2)
    acc = mfma32(G2[wm * 32 + lr][k + h], W1s[k + h][wn * 32 + lr], acc);
  const int n = wn * 32 + lr;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = bm + wm * 32 + acc_row(r, h);
    if (m < M)
      o.g0[(size_t)m * kFV1 + n] = o.act0[(size_t)m * kFV1 + n] > 0.0f ? acc[r] : 0.0f;
  }
}

// The three weight-gradient GEMMs of mlp_backward ([dW | db] = dY^T [X | 1],
// split-K over the rows into slabs) in one launch of ntiles x splits
// workgroups: tile b enumerates layer 2's tile, layer 1's two and layer 0's
// n0 tiles, z the split.  Workgroups are dispatched round-robin over the 8
// XCDs, so (when splits % 8 == 0) XCD x runs the splits x S/8 .. (x+1) S/8 - 1
// with all their tiles back to back: the tiles of a split read the same rows
// of dY (layer 0's tiles the same dZ1 rows), and one L2 serves them, where
// tile-major order spread them over several XCDs (config 3: each dZ1 row
// fetched three times).  Every tile sums the same rows in the same order
// either way.
template <class LB0, class EP0>
__global__ __launch_bounds__(256) void mlp3_weight_grad_kernel(
    ColMajor d2, RowsOnes x2, EpSlab e2, ColMajor d1, RowsOnes x1, EpSlab e1,
    ColMajor d0, LB0 x0, EP0 e0, int N0, int K, int ntiles, int splits) {
  __shared__ float As[BK][BM + PAD];
  __shared__ float Bs[BK][BN + PAD];
  const int L = blockIdx.x;
  int b, z;  // uniform
  if ((splits & 7) == 0) {
    const int slot = L >> 3;
    z = (L & 7) * (splits >> 3) + slot / ntiles;
    b = slot % ntiles;
  } else {
    z = L / ntiles;
    b = L % ntiles;
  }
  int kper = (K + splits - 1) / splits;
  kper = (kper + BK - 1) / BK * BK;
  const int k0 = z * kper, k1 = min(K, k0 + kper);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lr = lane & 31, h = lane >> 5, wm = w & 1, wn = w >> 1;
  auto out = [&](const f32x16 &acc, int M, int N, int bn, auto &ep) {
    const int n = bn + wn * 32 + lr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = wm * 32 + acc_row(r, h);
      if (m < M && n < N) ep(m, n, z, acc[r]);
    }
  };
  if (b == 0) {
    out(gemm_tile(d2, x2, 1, kFV2 + 1, 0, 0, k0, k1, As, Bs), 1, kFV2 + 1, 0, e2);
  } else if (b < 3) {
    const int bn = (b - 1) * BN;
    out(gemm_tile(d1, x1, kFV2, kFV1 + 1, 0, bn, k0, k1, As, Bs), kFV2, kFV1 + 1, bn, e1);
  } else {
    const int bn = (b - 3) * BN;
    out(gemm_tile(d0, x0, kFV1, N0, 0, bn, k0, k1, As, Bs), kFV1, N0, bn, e0);
  }
}

template <class LA, class LB, class EP>
hipError_t gemm(LA la, LB lb, EP ep, int M, int N, int K, const int *rows,
                int dyn, int splits, hipStream_t s) {
  dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN, splits < 1 ? 1 : splits);
  hipLaunchKernelGGL((gemm_kernel<LA, LB, EP>), grid, dim3(256), 0, s, la, lb,
                     ep, M, N, K, rows, dyn);
  return hipGetLastError();
}

}  // namespace dense

// ------------------------------------------------- full MLPs (pg, value) --
// Layer l of a full MLP whose flat parameters follow model::parameters()
// (nn.h:499-508): widths w[0] = input, ..., w[L] = output.
static int layer_offset(const int *w, int l) {
  int off = 0;
  for (int i = 0; i < l; ++i) off += w[i + 1] * w[i] + w[i + 1];
  return off;
}

// Layer-0 weights on the reduced observation: out[n][k] for k < B*D is
// W[n][bin*2D + c], for k = B*D + c the sum over bins (ascending) of the
// item copies' weights W[n][bin*2D + D + c].
__global__ void reduce_w0_kernel(const float *W, int out, int B, int D,
                                 float *red) {
  const int BD = B * D, K = BD + D, in = 2 * BD;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < out * K;
       i += gridDim.x * blockDim.x) {
    const int n = i / K, k = i - n * K;
    float v;
    if (k < BD) {
      v = W[(size_t)n * in + (k / D) * 2 * D + k % D];
    } else {
      v = 0.0f;
      for (int b = 0; b < B; ++b) v += W[(size_t)n * in + b * 2 * D + D + (k - BD)];
    }
    red[i] = v;
  }
}

enum ValueKernel { kValGemm, kValMlp3, kValVnet };
static ValueKernel value_kernel(const MlpArgs &a) {
  const char *e = std::getenv("XH_VALUE_KERNEL");
  if (e && std::strcmp(e, "gemm") == 0) return kValGemm;
  const bool mlp3 = a.nlayers == 3 && a.w[1] == dense::kFV1 &&
                    a.w[2] == dense::kFV2 && a.w[3] == 1;
  if (!(e && std::strcmp(e, "mlp3") == 0) && vnet_shape_ok(a)) return kValVnet;
  return mlp3 ? kValMlp3 : kValGemm;
}
static bool value_fused(const MlpArgs &a) { return value_kernel(a) == kValMlp3; }
const char *value_kernel_name(const MlpArgs &a) {
  switch (value_kernel(a)) {
    case kValVnet: return "vnet_bf16";
    case kValMlp3: return "mlp3_fused";
    default: return "gemm";
  }
}
bool value_reduced_slab(const MlpArgs &a) {
  return value_kernel(a) == kValVnet || a.w0red != nullptr;
}

static hipError_t mlp3_forward(const MlpArgs &a, hipStream_t s) {
  using namespace dense;
  const int in = a.w[0];
  const float *W0 = a.params;
  const int o1 = layer_offset(a.w, 1), o2 = layer_offset(a.w, 2);
  Mlp3Fwd o{W0 + kFV1 * in, a.params + o1, a.params + o1 + kFV2 * kFV1,
            a.params + o2, a.params + o2 + kFV2, a.act[0], a.act[1], a.act[2],
            a.v_term ? a.term_list : nullptr, a.term_from, a.v_term};
  const dim3 grid((a.max_rows + BM - 1) / BM);
  auto run = [&](auto la, const RowMajor &w0, int K0) {
    hipLaunchKernelGGL((mlp3_forward_kernel<decltype(la), RowMajor>), grid,
                       dim3(256), 0, s, la, w0, o, a.max_rows, K0, a.rows);
    return hipGetLastError();
  };
  if (a.w0red) {
    const int K = a.env.B * a.env.D + a.env.D;
    int nb = (kFV1 * K + 255) / 256;
    nb = nb > 1024 ? 1024 : nb;
    hipLaunchKernelGGL(reduce_w0_kernel, dim3(nb), dim3(256), 0, s, W0, kFV1,
                       a.env.B, a.env.D, a.w0red);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const RowMajor wr{a.w0red, K};
    if (a.env.D == 1) return run(obs_loader<ObsRedA<1>>(a), wr, K);
    if (a.env.D == 2) return run(obs_loader<ObsRedA<2>>(a), wr, K);
    return run(obs_loader<ObsRedA<3>>(a), wr, K);
  }
  const RowMajor wt{W0, in};
  if (a.env.D == 1) return run(obs_loader<ObsA<1>>(a), wt, in);
  if (a.env.D == 2) return run(obs_loader<ObsA<2>>(a), wt, in);
  return run(obs_loader<ObsA<3>>(a), wt, in);
}

hipError_t mlp_forward(const MlpArgs &a, hipStream_t s) {
  using namespace dense;
  if (value_kernel(a) == kValVnet) return vnet_forward(a, s);
  if (value_fused(a)) return mlp3_forward(a, s);
  hipError_t e = hipSuccess;
  for (int l = 0; l < a.nlayers && e == hipSuccess; ++l) {
    const int in = a.w[l], out = a.w[l + 1];
    const float *W = a.params + layer_offset(a.w, l);
    EpBiasAct ep{a.act[l], out, W + out * in, l + 1 < a.nlayers};
    RowMajor wt{W, in};  // B(n = out unit, k) = W[n][k]
    if (l == 0 && a.w0red) {
      const int K = a.env.B * a.env.D + a.env.D;
      int nb = (out * K + 255) / 256;
      nb = nb > 1024 ? 1024 : nb;
      hipLaunchKernelGGL(reduce_w0_kernel, dim3(nb), dim3(256), 0, s, W, out,
                         a.env.B, a.env.D, a.w0red);
      e = hipGetLastError();
      if (e != hipSuccess) break;
      RowMajor wr{a.w0red, K};
      auto run = [&](auto la) {
        return gemm(la, wr, ep, a.max_rows, out, K, a.rows, a.rows ? 1 : 0, 1,
                    s);
      };
      if (a.env.D == 1)
        e = run(obs_loader<ObsRedA<1>>(a));
      else if (a.env.D == 2)
        e = run(obs_loader<ObsRedA<2>>(a));
      else
        e = run(obs_loader<ObsRedA<3>>(a));
    } else if (l == 0) {
      auto run = [&](auto la) {
        return gemm(la, wt, ep, a.max_rows, out, in, a.rows, a.rows ? 1 : 0, 1,
                    s);
      };
      if (a.env.D == 1)
        e = run(obs_loader<ObsA<1>>(a));
      else if (a.env.D == 2)
        e = run(obs_loader<ObsA<2>>(a));
      else
        e = run(obs_loader<ObsA<3>>(a));
    } else {
      RowMajor la{a.act[l - 1], in};
      e = gemm(la, wt, ep, a.max_rows, out, in, a.rows, a.rows ? 1 : 0, 1, s);
    }
  }
  if (e == hipSuccess && a.v_term && a.term_list)
    e = launch_scatter_list(a.term_list, a.term_n, a.act[a.nlayers - 1] + a.term_from,
                            a.v_term, a.max_rows - a.term_from, s);
  return e;
}

hipError_t mlp_backward(const MlpArgs &a, float *slab, int stride, int splits,
                        hipStream_t s) {
  using namespace dense;
  hipError_t e = hipSuccess;
  for (int l = a.nlayers - 1; l >= 0 && e == hipSuccess; --l) {
    const int in = a.w[l], out = a.w[l + 1];
    const int off = layer_offset(a.w, l);
    // [dW | db] = dY^T [X | 1] over the batch rows (nn.h:81-100)
    ColMajor dyT{a.grad[l], out};  // A(m = out unit, k = row) = dY[row][m]
    EpSlab es{slab, stride, off, off + out * in, in};
    if (l == 0 && a.w0red) {
      const int K = a.env.B * a.env.D + a.env.D;
      EpSlabRed er{slab, stride, off, off + out * in, in, a.env.B, a.env.D};
      auto run = [&](auto lb) {
        lb.ncol = K;
        return gemm(dyT, lb, er, out, K + 1, a.max_rows, a.rows,
                    a.rows ? 2 : 0, splits, s);
      };
      if (a.env.D == 1)
        e = run(obs_loader<ObsRedOnesB<1>>(a));
      else if (a.env.D == 2)
        e = run(obs_loader<ObsRedOnesB<2>>(a));
      else
        e = run(obs_loader<ObsRedOnesB<3>>(a));
    } else if (l == 0) {
      auto run = [&](auto lb) {
        lb.ncol = in;
        return gemm(dyT, lb, es, out, in + 1, a.max_rows, a.rows,
                    a.rows ? 2 : 0, splits, s);
      };
      if (a.env.D == 1)
        e = run(obs_loader<ObsOnesB<1>>(a));
      else if (a.env.D == 2)
        e = run(obs_loader<ObsOnesB<2>>(a));
      else
        e = run(obs_loader<ObsOnesB<3>>(a));
    } else {
      RowsOnes lb{a.act[l - 1], in, in};
      e = gemm(dyT, lb, es, out, in + 1, a.max_rows, a.rows, a.rows ? 2 : 0,
               splits, s);
      if (e != hipSuccess) break;
      // dX = (dY W) * relu'(X); layer 0 gets no backward (nn.h:516-526)
      RowMajor dy{a.grad[l], out};              // A(m = row, k = out unit)
      ColMajor wn{a.params + off, in};          // B(n = in unit, k) = W[k][n]
      EpReluMask em{a.grad[l - 1], in, a.act[l - 1]};
      e = gemm(dy, wn, em, a.max_rows, in, out, a.rows, a.rows ? 1 : 0, 1, s);
    }
  }
  return e;
}

hipError_t value_backward(const MlpArgs &a, const ValueArgs &va, float gamma,
                          float *targets, float *slab, int stride, int splits,
                          hipStream_t s) {
  using namespace dense;
  if (value_kernel(a) == kValVnet)
    return vnet_backward(a, va, gamma, targets, slab, stride, splits, s);
  if (!value_fused(a)) {
    ValueArgs v = va;
    v.row_g = a.grad[a.nlayers - 1];
    hipError_t e = launch_value_targets(v, gamma, targets, s);
    return e != hipSuccess ? e : mlp_backward(a, slab, stride, splits, s);
  }
  const int M = a.max_rows, in = a.w[0];
  const int o1 = layer_offset(a.w, 1), o2 = layer_offset(a.w, 2);
  Mlp3Bwd o{va, gamma, targets, a.params + o1, a.params + o2, a.act[0],
            a.act[1], a.grad[2], a.grad[1], a.grad[0]};
  hipLaunchKernelGGL(mlp3_backward_data_kernel, dim3((M + BM - 1) / BM), dim3(256),
                     0, s, o, M);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const ColMajor d2{a.grad[2], 1}, d1{a.grad[1], kFV2}, d0{a.grad[0], kFV1};
  const RowsOnes x2{a.act[1], kFV2, kFV2}, x1{a.act[0], kFV1, kFV1};
  const EpSlab e2{slab, stride, o2, o2 + kFV2, kFV2};
  const EpSlab e1{slab, stride, o1, o1 + kFV2 * kFV1, kFV1};
  const int sp = splits < 1 ? 1 : splits;
  auto run = [&](auto x0, auto e0, int N0) {
    const int nt = 3 + (N0 + BN - 1) / BN;
    hipLaunchKernelGGL((mlp3_weight_grad_kernel<decltype(x0), decltype(e0)>),
                       dim3(nt * sp), dim3(256), 0, s, d2, x2, e2, d1, x1, e1, d0, x0,
                       e0, N0, M, nt, sp);
    return hipGetLastError();
  };
  if (a.w0red) {
    const int K = a.env.B * a.env.D + a.env.D;
    const EpSlabRed er{slab, stride, 0, kFV1 * in, in, a.env.B, a.env.D};
    auto go = [&](auto lb) {
      lb.ncol = K;
      return run(lb, er, K + 1);
    };
    if (a.env.D == 1) return go(obs_loader<ObsRedOnesB<1>>(a));
    if (a.env.D == 2) return go(obs_loader<ObsRedOnesB<2>>(a));
    return go(obs_loader<ObsRedOnesB<3>>(a));
  }
  const EpSlab es{slab, stride, 0, kFV1 * in, in};
  auto go = [&](auto lb) {
    lb.ncol = in;
    return run(lb, es, in + 1);
  };
  if (a.env.D == 1) return go(obs_loader<ObsOnesB<1>>(a));
  if (a.env.D == 2) return go(obs_loader<ObsOnesB<2>>(a));
  return go(obs_loader<ObsOnesB<3>>(a));
}

// ------------------------------------------------ model::eval on device --
// softmax_layer / softmax_cross_entropy_layer forward (nn.h:382-392, 424-431):
// exp(z) / sum exp(z) over each row, no max shift, the sum in column order.
__global__ void softmax_rows_kernel(float *y, int rows, int cols) {
#pragma clang fp contract(off)
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < rows;
       r += gridDim.x * blockDim.x) {
    float *row = y + (size_t)r * cols;
    float sum = 0.0f;
    for (int c = 0; c < cols; ++c) {
      row[c] = expf(row[c]);
      sum += row[c];
    }
    for (int c = 0; c < cols; ++c) row[c] = row[c] / sum;
  }
}

__global__ void relu_kernel(float *y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    y[i] = y[i] > 0.0f ? y[i] : 0.0f;
}

// Forward of a layer chain over `rows` input rows of `cols` features (every
// buffer device memory; a and b are ping-pong buffers big enough for the
// widest activation).  Dense layers run on the f32 MFMA GEMM with the bias
// and a following relu fused into the epilogue; conv1d_1 is the same GEMM
// over rows * (cols / in) points (nn.h:127-147).  Returns the output's
// buffer and column count.
hipError_t model_forward(const ModelLayer *layers, int nl, const float *params,
                         const float *x, int rows, int cols, float *a, float *b,
                         const float **out, int *out_cols, hipStream_t s) {
  using namespace dense;
  const float *cur = x;
  float *bufs[2] = {a, b};
  int which = 0;
  size_t poff = 0;
  hipError_t e = hipSuccess;
  for (int l = 0; l < nl && e == hipSuccess; ++l) {
    const ModelLayer &L = layers[l];
    float *dst = bufs[which];
    if (L.kind == kLayerFull || L.kind == kLayerConv1d) {
      const int pts = L.kind == kLayerFull ? 1 : cols / L.in;
      const int M = rows * pts;
      const float *W = params + poff;
      const bool fuse = l + 1 < nl && layers[l + 1].kind == kLayerRelu;
      EpBiasAct ep{dst, L.out, W + (size_t)L.out * L.in, fuse ? 1 : 0};
      RowMajor la{cur, L.in};
      RowMajor wt{W, L.in};
      e = gemm(la, wt, ep, M, L.out, L.in, nullptr, 0, 1, s);
      poff += (size_t)L.out * L.in + L.out;
      cols = pts * L.out;
      if (fuse) ++l;
    } else {
      const long n = (long)rows * cols;
      if (cur != dst)
        e = hipMemcpyAsync(dst, cur, n * 4, hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess) {
        if (L.kind == kLayerRelu)
          hipLaunchKernelGGL(relu_kernel, dim3((unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096)),
                             dim3(256), 0, s, dst, n);
        else
          hipLaunchKernelGGL(softmax_rows_kernel, dim3((rows + 255) / 256),
                             dim3(256), 0, s, dst, rows, cols);
        e = hipGetLastError();
      }
    }
    cur = dst;
    which ^= 1;
  }
  *out = cur;
  *out_cols = cols;
  return e;
}

// ------------------------------------- one layer: forward / backward / grad --
// The reference's layer interface (nn.h:20-33) on the device, one layer at a
// time, for model::forward / model::gradient / optimizer::step of the drop-in
// layer (xh_model_forward, xh_model_gradient, xh_layer_backward,
// xh_layer_gradient).  Dense layers (full: nn.h:71-100; conv1d_1: the same
// Dense over rows * points, nn.h:127-186) run on the f32 MFMA GEMM above.
struct EpStore {  // Y[m][n] = c
  float *y;
  int ld;
  __device__ void operator()(int m, int n, int, float c) const {
    y[(size_t)m * ld + n] = c;
  }
};

// relu_activation::backward (nn.h:363-376): the input's sign gates backprop
__global__ void relu_backward_kernel(const float *x, const float *bp, float *out,
                                     long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    out[i] = x[i] > 0.0f ? bp[i] : 0.0f;
}

// softmax_layer::backward (nn.h:393-417): the row's softmax s (the forward's
// exp / sum, no max shift) and the Jacobian product (diag(s) - s s^T) g,
// evaluated as s_j g_j - s_j (s . g) (the same sum, one rounding per term
// instead of a B x B matrix).  One thread per row.
__global__ void softmax_backward_kernel(const float *x, const float *bp,
                                        float *out, int rows, int cols) {
#pragma clang fp contract(off)
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < rows;
       r += gridDim.x * blockDim.x) {
    const float *xr = x + (size_t)r * cols, *g = bp + (size_t)r * cols;
    float *o = out + (size_t)r * cols;
    float sum = 0.0f;
    for (int c = 0; c < cols; ++c) sum += expf(xr[c]);
    float dot = 0.0f;
    for (int c = 0; c < cols; ++c) dot += (expf(xr[c]) / sum) * g[c];
    for (int c = 0; c < cols; ++c) {
      const float sj = expf(xr[c]) / sum;
      o[c] = sj * g[c] - sj * dot;
    }
  }
}

static unsigned elem_blocks(long n) {
  const long b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

// points of a Dense layer's input row (1 for full_layer)
static int layer_points(const ModelLayer &L, int cols) {
  return L.kind == kLayerFull ? 1 : cols / L.in;
}

hipError_t layer_forward(const ModelLayer &L, const float *W, const float *x,
                         int rows, int cols, float *y, hipStream_t s) {
  using namespace dense;
  const long n = (long)rows * cols;
  switch (L.kind) {
    case kLayerFull:
    case kLayerConv1d: {
      const int M = rows * layer_points(L, cols);
      EpBiasAct ep{y, L.out, W + (size_t)L.out * L.in, 0};
      return gemm(RowMajor{x, L.in}, RowMajor{W, L.in}, ep, M, L.out, L.in,
                  nullptr, 0, 1, s);
    }
    case kLayerRelu: {
      hipError_t e = hipMemcpyAsync(y, x, n * 4, hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(relu_kernel, dim3(elem_blocks(n)), dim3(256), 0, s, y, n);
      return hipGetLastError();
    }
    default: {  // softmax / softmax_cross_entropy: the same forward
      hipError_t e = hipMemcpyAsync(y, x, n * 4, hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(softmax_rows_kernel, dim3((rows + 255) / 256),
                         dim3(256), 0, s, y, rows, cols);
      return hipGetLastError();
    }
  }
}

hipError_t layer_backward(const ModelLayer &L, const float *W, const float *x,
                          int rows, int cols, const float *bp, float *out,
                          hipStream_t s) {
  using namespace dense;
  const long n = (long)rows * cols;
  switch (L.kind) {
    case kLayerFull:
    case kLayerConv1d: {  // dX = dY W (nn.h:77-79, 149-162)
      const int M = rows * layer_points(L, cols);
      return gemm(RowMajor{bp, L.out}, ColMajor{W, L.in}, EpStore{out, L.in}, M,
                  L.in, L.out, nullptr, 0, 1, s);
    }
    case kLayerRelu:
      hipLaunchKernelGGL(relu_backward_kernel, dim3(elem_blocks(n)), dim3(256),
                         0, s, x, bp, out, n);
      return hipGetLastError();
    case kLayerSoftmax:
      hipLaunchKernelGGL(softmax_backward_kernel, dim3((rows + 255) / 256),
                         dim3(256), 0, s, x, bp, out, rows, cols);
      return hipGetLastError();
    default:  // softmax_cross_entropy_layer::backward passes backprop through
      return hipMemcpyAsync(out, bp, n * 4, hipMemcpyDeviceToDevice, s);
  }
}

int layer_gradient_splits(const ModelLayer &L, int rows, int cols) {
  if (L.kind != kLayerFull && L.kind != kLayerConv1d) return 0;
  const long M = (long)rows * layer_points(L, cols);
  const long sp = (M + 1023) / 1024;
  return (int)(sp < 1 ? 1 : (sp > 64 ? 64 : sp));
}

hipError_t layer_gradient(const ModelLayer &L, const float *x, int rows,
                          int cols, const float *bp, float *slab, int stride,
                          float *grad, hipStream_t s) {
  using namespace dense;
  if (L.kind != kLayerFull && L.kind != kLayerConv1d) return hipSuccess;
  // [dW | db] = dY^T [X | 1] over rows * points (nn.h:81-100, 164-186),
  // split-K over the rows into slabs, then the fixed-order slab sum
  const int M = rows * layer_points(L, cols);
  const int splits = layer_gradient_splits(L, rows, cols);
  EpSlab es{slab, stride, 0, L.out * L.in, L.in};
  hipError_t e = gemm(ColMajor{bp, L.out}, RowsOnes{x, L.in, L.in}, es, L.out,
                      L.in + 1, M, nullptr, 0, splits, s);
  if (e != hipSuccess) return e;
  return launch_slab_reduce(slab, splits, stride, L.out * L.in + L.out, grad, s);
}

// xylo::matmul_transposed / matmul (tensor.cc:218-230) on device arrays
hipError_t launch_tensor_gemm(bool b_nk, const float *A, const float *B,
                              float *C, int M, int N, int K, hipStream_t st) {
  using namespace dense;
  if (M <= 0 || N <= 0) return hipSuccess;
  const RowMajor la{A, K};
  const EpStore ep{C, N};
  if (b_nk) return gemm(la, RowMajor{B, K}, ep, M, N, K, nullptr, 0, 1, st);
  return gemm(la, ColMajor{B, N}, ep, M, N, K, nullptr, 0, 1, st);
}

}  // namespace xh
