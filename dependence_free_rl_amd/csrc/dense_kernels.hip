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
  const int n = bn + wn * 32 + lr;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = bm + wm * 32 + acc_row(r, h);
    if (m < M && n < N) ep(m, n, blockIdx.z, acc[r]);
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

hipError_t mlp_forward(const MlpArgs &a, hipStream_t s) {
  using namespace dense;
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

}  // namespace xh
