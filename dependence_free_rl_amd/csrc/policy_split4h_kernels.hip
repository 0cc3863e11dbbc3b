// policy_split4h_kernels.hip -- the PPO / actor-critic train epoch of the
// 32-bin 1-D [64,64] policy (BASELINE config 2): the pipelined kernel of
// policy_split8wh_kernels.hip (f16 pairs for layer 2 and dH1, the exact
// bf16 split for dW2, rank-1 backward; see its header and xh_split.h) for
// 64 features and 64-row groups of two 32-bin envs.
//
// Four waves per workgroup, wave w owning features 16 w .. 16 w + 15 of every
// product, two workgroups per CU (two waves per SIMD, 256 registers each).
// Per group: layer 2 24 f16 MFMAs per wave (K = 64: two K-slices), dW2 24
// bf16, dH1 16 f16.  The two envs of a group are rows 0-31 and 32-63: the
// softmax and its sums run over 32-lane segments, each env has its record
// (action, old probability, advantage) and its item -- the layer-1 bias
// (item folded in) is chosen per r-tile, the dW1 item sums per env.
//
//   X(j): MFMA layer 2 of group j+1 | VALU softmax + g of group j, masks,
//         dW3 / db2, g (x) H1 of K-step 0 (env A's rows); group j+1's
//         partial logits                                     -> barrier
//   Y(j): MFMA dW2 and dH1 of group j | VALU g (x) H1 of K-step 1 (env B's
//         rows), layer 1 of group j+2, dW1 of group j        -> barrier
//
// Images keep the 256-byte rows (and swizzles) of the 128-feature kernels
// with 64 features used.
#include <cstdlib>

#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

// Built twice (Makefile), as policy_split8wh_kernels.hip: the PPO /
// actor-critic kernel, and with XH_4H_KL_TU=1 (policy_split4h_kl_kernels.o)
// its KL-PPO form, policy_train_split4h_kl_kernel; the KL additions are
// preprocessor blocks, so the first object compiles from exactly its
// measured source.
#ifndef XH_4H_KL_TU
#define XH_4H_KL_TU 0
#endif
#if XH_4H_KL_TU
#define KLTU(...) __VA_ARGS__
#else
#define KLTU(...)
#endif

// Phase stamps (trace build, tools/build_trace4h.sh: -DXH_DIAG_TRACE=1, run
// with XH_PHASE_TRACE=1): lane 0 of every wave of the first kTraceBlocks
// workgroups records the cycle counter at 0 X start, 1 layer 2 (+ group j's
// VALU) done, 2 partial logits written, 3 after the X barrier, 4 dW2 / dH1
// blocks done, 5 dW1 tail done, 6 after the Y barrier (7 = 6) for groups
// j < kTraceGroups - 1; trace group kTraceGroups - 1 holds the kernel-level
// stamps 0 start, 1 pipeline filled, 2 groups done, 3 slab written.
#ifndef XH_DIAG_TRACE
#define XH_DIAG_TRACE 0
#endif
#if XH_DIAG_TRACE
#define S4H_STAMP(a, gi, w, lane, slot)                                         \
  do {                                                                        \
    if ((a).trace && blockIdx.x < kTraceBlocks && (gi) < kTraceGroups &&      \
        (lane) == 0)                                                          \
      (a).trace[((blockIdx.x * kTraceGroups + (gi)) * 8 + (w)) * kTraceSlots + \
                (slot)] = clock64();                                          \
  } while (0)
#else
#define S4H_STAMP(a, gi, w, lane, slot) \
  do {                                  \
  } while (0)
#endif

namespace xh {
namespace s4h {

constexpr int kD = 1, kF0 = 2 * kD, kH = 64;
constexpr int kNW = 4;                   // waves
constexpr int kThreads = 64 * kNW;
constexpr int kImg = 64 * kImgRow;       // one 64-row part image, 16 KB
constexpr int L_H1 = 0;                  // H1 as two f16 parts (S_H)
constexpr int L_MASK = 2 * kImg;         // relu mask (0 / 2.0: dW2 bf16, dH1 f16)
// (3 * kImg: the f16 mask image before the one-image masks, unused)
constexpr int L_F = 4 * kImg;
constexpr int F_W1T = 0;                 // [64 i]: W1[i][0], the bin column
constexpr int F_B1F = F_W1T + kH;        // [2 items][64]: b1 + the item's part
constexpr int F_B2 = F_B1F + 2 * kH;     // [64] b2 S_W S_H
constexpr int F_W3 = F_B2 + kH;          // [64] w3 / (S_W S_H)
constexpr int F_B3 = F_W3 + kH;          // [4]
constexpr int F_Z = F_B3 + 4;            // [2 parity][64 rows][4 waves] partial logits
constexpr int F_GW = F_Z + 2 * 64 * kNW; // [4 waves][64 rows] g, row order
constexpr int F_GP = F_GW + kNW * 64;    // [4 waves][16 li][4 rt] g, C-layout order
constexpr int F_X = F_GP + kNW * 64;     // [3 slots][64 rows] bins / 8
constexpr int F_XP = F_X + 3 * 64;       // [3 slots][16 li][4 rt]
constexpr int F_IT = F_XP + 3 * 64;      // [3 slots][2 envs] item is item_a (+ pad)
constexpr int F_REC = F_IT + 8;          // [3 slots][2 envs][action, pold, adv, -]
constexpr int F_SC = F_REC + 3 * 8;      // [16] the scales' reduction
constexpr int F_W3G = F_SC + 16;         // [64] w3 (the slab write-out's)
#if XH_4H_KL_TU
constexpr int F_Q = F_W3G + kH;          // KL-PPO: [3 slots][64 rows] old distribution
constexpr int F_END = F_Q + 3 * 64;
#else
constexpr int F_END = F_W3G + kH;
#endif
constexpr size_t kLds = L_F + sizeof(float) * F_END;
static_assert(2 * kLds <= 160 * 1024, "LDS: two workgroups per CU");
static_assert(F_REC % 4 == 0 && F_GW % 4 == 0 && F_GP % 4 == 0 && F_X % 4 == 0 &&
                  F_XP % 4 == 0 && F_Z % 4 == 0 && F_W1T % 4 == 0 && F_B1F % 4 == 0 &&
                  F_B2 % 4 == 0 && F_W3 % 4 == 0,
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
#define FENCE() __builtin_amdgcn_sched_barrier(0)
// XCD-aware work order (as policy_split8wh_kernels.hip: the adjacent
// records that share a 128-byte line are read by one XCD's L2)
#ifndef XH_4H_XCD
#define XH_4H_XCD 1
#endif

#if XH_4H_KL_TU
// kl_ppo_learner's epoch over every row of its state matrix (rows 0..TN-1
// the transitions, TN..TN+N-1 the open trajectories' end rows, then the
// n_end terminal end rows of end_list), two rows per 64-row group: each
// half resolves its own row, kind and validity (the last group's second
// half may lie past the rows: not valid).
__global__ __launch_bounds__(kThreads, 2) void policy_train_split4h_kl_kernel(
    PolicyTrainArgs a) {
#else
__global__ __launch_bounds__(kThreads, 2) void policy_train_split4h_kernel(
    PolicyTrainArgs a) {
#endif
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH, kH};
  const float *P = a.params;
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int l = tid & 63, G = l >> 4, li = l & 15;
  constexpr int kKG = kTraceGroups - 1;  // the kernel-level stamps' group
  S4H_STAMP(a, kKG, w, l, 0);
#if XH_4H_KL_TU
  const int NT = a.b.T * a.b.N;
  const int n_end = *a.n_end;
  const int nrows = NT + a.b.N + n_end;
  const int ngroups = (nrows + 1) / 2;  // 64-row groups of two rows
  const float beta = *a.beta;
#else
  const int ngroups = a.b.T * a.b.N / 2;  // 64-row groups of two envs
#endif
#if XH_4H_XCD
  const int b0 = ((int)gridDim.x & 7) == 0
                     ? ((int)blockIdx.x & 7) * ((int)gridDim.x >> 3) + ((int)blockIdx.x >> 3)
                     : (int)blockIdx.x;
#else
  const int b0 = (int)blockIdx.x;
#endif
  const int J = b0 < ngroups ? (ngroups - b0 + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  if (J == 0) return;  // uniform over the workgroup
  int gstep = (int)gridDim.x;
  // group index of this workgroup's group j (clamped: work past the end is
  // discarded); its envs are transitions 2 g and 2 g + 1 of the [T][N] arrays
  auto gindex = [&](int j) {
    return (size_t)(b0 + min(j, J - 1) * gstep);
  };

  // wave 0 stages group j+2 during X(j): branch-free loads at its start
  // (lane = row: its bin; lanes 0-2 / 3-5 env A's / B's action, old
  // probability and advantage, lanes 6 / 7 their items), the stores late
#if XH_4H_KL_TU
  struct Raw {
    int bi, rec;
    float q;     // the old distribution's entry of this lane's row and bin
    int ended;   // this lane's half, an open end row: step T - 1 ended
  };
  // row r of the learner's state matrix: its row of the [T+1][N] arrays and
  // of its old distribution, its kind (0 transition, 1 open end row, 2
  // terminal end row) and whether it counts (r is wave-uniform)
  auto kl_row = [&](int r, size_t &ti, size_t &qi, int &kind, bool &inr) {
    const int N = a.b.N;
    r = __builtin_amdgcn_readfirstlane(r);
    inr = r < nrows;
    if (r < NT) {
      ti = qi = (size_t)r;
      kind = 0;
    } else if (r < NT + N) {
      ti = (size_t)NT + (r - NT);
      qi = (size_t)(NT - N) + (r - NT);
      kind = 1;
    } else {
      const int jj = r - NT - N;
      const int te = jj < n_end ? __builtin_amdgcn_readfirstlane(a.end_list[jj]) : 0;
      ti = qi = (size_t)te;
      kind = 2;
    }
  };
#else
  struct Raw {
    int bi, rec;
  };
#endif
  // (every wave loads -- the loads are tiny -- and only wave 0 stores: no
  // branch around the loads, whose results then stay in flight until the
  // store; the byte is sign-extended there, and the record address is chosen
  // by selects, not branches)
#if XH_4H_KL_TU
  auto stage_load = [&](int j) {
    const int g = (int)gindex(j);
    size_t tA, qA, tB, qB;
    int kA, kB2;
    bool iA, iB;
    kl_row(2 * g, tA, qA, kA, iA);
    kl_row(2 * g + 1, tB, qB, kB2, iB);
    const bool eB = l >= 32;
    const size_t tl = eB ? tB : tA, ql = eB ? qB : qA;
    const int bins = (int)*reinterpret_cast<const unsigned char *>(a.b.bins + tl * 32 + (l & 31));
    // the record lanes: 0-2 row A's action, p_old, advantage (rows of the
    // [T][N] arrays: the old distribution's), 3-5 row B's, 6 / 7 the items
    const size_t ri = (l >= 3 && l != 6) ? qB : qA;
    const int k = l % 3;
    const unsigned long long p0 = (unsigned long long)(a.b.action + ri);
    const unsigned long long p1 = (unsigned long long)(a.b.pold + ri);
    const unsigned long long p2 = (unsigned long long)(a.adv + ri);
    const unsigned long long p3 = (unsigned long long)(a.b.items + ((l & 1) ? tB : tA) * 4);
    unsigned long long pa = k == 1 ? p1 : p2;
    pa = k == 0 ? p0 : pa;
    pa = l >= 6 ? p3 : pa;
    Raw r{bins, *reinterpret_cast<const int *>(pa), a.qold[ql * 32 + (l & 31)], 0};
    const bool open = eB ? kB2 == 1 : kA == 1;
    if (open) r.ended = a.b.done[ql];
    return r;
  };
#else
  auto stage_load = [&](int j) {
    const size_t g = gindex(j);
    int lo = l;
    asm volatile("" : "+v"(lo));
    const int bins = (int)*reinterpret_cast<const unsigned char *>(a.b.bins + g * 64 + lo);
    const size_t ti = 2 * g + (l >= 3 && l != 6);
    const int k = l % 3;
    const unsigned long long p0 = (unsigned long long)(a.b.action + ti);
    const unsigned long long p1 = (unsigned long long)(a.b.pold + ti);
    const unsigned long long p2 = (unsigned long long)(a.adv + ti);
    const unsigned long long p3 = (unsigned long long)(a.b.items + (2 * g + (l & 1)) * 4);
    unsigned long long pa = k == 1 ? p1 : p2;
    pa = k == 0 ? p0 : pa;
    pa = l >= 6 ? p3 : pa;
    return Raw{bins, *reinterpret_cast<const int *>(pa)};
  };
#endif
  // ---- prologue: every global load first (the scales' inputs, the small
  // parameters, this lane's W2 / W2' fragment values), then the scales
  // (every workgroup the same), then the f16 pairs of tile w
  const int rdb0 = rd_base(G, li);
  const Raw raw0 = stage_load(0), raw1 = stage_load(1);  // groups 0, 1's rows
  float4 wraw[2][2];   // W2[16 w + li][32 s + 8 G ..]
  float draw[2][8];    // W2[32 s + 8 G + j][16 w + li] * w3[32 s + 8 G + j]
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const float4 *src = reinterpret_cast<const float4 *>(
        P + PL.oW2() + (16 * w + li) * kH + 32 * s + 8 * G);
    wraw[s][0] = src[0];
    wraw[s][1] = src[1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = 32 * s + 8 * G + j, col = 16 * w + li;
      draw[s][j] = P[PL.oW2() + o * kH + col] * P[PL.ow3() + o];
    }
  }
  {
    float mw = 0.0f, md = 0.0f, mh = 0.0f;
    {
      // thread t: row t / 4 of W2, its quarter t % 4 (four 16-byte loads)
      const int o = tid >> 2;
      const float4 *src = reinterpret_cast<const float4 *>(P + PL.oW2() + o * kH + 16 * (tid & 3));
      const float w3o = P[PL.ow3() + o];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v4 = src[q];
        const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          mw = fmaxf(mw, fabsf(v[u]));
          md = fmaxf(md, fabsf(v[u] * w3o));
        }
      }
    }
    if (tid < kH) {
      const float wv = P[PL.oW1() + tid * kF0 + kD];
      const float w0v = P[PL.oW1() + tid * kF0];
      const float b1 = P[PL.ob1() + tid];
      const float ba = b1 + wv * ((float)a.env.item_a[0] / (float)kCapacity);
      const float bb = b1 + wv * ((float)a.env.item_b[0] / (float)kCapacity);
      mh = fabsf(w0v) + fmaxf(fabsf(ba), fabsf(bb));
      // the small parameters that need no scale
      lf[F_W1T + tid] = w0v;
      lf[F_B1F + tid] = ba;
      lf[F_B1F + kH + tid] = bb;
      lf[F_W3G + tid] = P[PL.ow3() + tid];
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      mw = fmaxf(mw, __shfl_xor(mw, o, kWave));
      md = fmaxf(md, __shfl_xor(md, o, kWave));
      mh = fmaxf(mh, __shfl_xor(mh, o, kWave));
    }
    if (l == 0) {
      lf[F_SC + w] = mw;
      lf[F_SC + 4 + w] = md;
      lf[F_SC + 8 + w] = mh;
    }
    __syncthreads();
    if (tid == 0) {
      float MW = 0.0f, MD = 0.0f, MH = 0.0f;
#pragma unroll
      for (int v = 0; v < kNW; ++v) {
        MW = fmaxf(MW, lf[F_SC + v]);
        MD = fmaxf(MD, lf[F_SC + 4 + v]);
        MH = fmaxf(MH, lf[F_SC + 8 + v]);
      }
      lf[F_SC + 12] = f16_scale_for(MW);  // S_W
      lf[F_SC + 13] = f16_scale_for(MD);  // S_D
      lf[F_SC + 14] = f16_scale_for(MH);  // S_H
      lf[F_B3] = P[PL.ob3()];
    }
    __syncthreads();
  }
  const float SW = lf[F_SC + 12], SD = lf[F_SC + 13], SH = lf[F_SC + 14];
  const float S2 = SW * SH;  // layer 2's pre-activations are in units of S2
  if (tid < kH) {
    lf[F_B2 + tid] = P[PL.ob2() + tid] * S2;
    lf[F_W3 + tid] = lf[F_W3G + tid] * (1.0f / S2);
  }
  f16x8 wl[2][2], wd[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const float v[8] = {wraw[s][0].x, wraw[s][0].y, wraw[s][0].z, wraw[s][0].w,
                        wraw[s][1].x, wraw[s][1].y, wraw[s][1].z, wraw[s][1].w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 x0, x1;
      split2h(v[j] * SW, x0, x1);
      wl[s][0][j] = x0;
      wl[s][1][j] = x1;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 x0, x1;
      split2h(draw[s][j] * SD, x0, x1);
      wd[s][0][j] = x0;
      wd[s][1][j] = x1;
    }
  }
  const int trm00 = trm_base(l, 0), trm10 = trm_base(l, 1);  // ^ 32 ot, + L_MASK
  const int stb0 = st_base(G, li) ^ (32 * w);  // + L_H1 / L_MASK + 4096 rt
  const int fo = 16 * w + 4 * G;  // this lane's 4 features in the C layout
  float *gw = lf + F_GW + 64 * w;  // this wave's copies of the rows' g
  float *gp = lf + F_GP + 64 * w;

  f32x4 accW2[4];
#pragma unroll
  for (int ot = 0; ot < 4; ++ot)
#pragma unroll
    for (int j = 0; j < 4; ++j) accW2[ot][j] = 0.0f;
  float accW3[4] = {0.0f, 0.0f, 0.0f, 0.0f}, accB2[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float accB3 = 0.0f, w0 = 0.0f, sa = 0.0f, sb = 0.0f;
#if XH_4H_KL_TU
  double kl_acc = 0.0;  // sum of KL(q || p) over this wave's rows
#endif

#if XH_4H_KL_TU
  auto stage_store = [&](const Raw &r, int s, int j) {
    const int g = (int)gindex(j);
    size_t tA, qA, tB, qB;
    int kA, kB2;
    bool iA, iB;
    kl_row(2 * g, tA, qA, kA, iA);
    kl_row(2 * g + 1, tB, qB, kB2, iB);
    const bool eB = l >= 32;
    // the terminal view: the chosen bin without the item (rl.h:336-343)
    const int cA = __builtin_amdgcn_readlane(r.rec, 0), cB = __builtin_amdgcn_readlane(r.rec, 3);
    const int iA8 = __builtin_amdgcn_readlane(r.rec, 6), iB8 = __builtin_amdgcn_readlane(r.rec, 7);
    const bool sub = (eB ? kB2 : kA) == 2 && (l & 31) == (eB ? cB : cA);
    const int bv = (signed char)(r.bi & 0xff) - (sub ? (signed char)((eB ? iB8 : iA8) & 0xff) : 0);
    const float x = (float)bv / (float)kCapacity;
    lf[F_Q + s * 64 + l] = r.q;
    // each half's validity (its own lanes' r.ended)
    const int endA = __builtin_amdgcn_readlane(r.ended, 0), endB = __builtin_amdgcn_readlane(r.ended, 32);
    const bool vA = iA && (kA == 0 || (kA == 1 ? endA == 0 : true));
    const bool vB = iB && (kB2 == 0 || (kB2 == 1 ? endB == 0 : true));
#else
  auto stage_store = [&](const Raw &r, int s) {
    const float x = (float)(signed char)(r.bi & 0xff) / (float)kCapacity;
#endif
    lf[F_X + s * 64 + l] = x;
    lf[F_XP + s * 64 + 4 * (l & 15) + (l >> 4)] = x;
    const int itA = __builtin_amdgcn_readlane(r.rec, 6);
    const int itB = __builtin_amdgcn_readlane(r.rec, 7);
    if (l == 0) {
      lf[F_IT + 2 * s] = (signed char)(itA & 0xff) == a.env.item_a[0] ? 1.0f : 0.0f;
      lf[F_IT + 2 * s + 1] = (signed char)(itB & 0xff) == a.env.item_a[0] ? 1.0f : 0.0f;
    }
#if XH_4H_KL_TU
    // the records: action and advantage of a transition, 0 for end rows;
    // slots 3 / 7 whether the row counts
    if (l == 0 || l == 2) lf[F_REC + 8 * s + l] = kA == 0 ? __int_as_float(r.rec) : 0.0f;
    if (l == 3 || l == 5)
      lf[F_REC + 8 * s + 4 + l - 3] = kB2 == 0 ? __int_as_float(r.rec) : 0.0f;
    if (l == 6) lf[F_REC + 8 * s + 3] = vA ? 1.0f : 0.0f;
    if (l == 7) lf[F_REC + 8 * s + 7] = vB ? 1.0f : 0.0f;
#else
    if (l < 6) lf[F_REC + 8 * s + (l >= 3 ? 4 + l - 3 : l)] = __int_as_float(r.rec);
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
  // the layer-1 bias row (item folded in) of env e of the group in slot s
  auto b1row = [&](int s, int e) {
    const bool ia = __builtin_amdgcn_readfirstlane(__float_as_int(lf[F_IT + 2 * s + e])) != 0;
    return lf + F_B1F + (ia ? 0 : kH);
  };
  // layer 1 (C layout) of the group in slot s, all four r-tiles -> H1 image
  auto layer1_all = [&](int s, int stb) {
    const f32x4 wa = lds4v(lf + F_W1T + fo);
    const f32x4 bbA = lds4v(b1row(s, 0) + fo), bbB = lds4v(b1row(s, 1) + fo);
    const f32x4 x0 = lds4v(lf + F_XP + s * 64 + 4 * li);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      const f32x4 &bb = rt < 2 ? bbA : bbB;
      f32x4 t;
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = relu(fmaf(x0[rt], wa[j], bb[j]));
      store_h1(t, stb, rt);
    }
  };
  // layer 2 of the group whose H1 is in the image: 8 steps of 3 f16 MFMAs,
  // task(k) after each MFMA (k = 0 .. 23)
  auto layer2 = [&](int rdb, f32x4 (&pre)[4], auto &&task) {
    const f32x4 b2 = lds4v(lf + F_B2 + fo);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) pre[rt] = b2;
    f16x8 b_c[2], b_n[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) b_c[p] = ld8h(rdb + L_H1 + p * kImg);
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const int s = st >> 2, rt = st & 3;
      if (st + 1 < 8) {
        const int s1 = (st + 1) >> 2, r1 = (st + 1) & 3;
#pragma unroll
        for (int p = 0; p < 2; ++p)
          b_n[p] = ld8h((rdb ^ (64 * s1)) + L_H1 + p * kImg + 4096 * r1);
      }
      FENCE();
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
  // (lane group G ends with r-tile G's sum: sum_groups_t)
  auto partials = [&](const f32x4 (&pre)[4], const f32x4 &w3, int zs) {
    float zp[4];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      zp[rt] = relu(pre[rt][0]) * w3[0];
      zp[rt] = fmaf(relu(pre[rt][1]), w3[1], zp[rt]);
      zp[rt] = fmaf(relu(pre[rt][2]), w3[2], zp[rt]);
      zp[rt] = fmaf(relu(pre[rt][3]), w3[3], zp[rt]);
    }
    lf[F_Z + zs * 256 + (16 * G + li) * kNW + w] = sum_groups_t(zp);
  };
  auto no_task = [](int) {};

  // ---- pipeline prologue: groups 0 and 1 staged, layer 1 and layer 2 of
  // group 0 (its partial logits), layer 1 of group 1
  f32x4 pre_cur[4];
  Raw raw = {0, 0};
  if (w == 0) {
    stage_store(raw0, 0 KLTU(, 0));
    stage_store(raw1, 1 KLTU(, 1));
  }
  __syncthreads();
  layer1_all(0, stb0);
  __syncthreads();
  layer2(rdb0, pre_cur, no_task);
  partials(pre_cur, lds4v(lf + F_W3 + fo), 0);
  __syncthreads();
  layer1_all(1, stb0);
  __syncthreads();
  S4H_STAMP(a, kKG, w, l, 1);

  for (int j = 0; j < J; ++j) {
    [[maybe_unused]] const int gj = j < kKG ? j : kTraceGroups;  // stamped groups
    S4H_STAMP(a, gj, w, l, 0);
    const int cs = j % 3, ns = (j + 2) % 3;  // slots of groups j and j + 2
    int rdb = rdb0, trm0 = trm00, trm1 = trm10, stb = stb0;
    asm volatile("" : "+v"(rdb), "+v"(trm0), "+v"(trm1), "+v"(stb), "+s"(gstep));
    raw = stage_load(j + 2);
    const float *xim = lf + F_X + cs * 64;
    const float w1a = lf[F_W1T + 16 * w + li];  // T layout: feature 16 w + li

    // ================= X(j): layer 2 of group j+1 with group j's VALU ====
    const f32x4 z4 = lds4v(lf + F_Z + (j & 1) * 256 + kNW * l);
    const float b3 = lf[F_B3];
    const f32x4 recA = lds4v(lf + F_REC + 8 * cs), recB = lds4v(lf + F_REC + 8 * cs + 4);
    const float itA = lf[F_IT + 2 * cs], itB = lf[F_IT + 2 * cs + 1];
#if XH_4H_KL_TU
    const float qv = lf[F_Q + cs * 64 + l];
    float kp = 0.0f, kg = 0.0f;
#endif
    f32x4 gx0[2];
    float ex = 0.0f, se = 0.0f, gz = 0.0f;
    f32x4 gr4, ggk[2], hT[2];
    bf16x8 bq0[3];
    bool iaA = false, iaB = false;
    float b1tA = 0.0f, b1tB = 0.0f;
    f32x4 w3;
    auto xtask = [&](int k) {
      if (k == 0) {
        ex = __expf(((z4[0] + z4[1]) + (z4[2] + z4[3])) + b3);
      } else if (k == 1) {
        se = seg_sum<32>(ex);  // per env (32-lane segment)
#if XH_4H_KL_TU
      } else if (k == 2) {
        // kl_regulated_loss (policy_gradient.h:41-85) through
        // softmax_layer::backward (the Jacobian's sum in the next slot), per
        // 32-lane row; the KL sum on one wave per group, in turn
        const int cA = __builtin_amdgcn_readfirstlane(__float_as_int(recA[0]));
        const int cB = __builtin_amdgcn_readfirstlane(__float_as_int(recB[0]));
        const bool eB = l >= 32;
        const int c = eB ? cB : cA;
        const float Ac = __int_as_float(__builtin_amdgcn_readfirstlane(
                             __float_as_int(recA[2]))) * (eB ? 0.0f : 1.0f) +
                         __int_as_float(__builtin_amdgcn_readfirstlane(
                             __float_as_int(recB[2]))) * (eB ? 1.0f : 0.0f);
        kp = ex * __builtin_amdgcn_rcpf(se);
        kg = fmaf(beta, kp - qv, kp * Ac);
        if ((l & 31) == c) kg -= Ac;
        const bool vA = __builtin_amdgcn_readfirstlane(__float_as_int(recA[3])) != 0;
        const bool vB = __builtin_amdgcn_readfirstlane(__float_as_int(recB[3])) != 0;
        if ((j & 3) == w && (eB ? vB : vA)) kl_acc += (double)(qv * logf(qv / kp));
#else
      } else if (k == 2) {
        const int cA = __builtin_amdgcn_readfirstlane(__float_as_int(recA[0]));
        const int cB = __builtin_amdgcn_readfirstlane(__float_as_int(recB[0]));
        const bool eB = l >= 32;
        const float p = ex * __builtin_amdgcn_rcpf(se);
        const float pcA = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), cA));
        const float pcB = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), 32 + cB));
        const int c = eB ? cB : cA;
        const float pc = eB ? pcB : pcA;
        const float Ac = __int_as_float(__builtin_amdgcn_readfirstlane(
                             __float_as_int(recA[2]))) * (eB ? 0.0f : 1.0f) +
                         __int_as_float(__builtin_amdgcn_readfirstlane(
                             __float_as_int(recB[2]))) * (eB ? 1.0f : 0.0f);
        if (a.algo == kPPO) {
          // clipped_gradient (rl.h:54-74) through softmax_layer::backward
          const float poA = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(recA[1])));
          const float poB = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(recB[1])));
          const float po = eB ? poB : poA;
          const float ratio = pc * __builtin_amdgcn_rcpf(po);
          float ce = a.clip_eps;
          asm volatile("" : "+s"(ce));
          const float clipped = fminf(fmaxf(ratio, 1.0f - ce), 1.0f + ce);
          const float ig = fminf(clipped * Ac, ratio * Ac) * -1.0f;
          const float gc = ig * __builtin_amdgcn_rcpf(pc);
          const float lin = (l & 31) == c ? p : 0.0f;
          gz = (lin - p * pc) * gc;
        } else {
          // softmax_gradient_log (rl.h:45-52) through softmax-xent
          gz = p * Ac;
          if ((l & 31) == c) gz -= Ac;
        }
#endif
      } else if (k == 3) {
#if XH_4H_KL_TU
        {
          const float sgv = seg_sum<32>(kp * kg);
          const bool vA = __builtin_amdgcn_readfirstlane(__float_as_int(recA[3])) != 0;
          const bool vB = __builtin_amdgcn_readfirstlane(__float_as_int(recB[3])) != 0;
          gz = (l >= 32 ? vB : vA) ? kp * (kg - sgv) : 0.0f;
        }
#endif
        gw[l] = gz;
        gp[4 * (l & 15) + (l >> 4)] = gz;
        accB3 += gz;  // wave 0's is written out
        iaA = __builtin_amdgcn_readfirstlane(__float_as_int(itA)) != 0;
        iaB = __builtin_amdgcn_readfirstlane(__float_as_int(itB)) != 0;
        b1tA = lf[F_B1F + (iaA ? 0 : kH) + 16 * w + li];
        b1tB = lf[F_B1F + (iaB ? 0 : kH) + 16 * w + li];
        // the rows of K-step 0 (env A; T layout)
#pragma unroll
        for (int h = 0; h < 2; ++h) gx0[h] = lds4v(xim + 16 * h + 4 * G);
      } else if (k == 4) {
        gr4 = lds4v(gp + 4 * li);  // g of rows 16 rt + li
#pragma unroll
        for (int h = 0; h < 2; ++h) ggk[h] = lds4v(gw + 16 * h + 4 * G);
      } else if (k == 6 || k == 7) {
        const int h = k - 6;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) hT[h][jj] = relu(fmaf(gx0[h][jj], w1a, b1tA));
      } else if (k >= 8 && k < 12) {
        // r-tile rt: the relu masks -> the mask image (0 / 0x4000: 2.0 as bf16
        // for dW2 and as f16 for dH1; the factor 2 is taken back exactly at
        // the write-out), dW3 / db2 (pre-activations in units of S2) from the
        // same mask bits
        const int rt = k - 8;
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        unsigned m[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) m[jj] = (unsigned)relu_bit(pre_cur[rt][jj]);
        // times the 2.0 bits by the full-rate 24-bit multiply (the 32-bit one
        // is quarter rate)
        const u32x2 mm = {(unsigned)__umul24(m[0] | (m[1] << 16), 0x4000u),
                          (unsigned)__umul24(m[2] | (m[3] << 16), 0x4000u)};
        st4(stb + L_MASK + 4096 * rt, __builtin_bit_cast(bf16x4, mm));
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float v = pre_cur[rt][jj];
          const float gm = gr4[rt] * (float)m[jj];
          accW3[jj] = fmaf(gm, v, accW3[jj]);
          accB2[jj] += gm;
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
      } else if (k == 20) {
        w3 = lds4v(lf + F_W3 + fo);  // for the partial logits after layer 2
      } else if (k == 22) {
        if (w == 0) stage_store(raw, ns KLTU(, j + 2));  // group j+2's rows
      }
    };
    f32x4 pre_nx[4];
    layer2(rdb, pre_nx, xtask);
    S4H_STAMP(a, gj, w, l, 1);
    partials(pre_nx, w3, (j + 1) & 1);
    S4H_STAMP(a, gj, w, l, 2);
    __syncthreads();
    S4H_STAMP(a, gj, w, l, 3);

    // ================= Y(j): dW2 / dH1 of group j with VALU of j, j+2 =====
    // 16 blocks: b < 4 dW2 of K-step 0 (ot = b), three bf16 MFMAs; 4 <= b <
    // 12 dH1, two f16 MFMAs (rt = (b - 4) / 2, s = (b - 4) % 2); b >= 12 dW2
    // of K-step 1 (its operand is built in blocks 2-5); operands one block
    // ahead
    {
      float sgA = 0.0f, sgB = 0.0f;
      bf16x8 bq1[3];
      f32x4 rx0[2], rgg[2], hT1[2];
      f32x4 wa, bbA, bbB, xp0, t1;
      float itnA = 0.0f, itnB = 0.0f;
      f32x4 dx0, dgg;
      f32x4 dh[2];
      // blocks alternate: even bb_ dW2 block d = bb_ / 2 (K-step d / 4,
      // o-tile d % 4), odd bb_ dH1 block h = bb_ / 2 (r-tile h / 2, K-slice
      // h % 2)
      auto load_ops = [&](int bb_, bf16x8 &A) {
        const int d = bb_ >> 1;
        if ((bb_ & 1) == 0) {
          const int ks = d >> 2, ot = d & 3;
          A = ldtr((trm0 ^ (32 * ot)) + L_MASK + 8192 * ks,
                   (trm1 ^ (32 * ot)) + L_MASK + 8192 * ks);
        } else {
          const int rt = d >> 1, s = d & 1;
          A = ld8((rdb ^ (64 * s)) + L_MASK + 4096 * rt);  // read as f16
        }
      };
      // dW1 / db1 / item sums of value jj of r-tile rt (T layout; r-tiles 0,
      // 1 env A, 2, 3 env B)
      auto dw1 = [&](int jj, int rt) {
        const int q = rt & 1;
        // relu'(layer 1) from the T-layout H1 values of g (x) H1 (the same
        // rows: hT env A's r-tiles 0, 1, hT1 env B's 2, 3)
        const float hv = rt == 0 ? hT[0][jj] : rt == 1 ? hT[1][jj] : rt == 2 ? hT1[0][jj] : hT1[1][jj];
        const float d = hv > 0.0f ? dh[q][jj] * dgg[jj] : 0.0f;
        if (rt < 2)
          sgA += d;
        else
          sgB += d;
        w0 = fmaf(d, dx0[jj], w0);
      };
      auto ytask = [&](int b) {
        if (b == 0) {
          // rows of K-step 1 (env B; T layout) and their g; group j+2's items
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int r0 = 32 + 16 * h + 4 * G;
            rx0[h] = lds4v(xim + r0);
            rgg[h] = lds4v(gw + r0);
          }
          itnA = lf[F_IT + 2 * ns];
          itnB = lf[F_IT + 2 * ns + 1];
        } else if (b == 1) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) hT1[h][jj] = relu(fmaf(rx0[h][jj], w1a, b1tB));
        } else if (b >= 2 && b < 6) {
          // g (x) H1 of K-step 1, two values per slot
          const int h = (b - 2) >> 1, j0 = 2 * ((b - 2) & 1);
#pragma unroll
          for (int jj = j0; jj < j0 + 2; ++jj) {
            __bf16 p0, p1, p2;
            split3(hT1[h][jj] * rgg[h][jj], p0, p1, p2);
            bq1[0][4 * h + jj] = p0;
            bq1[1][4 * h + jj] = p1;
            bq1[2][4 * h + jj] = p2;
          }
          if (b == 2) {
            wa = lds4v(lf + F_W1T + fo);
            xp0 = lds4v(lf + F_XP + ns * 64 + 4 * li);
          } else if (b == 3) {
            const bool ia = __builtin_amdgcn_readfirstlane(__float_as_int(itnA)) != 0;
            const bool ib = __builtin_amdgcn_readfirstlane(__float_as_int(itnB)) != 0;
            bbA = lds4v(lf + F_B1F + (ia ? 0 : kH) + fo);
            bbB = lds4v(lf + F_B1F + (ib ? 0 : kH) + fo);
          }
        }
        if (b >= 6 && b < 14) {
          // layer 1 of group j+2, r-tile (b - 6) / 2: values, then the stores
          const int rt = (b - 6) >> 1;
          if (((b - 6) & 1) == 0) {
            const f32x4 &bb = rt < 2 ? bbA : bbB;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) t1[jj] = relu(fmaf(xp0[rt], wa[jj], bb[jj]));
          } else {
            store_h1(t1, stb, rt);
          }
        }
        if (b & 1) {
          // dW1 of the previous r-tile (two values per slot), the next rows
          const int rt = (b >> 1) >> 1, s = (b >> 1) & 1;
          if (rt > 0) {
            dw1(2 * s, rt - 1);
            dw1(2 * s + 1, rt - 1);
          }
          if (s == 1) {
            const int r0 = 16 * rt + 4 * G;
            dx0 = lds4v(xim + r0);
            dgg = lds4v(gw + r0);
          }
        }
      };
      bf16x8 A_c, A_n;
      load_ops(0, A_c);
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        if (b + 1 < 16) load_ops(b + 1, A_n);
        FENCE();
        if ((b & 1) == 0) {
          const int ot = (b >> 1) & 3;
          const bf16x8(&bq)[3] = (b >> 1) < 4 ? bq0 : bq1;
          accW2[ot] = mfma16(A_c, bq[2], accW2[ot]);
          accW2[ot] = mfma16(A_c, bq[1], accW2[ot]);
          accW2[ot] = mfma16(A_c, bq[0], accW2[ot]);
        } else {
          const int rt = (b >> 1) >> 1, s = (b >> 1) & 1, q = rt & 1;
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
      S4H_STAMP(a, gj, w, l, 4);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) dw1(jj, 3);  // the last r-tile's
      if (iaA)
        sa += sgA;
      else
        sb += sgA;
      if (iaB)
        sa += sgB;
      else
        sb += sgB;
    }
    S4H_STAMP(a, gj, w, l, 5);
    __syncthreads();
    S4H_STAMP(a, gj, w, l, 6);
    S4H_STAMP(a, gj, w, l, 7);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) pre_cur[rt] = pre_nx[rt];
  }
  S4H_STAMP(a, kKG, w, l, 2);

#if XH_4H_KL_TU
  {
    // the workgroup's KL sum (the loop's last barrier is behind: F_Z is free)
    double dv = kl_acc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) dv += __shfl_xor(dv, o, kWave);
    double *kd = reinterpret_cast<double *>(lf + F_Z);
    if (l == 0) kd[w] = dv;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
#pragma unroll
      for (int v4 = 0; v4 < kNW; ++v4) t += kd[v4];
      a.kl_part[blockIdx.x] = t;
    }
  }
#endif

  // ---------------------------------------------------- slab write-out ----
  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
  const float *w3g = lf + F_W3G;
#pragma unroll
  for (int ot = 0; ot < 4; ++ot)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = 16 * ot + 4 * G + j;
      slab[PL.oW2() + o * kH + 16 * w + li] = (accW2[ot][j] * 0.5f) * w3g[o];
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float s3 = seg_sum<16>(accW3[j]);
    const float s2 = seg_sum<16>(accB2[j]);
    const int o = 16 * w + 4 * G + j;
    if (li == 0) {
      slab[PL.ow3() + o] = s3 * (1.0f / S2);
      slab[PL.ob2() + o] = s2 * w3g[o];
    }
  }
  if (w == 0) {
    const float v3 = seg_sum<64>(accB3);
    if (l == 0) slab[PL.ob3()] = v3;
  }
  {
    float tw0 = w0 + __shfl_xor(w0, 16, kWave);
    float va = sa + __shfl_xor(sa, 16, kWave);
    float vb = sb + __shfl_xor(sb, 16, kWave);
    tw0 += __shfl_xor(tw0, 32, kWave);
    va += __shfl_xor(va, 32, kWave);
    vb += __shfl_xor(vb, 32, kWave);
    // dH1 was in units of S_D
    tw0 *= 0.5f / SD;  // (and the masks were 2.0)
    va *= 0.5f / SD;
    vb *= 0.5f / SD;
    if (G == 0) {
      const int i = 16 * w + li;
      slab[PL.oW1() + i * kF0 + 0] = tw0;
      slab[PL.oW1() + i * kF0 + kD] = va * ((float)a.env.item_a[0] / (float)kCapacity) +
                                      vb * ((float)a.env.item_b[0] / (float)kCapacity);
      slab[PL.ob1() + i] = va + vb;
    }
  }
  S4H_STAMP(a, kKG, w, l, 3);
}
#undef FENCE

}  // namespace s4h

#if XH_4H_KL_TU
hipError_t launch_policy_train_split4h_kl(const PolicyTrainArgs &a, int grid,
                                          hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s4h::policy_train_split4h_kl_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s4h::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s4h::policy_train_split4h_kl_kernel, dim3(grid),
                     dim3(s4h::kThreads), s4h::kLds, s, a);
  return hipGetLastError();
}
#else
hipError_t launch_policy_train_split4h(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s) {
  if (a.algo == kKLPPO) return launch_policy_train_split4h_kl(a, grid, s);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)s4h::policy_train_split4h_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s4h::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(s4h::policy_train_split4h_kernel, dim3(grid),
                     dim3(s4h::kThreads), s4h::kLds, s, a);
  return hipGetLastError();
}
#endif

}  // namespace xh
