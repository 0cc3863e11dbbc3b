// policy_spec8_kernels.hip -- the PPO / actor-critic train epoch of the
// 64-bin 2-D [128,128] policy (BASELINE configs 3 and 4) with WAVE
// SPECIALISATION: of the workgroup's 8 waves, waves 0-3 ("matrix waves")
// issue the MFMAs of layer 2 and dW2, waves 4-7 ("vector waves") the VALU
// work of layer 1, g (x) H1, dW1 and the MFMAs of dH1.  Waves w and w + 4
// share a SIMD (a workgroup's waves go round the SIMDs with period 4), so
// every SIMD pairs one MFMA-heavy wave with one VALU-heavy wave.
//
// Why: in policy_train_split8wh_kernel both waves of a SIMD run the same
// phases, so the VALU of one phase cannot hide under the MFMAs of the other
// (about 10k cycles per 64-row group against 4096 of matrix pipe).  An
// MFMA-only wave and a VALU-only wave on one SIMD overlap almost fully
// (tools/probes/specialize_probe.hip, profiles/r05b_probe_specialize.txt:
// 32 v_mfma_f32_32x32x16 + 128 v_fma_f32 per iteration 1167 cycles against
// 1066 / 770 alone; 256 v_fma_f32: 1612 against 1066 / 1376), with the 32x32x16
// shape (16x16x32: 1812).
//
// Numerics as policy_train_split8wh_kernel: layer 2 and
// dH1 on f16 pairs scaled by powers of two (S_W W2, S_D W2' = S_D diag(w3)
// W2, S_H H1; three / two f16 MFMAs per K slice), dW2 on the exact bf16
// three-part split of S_H g (x) H1 against the 0/1 relu mask; only the MFMA
// shape (32x32x16) and so the f32 accumulation order differ.
//
// Per 64-row group g (one transition's 64 bins), the work by role:
//   vector  L1(g)   layer 1 -> H1 image (f16 pair, [i][r]), H1 kept in registers
//   matrix  L2(g)   layer 2 (48 MFMAs per wave: its 32 outputs o x 64 rows)
//                   -> partial logits over its o
//   matrix  SM(g)   softmax + loss gradient g of the 64 rows (every matrix
//                   wave, from the four partial logits), dW3 / db2 sums,
//                   relu masks -> the mask image ([r][o], 0 / 2.0: bf16 and
//                   f16 alike)
//   vector  DH(g)   dH1 = M (S_D W2') (32 MFMAs: its 32 features i), dW1 /
//                   db1 / item sums; g (x) H1 -> the split image ([i][r])
//   matrix  DW(g)   dW2 += M^T (g (x) H1) (48 MFMAs: its 32 features i)
// pipelined two phases per group, each closed by a barrier:
//   A(j): matrix L2(j+1) + partial logits    vector DH(j) + g (x) H1(j)
//   B(j): matrix SM(j+1) + DW(j)             vector dW1(j) + L1(j+2)
// (both phases carry 80 / 48 MFMAs per SIMD beside the vector wave's VALU).
// The two roles run separate code paths with the same barrier sequence, so
// the compiler allocates each path's registers alone (matrix: W2 pair 64,
// dW2 accumulators 64, layer-2 accumulators 32, dW3 / db2 sums 32; vector:
// W2' pair 64, dH1 accumulators 32, two groups' H1 64).
//
// LDS (dynamic, base 0): g (x) H1 three bf16 parts [128 i][64 r] (48 KB), H1
// two f16 parts [64 r][128 i] (32 KB), relu masks [64 r][128 o] (0x4000 = 2.0
// as bf16 and as f16)
// in two slots (32 KB apart, 16 KB used), then f32 vectors; image layout
// spec8_layout.h.
#include <cstdlib>
#include <type_traits>

#include "spec8_layout.h"
#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

// XH_SP8_ONLY (register-use study builds only): 1 / 2 compile every wave as
// a matrix / vector wave
#ifndef XH_SP8_ONLY
#define XH_SP8_ONLY 0
#endif
// XH_SP8_ABLATE (timing-study variant builds only, wrong results by design):
// bit 0 matrix waves skip their loop work, 1 vector waves skip theirs, 2
// vector skip DH / g (x) H1 (phase A), 3 vector skip layer 1, 4 matrix skip
// dW2 and its slot tasks (softmax, dW3 / db2, masks: phase B), 5 matrix
// skip layer 2 (phase A), 6 vector skip dW1 (barriers and staging kept)
#ifndef XH_SP8_ABLATE
#define XH_SP8_ABLATE 0
#endif
#define SP8_RUN(bits) ((XH_SP8_ABLATE & (bits)) == 0)
// XH_SP8_PRIO (A/B builds): s_setprio of the matrix (bits 0-1) and vector
// (bits 2-3) waves for their loops
#ifndef XH_SP8_PRIO
#define XH_SP8_PRIO 0
#endif
// XH_SP8_VBF (A/B builds): 0 lets the compiler schedule the vector waves'
// phase-B blocks (dW1, layer 1) across block boundaries
// XH_SP8_GH2 (A/B builds): 1 splits a block's two pairs in one MFMA slot
// (two independent chains interleaved) and stores in the next
// XH_SP8_VFIRST: the vector role to the first (older) wave on each SIMD, the
// matrix role to the second -- the older wave wins VALU issue arbitration and
// the vector waves carry the VALU (policy_train phase 7.29 -> 7.27 ms per
// iteration over three paired rounds); 0 = the matrix role first
#ifndef XH_SP8_VFIRST
#define XH_SP8_VFIRST 1
#endif
// XH_SP8_KL_TU=1 (policy_spec8_kl_kernels.o): the KL-PPO build,
// policy_train_spec8_kl_kernel -- kl_ppo_learner's epoch
// (policy_gradient.h:310-335) over every row of its state matrix as
// policy_train_split8wh_kl_kernel: the T N transitions, the open
// trajectories' end rows (slot T, q of step T - 1, valid unless step T - 1
// ended), the terminal end rows E_t of end_list (the chosen bin with the
// item taken back out, rl.h:336-343); end rows carry A = 0; the loss head is
// kl_regulated_loss (policy_gradient.h:41-85) through softmax_layer::backward
// (nn.h:393-417), and each workgroup sums KL(q || p) over its valid rows into
// kl_part.  Preprocessor blocks, so the PPO object compiles from exactly its
// measured source.
#ifndef XH_SP8_KL_TU
#define XH_SP8_KL_TU 0
#endif
#if XH_SP8_KL_TU
#define SP8KL(...) __VA_ARGS__
#else
#define SP8KL(...)
#endif
#ifndef XH_SP8_GH2
#define XH_SP8_GH2 0
#endif
// XH_SP8_DHI / XH_SP8_L2I (A/B builds): dH1's (vector) / layer 2's (matrix)
// 16 steps in the order (t = st & 1, ks = st >> 1), alternating the two
// r-tiles' accumulators, instead of all of r-tile 0's steps first (a
// dependent MFMA waits for its predecessor's result; the per-accumulator
// order of the products is unchanged: bit-identical)
#ifndef XH_SP8_DHI
#define XH_SP8_DHI 0
#endif
#ifndef XH_SP8_L2I
#define XH_SP8_L2I 0
#endif
#ifndef XH_SP8_VBF
#define XH_SP8_VBF 0
#endif
// XH_SP8_VAF (A/B builds): 0 lets the compiler schedule the vector waves'
// phase-A slots (g (x) H1) across the dH1 MFMAs
#ifndef XH_SP8_VAF
#define XH_SP8_VAF 1
#endif
#define VAFENCE()                                 \
  do {                                            \
    if (XH_SP8_VAF) __builtin_amdgcn_sched_barrier(0); \
  } while (0)
#define VBFENCE()                                 \
  do {                                            \
    if (XH_SP8_VBF) __builtin_amdgcn_sched_barrier(0); \
  } while (0)
namespace xh {
namespace sp8 {

constexpr int kB = 64, kD = 2, kF0 = 2 * kD, kH = 128;
constexpr int kThreads = 512;
constexpr int kImg = 16384;        // one [128][64] / [64][128] 16-bit image
constexpr int L_GH = 0;            // g (x) H1: hi, mid, lo
constexpr int L_H1 = 3 * kImg;     // H1: hi, lo
constexpr int L_MK = 5 * kImg;     // masks: slot s at + 2 kImg s (the second kImg unused)
constexpr int L_F = 9 * kImg;
constexpr int F_B2 = 0;            // [128] b2 S2 (layer 2's accumulator input)
constexpr int F_W3 = F_B2 + kH;    // [128] w3 / S2 (unscales the partial logits)
constexpr int F_Z = F_W3 + kH;     // [64 rows][4 matrix waves] partial logits
constexpr int F_G = F_Z + 256;     // [2 parities][3][64] g, g x0, g x1 of a group
constexpr int F_X = F_G + 384;     // [4 slots][2 dims][64 rows] bins / 8
constexpr int F_REC = F_X + 512;   // [4 slots][action, pold, adv, item is item_a]
constexpr int F_SC = F_REC + 16;   // [16] scale reduction scratch, the scales
constexpr int F_B3 = F_SC + 16;    // [4]
constexpr int F_DB3 = F_B3 + 4;    // [32] matrix wave 0's db3 sums, per lane
constexpr int F_SIMD = F_DB3 + 32; // [8] the SIMD each wave runs on (ints)
#if XH_SP8_KL_TU
constexpr int F_Q = F_SIMD + 8;    // [4 slots][64 bins] old distribution q
constexpr int F_KL = F_Q + 256;    // [4 matrix waves][32 lanes] KL sums (doubles)
constexpr int F_END = F_KL + 256;
#else
constexpr int F_END = F_SIMD + 8;
#endif
constexpr size_t kLds = L_F + sizeof(float) * F_END;
static_assert(kLds <= 160 * 1024, "LDS");
#define FENCE() __builtin_amdgcn_sched_barrier(0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x8 lbf16x8;
typedef __attribute__((address_space(3))) bf16x4 lbf16x4;
typedef __attribute__((address_space(3))) f16x8 lf16x8;
typedef __attribute__((address_space(3))) f16x4 lf16x4;
typedef __attribute__((address_space(3))) s16x4 ls16x4;

__device__ __forceinline__ bf16x8 ld8(int off) {
  return *(const lbf16x8 *)(size_t)(unsigned)off;
}
__device__ __forceinline__ f16x8 ld8h(int off) {
  return *(const lf16x8 *)(size_t)(unsigned)off;
}
__device__ __forceinline__ void st4(int off, bf16x4 v) {
  *(lbf16x4 *)(size_t)(unsigned)off = v;
}
__device__ __forceinline__ void st8h(int off, f16x8 v) {
  *(lf16x8 *)(size_t)(unsigned)off = v;
}
__device__ __forceinline__ void st4h(int off, f16x4 v) {
  *(lf16x4 *)(size_t)(unsigned)off = v;
}
// two ds_read_b64_tr_b16 (EXEC full): elements 0-3 from o0, 4-7 from o1
__device__ __forceinline__ bf16x8 ldtr(int o0, int o1) {
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ls16x4 *)(size_t)(unsigned)o0);
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ls16x4 *)(size_t)(unsigned)o1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ f16x8 ldtrh(int o0, int o1) {
  return __builtin_bit_cast(f16x8, ldtr(o0, o1));
}
__device__ __forceinline__ f32x4 lds4v(const float *p) {
  return *reinterpret_cast<const f32x4 *>(p);
}
__device__ __forceinline__ float relu(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}
// a lane base that the compiler must not re-derive (so that image offsets
// below 64 KB fold into the ds instructions' immediates)
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
template <int V>
using Par = std::integral_constant<int, V>;
// v + the other lane half's v, the same bits in both halves
__device__ __forceinline__ float add_halves(float v) {
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v),
                                                  false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

#if XH_SP8_KL_TU
__global__ __launch_bounds__(kThreads, 2) void policy_train_spec8_kl_kernel(PolicyTrainArgs a) {
#else
__global__ __launch_bounds__(kThreads, 2) void policy_train_spec8_kernel(PolicyTrainArgs a) {
#endif
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH, kH};
  const float *P = a.params;
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int l = tid & 63, h = l >> 5, l31 = l & 31;
#if XH_SP8_KL_TU
  const int NT = a.b.T * a.b.N;
  const int n_end = *a.n_end;
  const int ngroups = NT + a.b.N + n_end;
  const float beta = *a.beta;
#else
  const int ngroups = a.b.T * a.b.N;
#endif
  // this workgroup's groups g_j = b0 + j gridDim.x, j < J (XCD-aware b0 as
  // policy_train_split8wh_kernel); look-ahead indices past the end are
  // clamped to the last group and their results discarded
  const int b0 = ((int)gridDim.x & 7) == 0
                     ? ((int)blockIdx.x & 7) * ((int)gridDim.x >> 3) + ((int)blockIdx.x >> 3)
                     : (int)blockIdx.x;
  const int J = b0 < ngroups ? (ngroups - b0 + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  if (J == 0) return;  // uniform over the workgroup
  const int gstep = (int)gridDim.x;
  auto tindex = [&](int j) { return (size_t)(b0 + min(j, J - 1) * gstep); };

  // ---- prologue: the scales (maxima over the parameters, every workgroup
  // the same; as policy_train_split8wh_kernel), small parameters into LDS
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
    __syncthreads();
    float MW = 0.0f, MD = 0.0f;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      MW = fmaxf(MW, lf[F_SC + v]);
      MD = fmaxf(MD, lf[F_SC + 8 + v]);
    }
    __syncthreads();
    if (l == 0 && w < 2) lf[F_SC + w] = mh;  // waves 0-1 hold the 128 features
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
  for (int i = tid; i < kH; i += kThreads) {
    lf[F_B2 + i] = P[PL.ob2() + i] * S2;
    lf[F_W3 + i] = P[PL.ow3() + i] * (1.0f / S2);
  }
  if (tid == 0) lf[F_B3] = P[PL.ob3()];
  float *slab = a.slab + (size_t)blockIdx.x * a.slab_stride;
  const float *w3g = P + PL.ow3();
  // (the loop's barriers order these LDS writes before their first reads)

  // ---- roles by SIMD: the first wave (lowest index) on each SIMD takes
  // the vector role, the second the matrix role (XH_SP8_VFIRST; 0 swaps
  // them), so that every SIMD pairs one of each whatever order the hardware
  // placed the waves in (HW_ID SIMD_ID, bits 5:4); any other placement falls
  // back to waves 4-7 / 0-3.
  // s / v number the matrix / vector waves by their SIMD's rank.
  if (l == 0)
    reinterpret_cast<int *>(lf + F_SIMD)[w] =
        (int)((__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) >> 4) & 3);
  __syncthreads();
  int is_matrix = XH_SP8_VFIRST ? w >= 4 : w < 4, role_idx = w & 3;
  {
    const int *sid = reinterpret_cast<const int *>(lf + F_SIMD);
    int per[4] = {0, 0, 0, 0}, rank = 0;
    for (int u = 0; u < 8; ++u) {
      const int su = sid[u];
      if (u < w && su == sid[w]) ++rank;
      per[su & 3]++;
    }
    if (per[0] == 2 && per[1] == 2 && per[2] == 2 && per[3] == 2) {
      is_matrix = XH_SP8_VFIRST ? rank == 1 : rank == 0;
      role_idx = sid[w];
    }
  }
  is_matrix = __builtin_amdgcn_readfirstlane(is_matrix);
  role_idx = __builtin_amdgcn_readfirstlane(role_idx);

  if (XH_SP8_ONLY == 2 ? false : XH_SP8_ONLY == 1 ? true : is_matrix) {
    // ======================= matrix waves =================================
    const int s = role_idx;  // outputs o in [32 s, 32 s + 32) for layer 2 /
                             // SM, features i in [32 s, 32 s + 32) for dW2
    // W2 (S_W) as f16 pairs, A operand of layer 2: lane row o = 32 s + l31,
    // K-step ks: k = the H1 image's column 16 ks + 8 h + e, which holds
    // feature i = 32 (ks >> 1) + 16 h + 8 (e >> 2) + 4 (ks & 1) + (e & 3)
    // (the image's column order: each vector lane stores its 16 features of
    // a row as two whole 16-byte chunks, see layer1)
    f16x8 wl[8][2];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const float *row = P + PL.oW2() + (32 * s + l31) * kH + 32 * (ks >> 1) + 16 * h + 4 * (ks & 1);
      const float4 v0 = *reinterpret_cast<const float4 *>(row),
                   v1 = *reinterpret_cast<const float4 *>(row + 8);
      const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 x0, x1;
        split2h(v[e] * SW, x0, x1);
        wl[ks][0][e] = x0;
        wl[ks][1][e] = x1;
      }
    }
    // per-region lane bases: layer 2's B operand (H1 image, transposed
    // reads), dW2's A operand (mask images, transposed reads), dW2's B
    // operand (g (x) H1 image, lane column i = 32 s + l31, row reads), the
    // mask stores from layer 2's C layout (lane row r = 32 t + l31, o = 32 s +
    // 8 q + 4 h ..; + 8192 t)
    // (layer 2's B operand: row reads of the [r][column] H1 image, lane row
    // r = 32 t + l31, K-step ks: columns 16 ks + 8 h ..; + 8192 t + 1024 (ks
    // >> 1); the columns' features as in the W2 fragments above)
    const int rbH0 = opaque(rd_base(l31, 0, h, 4) + L_H1), rbH1 = opaque(rd_base(l31, 1, h, 4) + L_H1);
    const int trM0 = opaque(tr_base(l, 0) + L_MK), trM1 = opaque(tr_base(l, 1) + L_MK);
    const int rbg0 = rd_base(32 * s + l31, 0, h, 2) + L_GH,
              rbg1 = rd_base(32 * s + l31, 1, h, 2) + L_GH;
    int mwb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) mwb[q] = opaque(wr_base(l31, q, h, 4) + 1024 * s + L_MK);

    f32x16s accW2[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int e = 0; e < 16; ++e) accW2[mt][e] = 0.0f;
    float accb2[16];  // db2 sums, 2 g M (the f16 mask 2.0)
#pragma unroll
    for (int e = 0; e < 16; ++e) accb2[e] = 0.0f;
    if (s == 0 && h == 0) lf[F_DB3 + l31] = 0.0f;

    struct Raw {
      int bi, rec;
    };
    // wave 0 stages the rows of a group: raw loads (the row's two bins per
    // lane; lanes 0-2 the action, old probability, advantage, lanes 3.. the
    // item's first coordinates), the stores into an LDS slot a phase later
#if XH_SP8_KL_TU
    // the row of the [T+1][N] arrays group g reads and the row of its old
    // distribution (kind 0 transition, 1 open end row, 2 terminal end row);
    // g is wave-uniform: scalar branches, and only terminal end rows wait for
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
#endif
    auto stage_load = [&](int j) {
#if XH_SP8_KL_TU
      size_t ti = tindex(j), qi = 0;
      kl_rows((int)ti, ti, qi);
      const size_t ri = qi;  // (open end rows: their record values are unused)
#else
      const size_t ti = tindex(j);
      const size_t ri = ti;
#endif
      // the row's bins: a wave-uniform base and the lane id recomputed
      // (mbcnt), not a per-lane pointer held (or spilled) across the loop
      const int lane =
          opaque((int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)));
      const unsigned short *rowp =
          reinterpret_cast<const unsigned short *>(a.b.bins + ti * (kB * kD));
      const int bins = rowp[lane];
      const unsigned long long p0 = (unsigned long long)(a.b.action + ri);
#if XH_SP8_KL_TU
      // lane 1: the aligned word holding done[qi] (an open end row's validity)
      const unsigned long long p1 = (unsigned long long)(a.b.done + (qi & ~(size_t)3));
#else
      const unsigned long long p1 = (unsigned long long)(a.b.pold + ri);
#endif
      const unsigned long long p2 = (unsigned long long)(a.adv + ri);
      const unsigned long long p3 = (unsigned long long)(a.b.items + ti * 4);
      unsigned long long pa = l >= 3 ? p3 : p2;
      pa = l == 1 ? p1 : pa;
      pa = l == 0 ? p0 : pa;
#if XH_SP8_KL_TU
      // the old distribution straight into its LDS slot (j & 3; its group
      // j - 4 finished with it a period ago), waited for at stage_store
      typedef __attribute__((address_space(1))) void gvoid;
      typedef __attribute__((address_space(3))) void lvoid;
      __builtin_amdgcn_global_load_lds((gvoid *)(a.qold + qi * kB + l),
                                       (lvoid *)(lf + F_Q + (j & 3) * 64), 4, 0, 0);
#endif
      return Raw{bins, *reinterpret_cast<const int *>(pa)};
    };
    auto stage_store = [&](const Raw &r, int sl SP8KL(, int j)) {
#if XH_SP8_KL_TU
      const int g = __builtin_amdgcn_readfirstlane((int)tindex(j));
      const int kind = g < NT ? 0 : g < NT + a.b.N ? 1 : 2;
      // the terminal view: the chosen bin without the item (rl.h:336-343)
      const int itm = __builtin_amdgcn_readlane(r.rec, 3);
      const bool sub = kind == 2 && l == __builtin_amdgcn_readfirstlane(r.rec);
      const float x0 =
          (float)((signed char)(r.bi & 0xff) - (sub ? (signed char)(itm & 0xff) : 0)) /
          (float)kCapacity;
      const float x1 =
          (float)((signed char)((r.bi >> 8) & 0xff) - (sub ? (signed char)((itm >> 8) & 0xff) : 0)) /
          (float)kCapacity;
      // the old distribution's LDS-direct load (issued with this group's
      // staging loads, a phase ago): complete before the phase's barrier
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
      const float x0 = (float)(signed char)(r.bi & 0xff) / (float)kCapacity;
      const float x1 = (float)(signed char)((r.bi >> 8) & 0xff) / (float)kCapacity;
#endif
      lf[F_X + sl * 128 + l] = x0;
      lf[F_X + sl * 128 + 64 + l] = x1;
      const int item = __builtin_amdgcn_readlane(r.rec, 3);
      const int i0 = (signed char)(item & 0xff), i1 = (signed char)((item >> 8) & 0xff);
#if XH_SP8_KL_TU
      // the record: action (lane 0), whether the row counts (lane 1: not a
      // terminal row past n_end, nor an open end row whose env ended at step
      // T - 1), advantage (lane 2, 0 for end rows)
      const int dw = __builtin_amdgcn_readlane(r.rec, 1);
      const size_t qi1 = kind == 1 ? (size_t)(NT - a.b.N) + (g - NT) : 0;
      const int ended = (dw >> (8 * (int)(qi1 & 3))) & 0xff;
      const bool valid = kind == 0 || (kind == 1 ? ended == 0 : g - NT - a.b.N < n_end);
      if (l == 0 || l == 2) lf[F_REC + 4 * sl + l] = kind == 0 ? __int_as_float(r.rec) : 0.0f;
      if (l == 1) lf[F_REC + 4 * sl + 1] = valid ? 1.0f : 0.0f;
#else
      if (l < 3) lf[F_REC + 4 * sl + l] = __int_as_float(r.rec);
#endif
      if (l == 3)
        lf[F_REC + 4 * sl + 3] =
            (i0 == a.env.item_a[0] && i1 == a.env.item_a[1]) ? 1.0f : 0.0f;
    };

    // layer 2 of the group in the H1 image: C[o][r] = S2 (b2 + W2 . H1) for
    // this wave's 32 o (registers) x r-tile t (lanes), 16 steps (t = st / 8,
    // K-step ks = st % 8) of three f16 MFMAs; the B operand (H1 pair, row
    // reads) one step ahead in ping-pong registers (the unrolled
    // step picks its buffer: no copies); task(k) after MFMA k
    auto layer2 = [&](f32x16s (&c)[2], auto &&task) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 b2 = lds4v(lf + F_B2 + 32 * s + 8 * q + 4 * h);
#pragma unroll
        for (int u = 0; u < 4; ++u) c[0][4 * q + u] = c[1][4 * q + u] = b2[u];
      }
      f16x8 bh[2], bl[2];
      auto ldB = [&](int st) {
        const int t = XH_SP8_L2I ? st & 1 : st >> 3, ks = XH_SP8_L2I ? st >> 1 : st & 7;
        const int o = ((ks & 1) ? rbH1 : rbH0) + 8192 * t + 1024 * (ks >> 1);
        bh[st & 1] = ld8h(o);
        bl[st & 1] = ld8h(o + kImg);
      };
      ldB(0);
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int t = XH_SP8_L2I ? st & 1 : st >> 3, ks = XH_SP8_L2I ? st >> 1 : st & 7,
                  cb = st & 1;
        if (st + 1 < 16) ldB(st + 1);
        FENCE();
        c[t] = mfma_f16(wl[ks][1], bh[cb], c[t]);  // the three products,
        FENCE();                                   // small terms first
        task(3 * st);
        FENCE();
        c[t] = mfma_f16(wl[ks][0], bl[cb], c[t]);
        FENCE();
        task(3 * st + 1);
        FENCE();
        c[t] = mfma_f16(wl[ks][0], bh[cb], c[t]);
        FENCE();
        task(3 * st + 2);
        FENCE();
      }
    };
    // partial logits of rows 32 t + l31 over this wave's o -> F_Z: block q of
    // four values into its own partial sum (four independent chains); w3 of
    // block q in a two-deep ring (ld_w3 a slot or more before partial_q)
    float zq[4];
    f32x4 w3v[2];
    auto ld_w3 = [&](int q) { w3v[q & 1] = lds4v(lf + F_W3 + 32 * s + 8 * q + 4 * h); };
    auto partial_q = [&](const f32x16s &ct, int q) {
      float z = relu(ct[4 * q]) * w3v[q & 1][0];
#pragma unroll
      for (int u = 1; u < 4; ++u) z = fmaf(relu(ct[4 * q + u]), w3v[q & 1][u], z);
      zq[q] = z;
    };
    auto partial_store = [&](int t) {
      const float z = add_halves((zq[0] + zq[1]) + (zq[2] + zq[3]));
      if (h == 0) lf[F_Z + 4 * (32 * t + l31) + s] = z;
    };
    // all four blocks of r-tile t, nothing to hide under
    auto partials_tail = [&](const f32x16s &ct, int t) {
      ld_w3(0);
      ld_w3(1);
      partial_q(ct, 0);
      ld_w3(2);
      partial_q(ct, 1);
      ld_w3(3);
      partial_q(ct, 2);
      partial_q(ct, 3);
      partial_store(t);
    };
    // softmax + loss gradient of group gi (partial logits in F_Z) -> gz
    // (rows l31, 32 + l31), in stages so that its dependent steps sit in
    // dW2's MFMA slots: stage(0) loads, stage(1) .. (6) the arithmetic; wave
    // 0 also stores g, g x0, g x1 -> F_G (the vector waves') and the db3 sums
    float gz[2];
    struct Sm {
      f32x4 rec, z0, z1, x;  // x: wave 0's bins of rows l31, 32 + l31
      float b3, ex0, ex1, se, p0, p1, gc, pc;
      int cu;
      float po, Ac;  // the record, wave-uniform from stage 1 on
#if XH_SP8_KL_TU
      float q0, q1;  // the old distribution of rows l31, 32 + l31 (pc, gc:
                     // the probability-space gradients; po: the row counts)
#endif
    } sm;
#if XH_SP8_KL_TU
    // KL(q || p) of the valid rows this wave summed: per-lane doubles in LDS
    // (ds_add_f64, nothing returned; a register pair held across the loop
    // spilled)
    double *kl_lane = reinterpret_cast<double *>(lf + F_KL) + 32 * s;
    if (h == 0) kl_lane[l31] = 0.0;
#endif
    auto softmax_stage = [&](int gi, int gpar, bool acc, int stage) {
      const int rs = gi & 3;
      switch (stage) {
        case 0:
          sm.rec = lds4v(lf + F_REC + 4 * rs);
          sm.b3 = lf[F_B3];
          sm.z0 = lds4v(lf + F_Z + 4 * l31);
          sm.z1 = lds4v(lf + F_Z + 4 * (32 + l31));
          if (s == 0) {
            // (wave 0's per-lane addresses recomputed here: held across the
            // loop they spilled)
            const float *xr = lf + F_X + rs * 128 + opaque(l31);
            sm.x = f32x4{xr[0], xr[32], xr[64], xr[96]};
          }
          break;
        case 1:
          sm.cu = __builtin_amdgcn_readfirstlane(__float_as_int(sm.rec[0]));
          sm.po = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sm.rec[1])));
          sm.Ac = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sm.rec[2])));
          sm.ex0 = __expf(((sm.z0[0] + sm.z0[1]) + (sm.z0[2] + sm.z0[3])) + sm.b3);
          sm.ex1 = __expf(((sm.z1[0] + sm.z1[1]) + (sm.z1[2] + sm.z1[3])) + sm.b3);
          break;
        case 2:
          // the half's sum (both halves hold all 64 rows), DPP only; lane 31
          // holds it
          sm.se = half_sum32(sm.ex0 + sm.ex1);
          break;
        case 3: {
#if XH_SP8_KL_TU
          sm.q0 = lf[F_Q + 64 * rs + l31];  // (used a slot later)
          sm.q1 = lf[F_Q + 64 * rs + 32 + l31];
#endif
          const float se = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm.se), 31));
          const float rse = __builtin_amdgcn_rcpf(se);
          sm.p0 = sm.ex0 * rse;
          sm.p1 = sm.ex1 * rse;
          break;
        }
#if XH_SP8_KL_TU
        case 4: {
          // kl_regulated_loss (policy_gradient.h:41-85): softmax_gradient_log
          // + beta (p - q) as a probability-space gradient (softmax_layer::
          // backward in the next two stages); the KL sum by one matrix wave
          // per group, in turn, lane half 0 (both halves hold the rows)
          const int cu = sm.cu;
          const float Ac = sm.Ac;
          float g0 = fmaf(beta, sm.p0 - sm.q0, sm.p0 * Ac);
          float g1 = fmaf(beta, sm.p1 - sm.q1, sm.p1 * Ac);
          if (l31 == cu) g0 -= Ac;
          if (32 + l31 == cu) g1 -= Ac;
          sm.pc = g0;
          sm.gc = g1;
          const bool vld = __float_as_int(sm.po) != 0;
          if (vld && (gi & 3) == s && h == 0)
            __hip_atomic_fetch_add(kl_lane + opaque(l31),
                                   (double)(sm.q0 * logf(sm.q0 / sm.p0)) +
                                       (double)(sm.q1 * logf(sm.q1 / sm.p1)),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          break;
        }
        case 5:
          sm.se = half_sum32(sm.p0 * sm.pc + sm.p1 * sm.gc);
          break;
        case 6: {
          const float sgv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm.se), 31));
          const bool vld = __float_as_int(sm.po) != 0;
          gz[0] = vld ? sm.p0 * (sm.pc - sgv) : 0.0f;
          gz[1] = vld ? sm.p1 * (sm.gc - sgv) : 0.0f;
          break;
        }
#else
        case 4: {
          const int cu = sm.cu;
          sm.pc = __int_as_float(
              __builtin_amdgcn_readlane(__float_as_int(cu >= 32 ? sm.p1 : sm.p0), cu & 31));
          if (a.algo == kPPO) {
            // clipped_gradient (rl.h:54-74) through softmax_layer::backward
            const float po = sm.po, Ac = sm.Ac;
            const float ratio = sm.pc * __builtin_amdgcn_rcpf(po);
            float ce = a.clip_eps;  // the bounds computed here, not held
            asm volatile("" : "+s"(ce));
            const float clipped = fminf(fmaxf(ratio, 1.0f - ce), 1.0f + ce);
            const float ig = fminf(clipped * Ac, ratio * Ac) * -1.0f;
            sm.gc = ig * __builtin_amdgcn_rcpf(sm.pc);
          }
          break;
        }
        case 5: {
          const int cu = sm.cu;
          const float Ac = sm.Ac;
          if (a.algo == kPPO) {
            gz[0] = ((l31 == cu ? sm.p0 : 0.0f) - sm.p0 * sm.pc) * sm.gc;
            gz[1] = ((32 + l31 == cu ? sm.p1 : 0.0f) - sm.p1 * sm.pc) * sm.gc;
          } else {
            // softmax_gradient_log (rl.h:45-52) through softmax-xent
            gz[0] = sm.p0 * Ac;
            gz[1] = sm.p1 * Ac;
            if (l31 == cu) gz[0] -= Ac;
            if (32 + l31 == cu) gz[1] -= Ac;
          }
          break;
        }
#endif
        default:
          if (s == 0 && h == 0) {
            const int lo = opaque(l31);
            float *gv = lf + F_G + 192 * gpar + lo;
            gv[0] = gz[0];
            gv[32] = gz[1];
            gv[64] = gz[0] * sm.x[0];
            gv[96] = gz[1] * sm.x[1];
            gv[128] = gz[0] * sm.x[2];
            gv[160] = gz[1] * sm.x[3];
            // db3: per-lane sums in LDS (ds_add_f32, nothing returned; a
            // register here spilled)
            if (acc)
              __hip_atomic_fetch_add(lf + F_DB3 + lo, gz[0] + gz[1], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          // a look-ahead group past the end: its dW3 / db2 terms vanish
          if (!acc) gz[0] = gz[1] = 0.0f;
      }
    };
    // the relu mask of layer-2 value e of r-tile t as 0 / 0x4000 (2.0 both
    // as bf16, dW2's A operand, and as f16, dH1's: one image serves both MFMA
    // types, the factor 2 taken back exactly at the write-outs); db2's sum
    // 2 g M by one v_fma_mix_f32 reading the word's low half as f16; the
    // words of block (t, q) stored into slot ms after its fourth value.  dW3
    // needs no per-row work: it is reassociated through dW2 after the loop.
    unsigned mwd[2];
    auto mv_e = [&](const f32x16s (&c)[2], int ms, int t, int e) {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const int q = e >> 2, u = e & 3;
      if ((u & 1) == 0) {
        // the pair's word: relu'(x) in {0, 1} from x's bits by v_med3_i32 (no
        // compare writing VCC), packed and times 0x4000 by the 24-bit multiply
        int m0, m1;
        asm("v_med3_i32 %0, %1, 0, 1" : "=v"(m0) : "v"(__float_as_int(c[t][e])));
        asm("v_med3_i32 %0, %1, 0, 1" : "=v"(m1) : "v"(__float_as_int(c[t][e + 1])));
        mwd[u >> 1] = (unsigned)__umul24((unsigned)m0 | ((unsigned)m1 << 16), 0x4000u);
        accb2[e] = fma_mix_lo(mwd[u >> 1], gz[t], accb2[e]);
      } else {
        accb2[e] = fma_mix_hi(mwd[u >> 1], gz[t], accb2[e]);
      }
      if (u == 3) {
        const int mb = 2 * kImg * ms;  // (mwb holds L_MK)
        const u32x2 mm = {mwd[0], mwd[1]};
        st4(mb + 8192 * t + mwb[q], __builtin_bit_cast(bf16x4, mm));
      }
    };
    // dW2 += M^T (S_H g (x) H1) of the group whose masks are in slot ms:
    // 16 steps (K-step ks = st / 4 of 16 rows, o-tile mt = st % 4) of three
    // bf16 MFMAs; A (mask, transposed reads) one step ahead, B (the three
    // parts) one K-step ahead, both ping-pong; task(k) after MFMA k
    auto dw2 = [&](int ms, auto &&task) {
      const int mb = 2 * kImg * ms;  // (trM holds L_MK)
      bf16x8 A[2], B[2][3];
      auto ldB = [&](int ks) {
        const int ob = L_GH + 1024 * (ks >> 1) + ((ks & 1) ? rbg1 : rbg0);
        B[ks & 1][0] = ld8(ob);
        B[ks & 1][1] = ld8(ob + kImg);
        B[ks & 1][2] = ld8(ob + 2 * kImg);
      };
      auto ldA = [&](int st) {
        const int o = mb + 1024 * (4 * (st >> 2) + (st & 3));
        A[st & 1] = ldtr(trM0 + o, trM1 + o);
      };
      ldB(0);
      ldA(0);
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int ks = st >> 2, mt = st & 3, ca = st & 1, cb = ks & 1;
        if (st + 1 < 16) {
          ldA(st + 1);
          if (mt == 3) ldB(ks + 1);
        }
        FENCE();
        accW2[mt] = mfma_bf16(A[ca], B[cb][2], accW2[mt]);
        FENCE();
        task(3 * st);
        FENCE();
        accW2[mt] = mfma_bf16(A[ca], B[cb][1], accW2[mt]);
        FENCE();
        task(3 * st + 1);
        FENCE();
        accW2[mt] = mfma_bf16(A[ca], B[cb][0], accW2[mt]);
        FENCE();
        task(3 * st + 2);
        FENCE();
      }
    };
    // B's VALU in dW2's 48 slots: the softmax stages (loads in slot 0, the
    // arithmetic from slot 3 on, one stage per slot), then group gi's masks
    // and db2 sums (slots 12 .. 43), a mask block stored every fourth slot
    auto b_task = [&](const f32x16s (&c)[2], int gi, int gpar, bool acc, int k) {
      if (k == 0)
        softmax_stage(gi, gpar, acc, 0);
      else if (k >= 3 && k < (XH_SP8_KL_TU ? 10 : 9))
        softmax_stage(gi, gpar, acc, k - 2);
      else if (k >= 12 && k < 44)
        mv_e(c, gpar, (k - 12) >> 4, (k - 12) & 15);
    };
    auto no_task = [](int) {};

    // ---- pipeline prologue (barriers as the vector path's)
    if (XH_SP8_PRIO & 3) __builtin_amdgcn_s_setprio(XH_SP8_PRIO & 3);
    f32x16s c[2];
    if (s == 0) {
      stage_store(stage_load(0), 0 SP8KL(, 0));
      stage_store(stage_load(1), 1 SP8KL(, 1));
      stage_store(stage_load(2), 2 SP8KL(, 2));
    }
    __syncthreads();  // P1: rows staged          (vector: L1(0))
    __syncthreads();  // P2
    layer2(c, no_task);
    partials_tail(c[0], 0);
    partials_tail(c[1], 1);
    __syncthreads();  // P3                       (vector: L1(1))
#pragma unroll
    for (int k = 0; k < 48; ++k) b_task(c, 0, 0, true, k);
    __syncthreads();  // P4
    // one period; P = j & 1 at compile time (mask / g slots, image offsets
    // fold into immediates)
    auto period = [&](int j, auto P) {
      constexpr int par = decltype(P)::value;
      Raw raw;
      if (s == 0) raw = stage_load(j + 3);
      // A(j): layer 2 of group j+1; r-tile 0's partial logits in r-tile 1's
      // MFMA slots, r-tile 1's after
#if XH_SP8_L2I
      // (r-tile 0 is complete only after step 14: its partials after it,
      // r-tile 1's at the tail)
      if (SP8_RUN(1 | 32)) layer2(c, [&](int k) {
        if (k == 40) ld_w3(0);
        if (k == 41) ld_w3(1);
      });
      if (SP8_RUN(1)) {
        partial_q(c[0], 0);
        ld_w3(2);
        partial_q(c[0], 1);
        ld_w3(3);
        partial_q(c[0], 2);
        partial_q(c[0], 3);
        partial_store(0);
        partials_tail(c[1], 1);
      }
#else
      if (SP8_RUN(1 | 32)) layer2(c, [&](int k) {
        // r-tile 0's blocks q at slots 27 + 3q, their w3 three slots ahead
        if (k >= 24 && k < 36 && k % 3 == 0) ld_w3((k - 24) / 3);
        if (k >= 27 && k < 39 && k % 3 == 0) partial_q(c[0], (k - 27) / 3);
        if (k == 40) partial_store(0);
      });
      if (SP8_RUN(1)) partials_tail(c[1], 1);
#endif
      __syncthreads();
      // B(j): dW2 of group j with group j+1's softmax, dW3 / db2 sums and
      // masks in its MFMA slots
      if (s == 0) stage_store(raw, (j + 3) & 3 SP8KL(, j + 3));
      const bool acc = j + 1 < J;
      if (SP8_RUN(1 | 16))
        dw2(par, [&](int k) { b_task(c, j + 1, 1 - par, acc, k); });
      __syncthreads();
    };
    for (int j = 0; j < J; j += 2) {
      period(j, Par<0>{});
      if (j + 1 < J) period(j + 1, Par<1>{});
    }

#if XH_SP8_KL_TU
    {
      // the workgroup's KL sum: the matrix waves' doubles in a fixed order
      // (the loop's last barrier is behind: F_Z is free; the vector waves
      // meet this barrier after their loop)
      double v = h == 0 ? kl_lane[l31] : 0.0;
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, kWave);
      double *kd = reinterpret_cast<double *>(lf + F_Z);
      if (l == 0) kd[s] = v;
      __syncthreads();
      if (s == 0 && l == 0) a.kl_part[blockIdx.x] = (kd[0] + kd[1]) + (kd[2] + kd[3]);
    }
#endif
    // ---- write-out (every entry has exactly one producing lane)
    const float rSH = 0.5f / SH;  // (the masks were 2.0)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int o = 32 * mt + 8 * (e >> 2) + 4 * h + (e & 3);
        slab[PL.oW2() + o * kH + 32 * s + l31] = (accW2[mt][e] * rSH) * w3g[o];
      }
    // dW3 = sum_r g_r relu(A2[r][o]), reassociated through A2 = H1 W2^T + b2:
    //   dW3[o] = sum_i W2[o][i] G[o][i] + b2[o] D[o],
    // G = M^T (g (x) H1) (dW2 before its w3 factor), D = M^T g (db2 before
    // it): no per-row work in the loop.  Its f32 error is of the order of the
    // rounding of A2 itself.  Each wave's partial sums over
    // its 32 features i meet in the free g (x) H1 image (one more barrier,
    // in both roles), summed in a fixed order.
    float *const d3p = reinterpret_cast<float *>(lds + L_GH);  // [4 s][128 o]
    float *const d3d = d3p + 4 * kH;                           // [128 o] D
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int o = 32 * mt + 8 * (e >> 2) + 4 * h + (e & 3);
        const float sv = seg_sum<32>((accW2[mt][e] * rSH) * P[PL.oW2() + o * kH + 32 * s + l31]);
        if (l31 == 0) d3p[s * kH + o] = sv;
      }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      // db2 of o = 32 s + 8 (e >> 2) + 4 h + (e & 3): sums over the 32 lanes
      // (rows) of the half
      const float s2 = seg_sum<32>(accb2[e]) * 0.5f;
      const int o = 32 * s + 8 * (e >> 2) + 4 * h + (e & 3);
      if (l31 == 0) {
        d3d[o] = s2;
        slab[PL.ob2() + o] = s2 * w3g[o];
      }
    }
    __syncthreads();  // the dW3 partials (vector: after their loop)
    if (h == 0) {
      const int o = 32 * s + l31;
      const float si = (d3p[o] + d3p[kH + o]) + (d3p[2 * kH + o] + d3p[3 * kH + o]);
      slab[PL.ow3() + o] = fmaf(P[PL.ob2() + o], d3d[o], si);
    }
    if (s == 0) {
      const float v3 = seg_sum<32>(lf[F_DB3 + l31]);
      if (l == 0) slab[PL.ob3()] = v3;
    }
  } else {
    // ======================= vector waves =================================
    const int v = role_idx;
    const int fi = 32 * v + l31;  // this lane's feature i
    // W2' = S_D diag(w3) W2 as f16 pairs, B operand of dH1: lane column i,
    // K-step ks: k = o = 16 ks + 8 h + e
    f16x8 wd[8][2];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int o = 16 * ks + 8 * h + e;
        _Float16 x0, x1;
        split2h((P[PL.oW2() + o * kH + fi] * P[PL.ow3() + o]) * SD, x0, x1);
        wd[ks][0][e] = x0;
        wd[ks][1][e] = x1;
      }
    // pre[r][i] = sum_k A[r][k] B[k][i] with A
    // = [x0, x1, 1, item is item_a, item is item_b] (exact in bf16: bins / 8)
    // and B = S_H [W1[i][0], W1[i][1], b1[i], W1[i][2..] . item_a / cap,
    // W1[i][2..] . item_b / cap] as three bf16 parts (the exact split:
    // products exact, the f32 sum within rounding of the fma chain); K
    // entries 5..15 zero.  B fragment: lane column i = fi, k = 8 h + e.
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    // the exact f32 chain for the values g (x) H1 and dW1's relu mask use:
    // S_H W1 columns and b1 + the item's part
    const float w1a = P[PL.oW1() + fi * kF0] * SH, w1b = P[PL.oW1() + fi * kF0 + 1] * SH;
    float b1a = P[PL.ob1() + fi], b1b = b1a;
#pragma unroll
    for (int d = 0; d < kD; ++d) {
      const float wv = P[PL.oW1() + fi * kF0 + kD + d];
      b1a += wv * ((float)a.env.item_a[d] / (float)kCapacity);
      b1b += wv * ((float)a.env.item_b[d] / (float)kCapacity);
    }
    b1a *= SH;
    b1b *= SH;
    auto h1_4 = [&](const f32x4 &x0, const f32x4 &x1, float b1, f32x4 &hv) {
#pragma unroll
      for (int u = 0; u < 4; ++u) hv[u] = relu(fmaf(x1[u], w1b, fmaf(x0[u], w1a, b1)));
    };
    auto b1_of = [&](int gi) {
      const bool ia =
          __builtin_amdgcn_readfirstlane(__float_as_int(lf[F_REC + 4 * (gi & 3) + 3])) != 0;
      return ia ? b1a : b1b;
    };
    // the layer-1 image (layer 2's f16-pair operand) from the matrix cores:
    bf16x8 w1p[3];
    {
      float ia = 0.0f, ib = 0.0f;
#pragma unroll
      for (int d = 0; d < kD; ++d) {
        const float wv = P[PL.oW1() + fi * kF0 + kD + d];
        ia += wv * ((float)a.env.item_a[d] / (float)kCapacity);
        ib += wv * ((float)a.env.item_b[d] / (float)kCapacity);
      }
      const float bv[5] = {P[PL.oW1() + fi * kF0], P[PL.oW1() + fi * kF0 + 1], P[PL.ob1() + fi],
                           ia, ib};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        __bf16 y0, y1, y2;
        split3(h == 0 && e < 5 ? bv[e] * SH : 0.0f, y0, y1, y2);
        w1p[0][e] = y0;
        w1p[1][e] = y1;
        w1p[2][e] = y2;
      }
    }
    // image stores (lane row i, values r = 32 t + 8 q + 4 h ..; + 1024 t):
    // the g (x) H1 image (region base 0) and the H1 image; dH1's A operand
    // (the mask image read as f16, lane row r = 32 t + l31)
    int vwb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) vwb[q] = opaque(wr_base(fi, q, h, 2) + L_GH);
    // the H1 image is [r][column]: lane row r = 32 t + l31 (+ 8192 t); this
    // lane's features i = 32 v + 8 q + 4 h + u go to columns 32 v + 16 h + 8
    // (q >> 1) + 4 (q & 1) + u, i.e. whole chunks 2 h and 2 h + 1 of column
    // tile v (one ds_write_b128 each, conflict-free in the poff layout)
    int vwH[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) vwH[j] = opaque(poff(l31, 32 * v + 16 * h + 8 * j, 4) + L_H1);
    const int rbm0 = opaque(rd_base(l31, 0, h, 4) + L_MK),
              rbm1 = opaque(rd_base(l31, 1, h, 4) + L_MK);
    float w0 = 0.0f, w1 = 0.0f, sa = 0.0f, sb = 0.0f;

    // S_H pre-activations of layer 1 of group gi (its bins in slot gi & 3)
    // for this wave's features: two r-tiles of three bf16 MFMAs with W1 as
    // the A operand, C[i][r] (lane column r = 32 t + l31, registers i = 32 v
    // + 8 q + 4 h + u): the [r][i] image's layout
    auto l1_mfma = [&](int gi, f32x16s (&pre)[2]) {
      const int sl = gi & 3;
      const bool ia =
          __builtin_amdgcn_readfirstlane(__float_as_int(lf[F_REC + 4 * sl + 3])) != 0;
      // X fragment (the B operand), lane column r = 32 t + l31, k = 8 h + e:
      // (x0, x1), (1, ia), (ib, 0), (0, 0) in lane half 0, zeros in half 1
      const unsigned d1 = h ? 0u : (ia ? 0x3F803F80u : 0x00003F80u);
      const unsigned d2 = h ? 0u : (ia ? 0u : 0x00003F80u);
      const float *xv = lf + F_X + sl * 128 + l31;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const unsigned d0 = __builtin_bit_cast(
            unsigned, bf16x2{(__bf16)xv[32 * t], (__bf16)xv[64 + 32 * t]});
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const bf16x8 X = __builtin_bit_cast(bf16x8, u32x4{h ? 0u : d0, d1, d2, 0u});
        pre[t] = mfma_bf16(w1p[2], X, f32x16s{});
        pre[t] = mfma_bf16(w1p[1], X, pre[t]);
        pre[t] = mfma_bf16(w1p[0], X, pre[t]);
      }
    };
    // B: layer 1 of group gi -> the H1 image (f16 pairs), block b = (t, q)
    // of four rows at a time; the values are recomputed where DH needs them
    auto layer1 = [&](int gi) {
      f32x16s pre[2];
      l1_mfma(gi, pre);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        // chunk j = b & 1 of r-tile t = b >> 1: blocks q = 2 j, 2 j + 1
        const int t = b >> 1, j = b & 1;
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        u32x4 hi, lo;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int q = 2 * j + (p >> 1), u = 2 * (p & 1);
          // f16 pairs: v_cvt_pk_f16_f32, the remainders by v_fma_mix (exact)
          unsigned h2, l2;
          split2h_x2(relu(pre[t][4 * q + u]), relu(pre[t][4 * q + u + 1]), h2, l2);
          hi[p] = h2;
          lo[p] = l2;
        }
        st8h(vwH[j] + 8192 * t, __builtin_bit_cast(f16x8, hi));
        st8h(vwH[j] + kImg + 8192 * t, __builtin_bit_cast(f16x8, lo));
      }
    };
    // x0, x1 -> three bf16 parts each, as bf16 pairs: v_cvt_pk_bf16_f32 and
    // the pair's f32 values from its bits (element 0 << 16, element 1 &
    // 0xffff0000; the compiler otherwise re-converts each element alone);
    // the differences are exact in f32.  11 VALU per pair.
    auto split3_pair = [](float x0, float x1, unsigned &ph, unsigned &pm, unsigned &pl) {
      auto cvt = [](float a, float b) {
        // (opaque: the compiler would re-convert element 0 alone for its
        // shift)
        return (unsigned)opaque((int)__builtin_bit_cast(unsigned, bf16x2{(__bf16)a, (__bf16)b}));
      };
      auto lo_f = [](unsigned u) { return __uint_as_float(u << 16); };
      auto hi_f = [](unsigned u) { return __uint_as_float(u & 0xffff0000u); };
      ph = cvt(x0, x1);
      const float r0 = x0 - lo_f(ph), r1 = x1 - hi_f(ph);
      pm = cvt(r0, r1);
      const float s0 = r0 - lo_f(pm), s1 = r1 - hi_f(pm);
      pl = cvt(s0, s1);
    };
    // A(gi): DH -- S_D dH1 = M (S_D W2') for this wave's features, 16 steps
    // of two f16 MFMAs (r-tile t = st / 8, K-step ks = st % 8; A, the f16
    // mask image, one step ahead) -- with, in the MFMA slots, the group's
    // layer-1 values (hk, kept for B's dW1) and S_H g (x) H1 -> the split
    // image: block b = (t, q) = (b / 4, b % 4) of four rows over slots 4b ..
    // 4b + 3, its bins and g two blocks ahead (a ring of three indexed by the
    // unrolled block).  dh stays in registers for B's dW1.  gpar = gi & 1.
    auto dh_gh = [&](int gi, int gpar, f32x16s (&hk)[2], f32x16s (&dh)[2]) {
      const int mb = 2 * kImg * gpar;  // the masks of slot gpar, read as f16 (rbm holds L_MK)
      const float *gv = lf + F_G + 192 * gpar;
      const float *xv = lf + F_X + (gi & 3) * 128;
      const float b1 = b1_of(gi);
      f16x8 A[2];
      auto ldA = [&](int st) {
        const int t = XH_SP8_DHI ? st & 1 : st >> 3, ks = XH_SP8_DHI ? st >> 1 : st & 7;
        A[st & 1] = ld8h(((ks & 1) ? rbm1 : rbm0) + mb + 8192 * t + 1024 * (ks >> 1));
      };
      f32x4 ring[3][3];  // [block % 3][x0, x1, g]
      auto ld3 = [&](int b) {
        const int r0 = 32 * (b >> 2) + 8 * (b & 3) + 4 * h;
        ring[b % 3][0] = lds4v(xv + r0);
        ring[b % 3][1] = lds4v(xv + 64 + r0);
        ring[b % 3][2] = lds4v(gv + r0);
      };
      ld3(0);
      ld3(1);
      float x[4];
      unsigned ph[2], pm[2], pl[2];
      auto gh_slot = [&](int k) {
        const int b = k >> 2, t = b >> 2, q = b & 3;
        const f32x4(&o)[3] = ring[b % 3];
        switch (k & 3) {
          case 0: {
            f32x4 hv;
            h1_4(o[0], o[1], b1, hv);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              hk[t][4 * q + u] = hv[u];
              x[u] = hv[u] * o[2][u];
            }
            if (b + 2 < 8) ld3(b + 2);
            break;
          }
          case 1:
            split3_pair(x[0], x[1], ph[0], pm[0], pl[0]);
            if (XH_SP8_GH2) split3_pair(x[2], x[3], ph[1], pm[1], pl[1]);
            break;
          case 2:
            if (!XH_SP8_GH2) split3_pair(x[2], x[3], ph[1], pm[1], pl[1]);
            break;
          default: {
            const int o2 = vwb[q] + 1024 * t;
            st4(o2, __builtin_bit_cast(bf16x4, u32x2{ph[0], ph[1]}));
            st4(o2 + kImg, __builtin_bit_cast(bf16x4, u32x2{pm[0], pm[1]}));
            st4(o2 + 2 * kImg, __builtin_bit_cast(bf16x4, u32x2{pl[0], pl[1]}));
          }
        }
      };
      ldA(0);
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int t = XH_SP8_DHI ? st & 1 : st >> 3, ks = XH_SP8_DHI ? st >> 1 : st & 7,
                  ca = st & 1;
        if (st + 1 < 16) ldA(st + 1);
        VAFENCE();
        if (ks == 0)
          dh[t] = mfma_f16(A[ca], wd[ks][1], f32x16s{});
        else
          dh[t] = mfma_f16(A[ca], wd[ks][1], dh[t]);
        VAFENCE();
        gh_slot(2 * st);
        VAFENCE();
        dh[t] = mfma_f16(A[ca], wd[ks][0], dh[t]);
        VAFENCE();
        gh_slot(2 * st + 1);
        VAFENCE();
      }
    };
    // B(gi): dW1 / db1 / item sums of group gi: d = relu'(H1) dH1 g; sums
    // d x0, d x1, d (g, g x0, g x1 staged by matrix wave 0), two partial
    // sums each; block b's vectors one block ahead (ping-pong)
    auto dw1 = [&](int gi, int gpar, const f32x16s (&hk)[2], const f32x16s (&dh)[2]) {
      const float *gv = lf + F_G + 192 * gpar;
      float a0[2] = {0.0f, 0.0f}, a1[2] = {0.0f, 0.0f}, ag[2] = {0.0f, 0.0f};
      f32x4 gb[2][3];
      auto ld3 = [&](int b) {
        const int r0 = 32 * (b >> 2) + 8 * (b & 3) + 4 * h;
        gb[b & 1][0] = lds4v(gv + r0);
        gb[b & 1][1] = lds4v(gv + 64 + r0);
        gb[b & 1][2] = lds4v(gv + 128 + r0);
      };
      ld3(0);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int t = b >> 2, q = b & 3;
        if (b + 1 < 8) ld3(b + 1);
        VBFENCE();
        const f32x4(&cur)[3] = gb[b & 1];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float m = hk[t][4 * q + u] > 0.0f ? dh[t][4 * q + u] : 0.0f;
          a0[u & 1] = fmaf(m, cur[1][u], a0[u & 1]);
          a1[u & 1] = fmaf(m, cur[2][u], a1[u & 1]);
          ag[u & 1] = fmaf(m, cur[0][u], ag[u & 1]);
        }
        VBFENCE();
      }
      w0 += a0[0] + a0[1];
      w1 += a1[0] + a1[1];
      const float sg = ag[0] + ag[1];
      const bool ia =
          __builtin_amdgcn_readfirstlane(__float_as_int(lf[F_REC + 4 * (gi & 3) + 3])) != 0;
      if (ia)
        sa += sg;
      else
        sb += sg;
    };

    f32x16s hk[2], dh[2];
    if (XH_SP8_PRIO >> 2) __builtin_amdgcn_s_setprio(XH_SP8_PRIO >> 2);
    __syncthreads();  // P1: rows staged
    layer1(0);
    __syncthreads();  // P2                       (matrix: L2(0))
    __syncthreads();  // P3
    layer1(1);
    __syncthreads();  // P4                       (matrix: SM(0))
    auto period = [&](int j, auto P) {
      constexpr int par = decltype(P)::value;
      if (SP8_RUN(2 | 4)) dh_gh(j, par, hk, dh);
      __syncthreads();  // A(j)
      if (SP8_RUN(2 | 64)) dw1(j, par, hk, dh);
      if (SP8_RUN(2 | 8)) layer1(j + 2);
      __syncthreads();  // B(j)
    };
    for (int j = 0; j < J; j += 2) {
      period(j, Par<0>{});
      if (j + 1 < J) period(j + 1, Par<1>{});
    }

#if XH_SP8_KL_TU
    __syncthreads();  // the matrix waves' KL sum
#endif
    __syncthreads();  // the matrix waves' dW3 partials
    // ---- write-out: dW1 / db1 of feature fi (the two lane halves hold row
    // subsets; dH1 was in units of S_D)
    float tw0 = w0 + __shfl_xor(w0, 32, kWave);
    float tw1 = w1 + __shfl_xor(w1, 32, kWave);
    float va = sa + __shfl_xor(sa, 32, kWave);
    float vb = sb + __shfl_xor(sb, 32, kWave);
    // (dH1 was in units of S_D, times the masks' 2)
    tw0 *= 0.5f / SD;
    tw1 *= 0.5f / SD;
    va *= 0.5f / SD;
    vb *= 0.5f / SD;
    if (h == 0) {
      slab[PL.oW1() + fi * kF0 + 0] = tw0;
      slab[PL.oW1() + fi * kF0 + 1] = tw1;
#pragma unroll
      for (int d = 0; d < kD; ++d)
        slab[PL.oW1() + fi * kF0 + kD + d] =
            va * ((float)a.env.item_a[d] / (float)kCapacity) +
            vb * ((float)a.env.item_b[d] / (float)kCapacity);
      slab[PL.ob1() + fi] = va + vb;
    }
  }
}

}  // namespace sp8

#if XH_SP8_KL_TU
hipError_t launch_policy_train_spec8_kl(const PolicyTrainArgs &a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)sp8::policy_train_spec8_kl_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sp8::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(sp8::policy_train_spec8_kl_kernel, dim3(grid), dim3(sp8::kThreads),
                     sp8::kLds, s, a);
  return hipGetLastError();
}
#else
hipError_t launch_policy_train_spec8(const PolicyTrainArgs &a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)sp8::policy_train_spec8_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sp8::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(sp8::policy_train_spec8_kernel, dim3(grid), dim3(sp8::kThreads),
                     sp8::kLds, s, a);
  return hipGetLastError();
}
#endif

}  // namespace xh
