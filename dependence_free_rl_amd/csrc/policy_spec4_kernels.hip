// policy_spec4_kernels.hip -- the PPO / actor-critic train epoch of the
// 32-bin 1-D [64,64] policy (BASELINE config 2) with WAVE SPECIALISATION, the
// design of policy_spec8_kernels.hip (config 3) for the [64,64] shape: one
// 8-wave workgroup per CU, and on every SIMD one "matrix" wave (layer 2, the
// softmax and loss gradient, the relu masks, dW3 / db2 sums, dW2) beside one
// "vector" wave (layer 1, g (x) H1, dH1, dW1), so the VALU of the one overlaps
// the MFMAs of the other (the probes in that header).
//
// Reference: the epoch is ppo_learner::optimize_action's optimizer::step
// (policy_gradient.h:297-307, nn.h:594-605) on the per-bin conv1d_1 policy
// (nn.h:127-186) of ppo_training.cc:12-31 -- clipped_gradient (rl.h:54-74)
// or softmax_gradient_log (rl.h:45-52, actor-critic) through
// softmax_layer::backward (nn.h:393-417); the gradients are row sums into
// one f32 slab per workgroup (nn.h:94-98), reduced in a fixed order after.
//
// Numerics as policy_train_split4h_kernel: layer 2
// and dH1 on f16 pairs scaled by powers of two, dW2 on the exact bf16
// three-part split of S_H g (x) H1 against the 0/1 relu mask, f32
// accumulation; the MFMA shape (32x32x16) and so the accumulation order
// differ.
//
// A 64-row group is two envs (rows 0-31 env A = transition 2 g, rows 32-63
// env B = transition 2 g + 1): the 32x32 r-tile of every product is one env.
// Matrix wave s: layer 2 / masks / dW3 / db2 of o-tile s & 1 and env s >> 1,
// the softmax of env s >> 1, dW2 tile (o-tile s & 1, i-tile s >> 1) over
// both envs; vector wave v: layer 1, g (x) H1, dH1 and dW1 of i-tile v & 1
// and env v >> 1.  Per group and wave: matrix 12 + 12 MFMAs, vector 3 + 8.
// Pipelined two phases per group, each closed by a barrier (as spec8):
//   A(j): matrix L2(j+1) + partial logits    vector DH(j) + g (x) H1(j)
//   B(j): matrix SM(j+1), masks, dW3 / db2 of j+1 + DW(j)
//                                            vector dW1(j) + L1(j+2)
// LDS: g (x) H1 three bf16 parts [64 i][64 r] (24 KB), H1 two f16 parts
// [64 r][64 i] (16 KB), relu masks [64 r][64 o] in two slots (0x4000 = 2.0
// as bf16 and as f16), then f32 vectors; image layout spec8_layout.h (ny 2).
#include <cstdlib>
#include <type_traits>

#include "spec8_layout.h"
#include "xh_device.h"
#include "xh_kernels.h"
#include "xh_split.h"

// XH_SP4_VFIRST: the vector role to the first (older) wave on each SIMD,
// which wins VALU issue arbitration (as XH_SP8_VFIRST)
#ifndef XH_SP4_VFIRST
#define XH_SP4_VFIRST 1
#endif

// Phase stamps (trace build, tools/build_trace_sp4.sh: -DXH_DIAG_TRACE=1,
// run with XH_PHASE_TRACE=1): lane 0 of every wave of the first kTraceBlocks
// workgroups records the cycle counter at 0 A(j) start, 1 its phase-A work
// done, 2 after the A barrier, 3 its phase-B work done, 4 after the B barrier
// (5 .. 7 = 4) for groups j < kTraceGroups - 1
#ifndef XH_DIAG_TRACE
#define XH_DIAG_TRACE 0
#endif
#if XH_DIAG_TRACE
#define SP4_STAMP(a, gi, w, lane, slot)                                               \
  do {                                                                                \
    if ((a).trace && blockIdx.x < kTraceBlocks && (gi) < kTraceGroups - 1 && (lane) == 0) \
      for (int k_ = (slot); k_ < ((slot) == 4 ? kTraceSlots : (slot) + 1); ++k_)      \
        (a).trace[((blockIdx.x * kTraceGroups + (gi)) * 8 + (w)) * kTraceSlots + k_] = \
            clock64();                                                                \
  } while (0)
#else
#define SP4_STAMP(a, gi, w, lane, slot) \
  do {                                  \
  } while (0)
#endif

namespace xh {
namespace sp4 {

using sp8::poff;
using sp8::rd_base;
using sp8::tr_base;
using sp8::wr_base;

constexpr int kB = 32, kD = 1, kF0 = 2 * kD, kH = 64;
constexpr int kThreads = 512;
constexpr int kNY = 2;             // 64 image columns = 2 column tiles
constexpr int kImg = 8192;         // one [64][64] 16-bit image
constexpr int L_GH = 0;            // g (x) H1: hi, mid, lo
constexpr int L_H1 = 3 * kImg;     // H1: hi, lo
constexpr int L_MK = 5 * kImg;     // masks: slot s at + kImg s
constexpr int L_F = 7 * kImg;
constexpr int F_B2 = 0;            // [64] b2 S2
constexpr int F_W3 = F_B2 + kH;    // [64] w3 / S2
constexpr int F_Z = F_W3 + kH;     // [64 rows][2 o-tiles] partial logits
constexpr int F_G = F_Z + 128;     // [2 parities][g, g x][64 rows]
constexpr int F_X = F_G + 256;     // [4 slots][64 rows] bins / 8
constexpr int F_REC = F_X + 256;   // [4 slots][2 envs][action, pold, adv, item is item_a]
constexpr int F_SC = F_REC + 32;   // [16] scale reduction scratch, the scales
constexpr int F_B3 = F_SC + 16;    // [4]
constexpr int F_SIMD = F_B3 + 4;   // [8] the SIMD each wave runs on (ints)
constexpr int F_END = F_SIMD + 8;
constexpr size_t kLds = L_F + sizeof(float) * F_END;
static_assert(kLds <= 160 * 1024, "LDS");
static_assert(F_Z % 4 == 0 && F_G % 4 == 0 && F_X % 4 == 0 && F_REC % 4 == 0 &&
                  F_B2 % 4 == 0 && F_W3 % 4 == 0,
              "16-byte aligned f32 vectors");
#define FENCE() __builtin_amdgcn_sched_barrier(0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) bf16x8 lbf16x8;
typedef __attribute__((address_space(3))) bf16x4 lbf16x4;
typedef __attribute__((address_space(3))) f16x8 lf16x8;
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
// two ds_read_b64_tr_b16 (EXEC full): elements 0-3 from o0, 4-7 from o1
__device__ __forceinline__ bf16x8 ldtr(int o0, int o1) {
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ls16x4 *)(size_t)(unsigned)o0);
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ls16x4 *)(size_t)(unsigned)o1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ f32x4 lds4v(const float *p) {
  return *reinterpret_cast<const f32x4 *>(p);
}
__device__ __forceinline__ f32x2 lds2v(const float *p) {
  return *reinterpret_cast<const f32x2 *>(p);
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

__global__ __launch_bounds__(kThreads, 2) void policy_train_spec4_kernel(PolicyTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float *lf = reinterpret_cast<float *>(lds + L_F);
  const PolicyLayout PL{kF0, kH, kH};
  const float *P = a.params;
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int l = tid & 63, h = l >> 5, l31 = l & 31;
  const int ngroups = a.b.T * a.b.N / 2;  // 64-row groups of two envs
  // this workgroup's groups g_j = b0 + j gridDim.x, j < J (XCD-aware b0:
  // the adjacent groups whose records share a 128-byte line are read by one
  // XCD's L2); look-ahead indices past the end are clamped to the last group
  // and their results discarded
  const int b0 = ((int)gridDim.x & 7) == 0
                     ? ((int)blockIdx.x & 7) * ((int)gridDim.x >> 3) + ((int)blockIdx.x >> 3)
                     : (int)blockIdx.x;
  const int J = b0 < ngroups ? (ngroups - b0 + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  if (J == 0) return;  // uniform over the workgroup
  const int gstep = (int)gridDim.x;
  auto gindex = [&](int j) { return (size_t)(b0 + min(j, J - 1) * gstep); };

  // ---- prologue: the scales (maxima over the parameters, every workgroup
  // the same), small parameters into LDS
  {
    float mw = 0.0f, md = 0.0f, mh = 0.0f;
    for (int e = tid; e < kH * kH; e += kThreads) {
      const float v = P[PL.oW2() + e];
      mw = fmaxf(mw, fabsf(v));
      md = fmaxf(md, fabsf(v * P[PL.ow3() + (e >> 6)]));
    }
    if (tid < kH) {
      const float wv = P[PL.oW1() + tid * kF0 + kD];
      const float b1 = P[PL.ob1() + tid];
      const float ba = b1 + wv * ((float)a.env.item_a[0] / (float)kCapacity);
      const float bb = b1 + wv * ((float)a.env.item_b[0] / (float)kCapacity);
      mh = fabsf(P[PL.oW1() + tid * kF0]) + fmaxf(fabsf(ba), fabsf(bb));
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
    if (l == 0 && w == 0) lf[F_SC + 0] = mh;  // wave 0 holds the 64 features
    __syncthreads();
    const float MH = lf[F_SC + 0];
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

  // ---- roles by SIMD (as spec8): the first wave on each SIMD takes the
  // vector role, the second the matrix role (XH_SP4_VFIRST; 0 swaps them);
  // any other placement falls back to waves 4-7 / 0-3
  if (l == 0)
    reinterpret_cast<int *>(lf + F_SIMD)[w] =
        (int)((__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) >> 4) & 3);
  __syncthreads();
  int is_matrix = XH_SP4_VFIRST ? w >= 4 : w < 4, role_idx = w & 3;
  {
    const int *sid = reinterpret_cast<const int *>(lf + F_SIMD);
    int per[4] = {0, 0, 0, 0}, rank = 0;
    for (int u = 0; u < 8; ++u) {
      const int su = sid[u];
      if (u < w && su == sid[w]) ++rank;
      per[su & 3]++;
    }
    if (per[0] == 2 && per[1] == 2 && per[2] == 2 && per[3] == 2) {
      is_matrix = XH_SP4_VFIRST ? rank == 1 : rank == 0;
      role_idx = sid[w];
    }
  }
  is_matrix = __builtin_amdgcn_readfirstlane(is_matrix);
  role_idx = __builtin_amdgcn_readfirstlane(role_idx);
  // the end-of-kernel combine of the two envs' partial sums (the images are
  // free after the loop's last barrier)
  float *cmb = reinterpret_cast<float *>(lds + L_GH);

  if (is_matrix) {
    // ======================= matrix waves =================================
    const int s = role_idx;
    const int ot = s & 1, rt = s >> 1;  // layer 2 / SM: o-tile, env
    const int it2 = s >> 1;             // dW2: i-tile (o-tile ot)
    // W2 (S_W) as f16 pairs, A operand of layer 2: lane row o = 32 ot + l31,
    // K-step ks: k = the H1 image's column 16 ks + 8 h + e, which holds
    // feature i = 32 (ks >> 1) + 16 h + 8 (e >> 2) + 4 (ks & 1) + (e & 3)
    // (each vector lane stores its 16 features of a row as two whole chunks)
    f16x8 wl[4][2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const float *row = P + PL.oW2() + (32 * ot + l31) * kH + 32 * (ks >> 1) + 16 * h + 4 * (ks & 1);
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
    // lane bases: layer 2's B operand (H1 image rows of env rt), dW2's A
    // operand (mask image, transposed reads) and B operand (g (x) H1 image,
    // lane column i = 32 it2 + l31, row reads), the mask stores from layer
    // 2's C layout (lane row r = 32 rt + l31, o = 32 ot + 8 q + 4 h ..)
    const int rbH0 = opaque(rd_base(32 * rt + l31, 0, h, kNY) + L_H1),
              rbH1 = opaque(rd_base(32 * rt + l31, 1, h, kNY) + L_H1);
    const int trM0 = opaque(tr_base(l, 0) + L_MK), trM1 = opaque(tr_base(l, 1) + L_MK);
    const int rbg0 = rd_base(32 * it2 + l31, 0, h, kNY) + L_GH,
              rbg1 = rd_base(32 * it2 + l31, 1, h, kNY) + L_GH;
    int mwb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      mwb[q] = opaque(wr_base(32 * rt + l31, q, h, kNY) + 1024 * ot + L_MK);

    // layer 2's bias (its accumulator's start) and w3 / S2 of this lane's
    // 16 outputs o = 32 ot + 8 q + 4 h + u, held for the launch
    float b2r[16], w3r[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int o = 32 * ot + 8 * (e >> 2) + 4 * h + (e & 3);
      b2r[e] = P[PL.ob2() + o] * S2;
      w3r[e] = P[PL.ow3() + o] * (1.0f / S2);
    }
    // dW2 in two accumulators (K-steps 0-1 and 2-3 of every group, summed at
    // the write-out: no dependent MFMA chain)
    f32x16s accW2, accW2b;
#pragma unroll
    for (int e = 0; e < 16; ++e) accW2[e] = accW2b[e] = 0.0f;
    float acc3[16], accb2[16], accb3 = 0.0f;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc3[e] = accb2[e] = 0.0f;

    struct Raw {
      int bi, rec;
    };
    // wave 0 stages the rows of a group: raw loads (lane = row: its bin;
    // lanes 0-2 / 3-5 env A's / B's action, old probability, advantage,
    // lanes 6 / 7 their items), the stores into an LDS slot a phase later
    auto stage_load = [&](int j) {
      const size_t g = gindex(j);
      const int lane =
          opaque((int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)));
      const int bins = (int)*reinterpret_cast<const unsigned char *>(a.b.bins + g * 64 + lane);
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
    auto stage_store = [&](const Raw &r, int sl) {
      lf[F_X + sl * 64 + l] = (float)(signed char)(r.bi & 0xff) / (float)kCapacity;
      const int itA = __builtin_amdgcn_readlane(r.rec, 6);
      const int itB = __builtin_amdgcn_readlane(r.rec, 7);
      if (l < 6) lf[F_REC + 8 * sl + (l >= 3 ? 4 + l - 3 : l)] = __int_as_float(r.rec);
      if (l == 6)
        lf[F_REC + 8 * sl + 3] = (signed char)(itA & 0xff) == a.env.item_a[0] ? 1.0f : 0.0f;
      if (l == 7)
        lf[F_REC + 8 * sl + 7] = (signed char)(itB & 0xff) == a.env.item_a[0] ? 1.0f : 0.0f;
    };

    // layer 2 of the group in the H1 image: C[o][r] = S2 (b2 + W2 . H1) for
    // this wave's 32 o (registers) x env rt (lanes), 4 K-steps of three f16
    // MFMAs; the B operand one step ahead (ping-pong); task(k) after MFMA k
    // (two accumulators, K-steps 0-1 and 2-3, their MFMAs interleaved: a
    // dependent 32x32x16 MFMA waits for its predecessor's whole result, so
    // one chain of 12 would expose every MFMA's latency; summed at the end)
    auto layer2 = [&](f32x16s &c, auto &&task) {
      f32x16s c1;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        c[e] = b2r[e];
        c1[e] = 0.0f;
      }
      f16x8 bh[4], bl[4];
      auto ldB = [&](int ks) {
        const int o = ((ks & 1) ? rbH1 : rbH0) + 1024 * (ks >> 1);
        bh[ks] = ld8h(o);
        bl[ks] = ld8h(o + kImg);
      };
      ldB(0);
      ldB(2);
#pragma unroll
      for (int kp = 0; kp < 2; ++kp) {  // K-steps kp (-> c) and 2 + kp (-> c1)
        const int ka = kp, kb = 2 + kp;
        if (kp == 0) {
          ldB(1);
          ldB(3);
        }
        FENCE();
        c = mfma_f16(wl[ka][1], bh[ka], c);  // the three products,
        FENCE();                              // small terms first
        task(6 * kp);
        FENCE();
        c1 = mfma_f16(wl[kb][1], bh[kb], c1);
        FENCE();
        task(6 * kp + 1);
        FENCE();
        c = mfma_f16(wl[ka][0], bl[ka], c);
        FENCE();
        task(6 * kp + 2);
        FENCE();
        c1 = mfma_f16(wl[kb][0], bl[kb], c1);
        FENCE();
        task(6 * kp + 3);
        FENCE();
        c = mfma_f16(wl[ka][0], bh[ka], c);
        FENCE();
        task(6 * kp + 4);
        FENCE();
        c1 = mfma_f16(wl[kb][0], bh[kb], c1);
        FENCE();
        task(6 * kp + 5);
        FENCE();
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) c[e] += c1[e];
    };
    // partial logits of rows 32 rt + l31 over this wave's o -> F_Z
    auto partials = [&](const f32x16s &c) {
      float zq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float z = relu(c[4 * q]) * w3r[4 * q];
#pragma unroll
        for (int u = 1; u < 4; ++u) z = fmaf(relu(c[4 * q + u]), w3r[4 * q + u], z);
        zq[q] = z;
      }
      const float z = add_halves((zq[0] + zq[1]) + (zq[2] + zq[3]));
      if (h == 0) lf[F_Z + 2 * (32 * rt + l31) + ot] = z;
    };
    // softmax + loss gradient of env rt of group gi (partial logits in F_Z)
    // -> gz (row 32 rt + l31, both lane halves), in stages so that they sit
    // in dW2's MFMA slots: stage(0) loads, (1) .. (5) the arithmetic, (6)
    // the o-tile-0 wave stores g, g x -> F_G and sums db3
    float gz = 0.0f;
    struct Sm {
      f32x4 rec;
      f32x2 z;
      float b3, x, ex, se, p, gc, pc, po, Ac;
      int cu;
    } sm;
    auto softmax_stage = [&](int gi, int gpar, bool acc, int stage) {
      const int rs = gi & 3;
      switch (stage) {
        case 0:
          sm.rec = lds4v(lf + F_REC + 8 * rs + 4 * rt);
          sm.b3 = lf[F_B3];
          sm.z = lds2v(lf + F_Z + 2 * (32 * rt + l31));
          sm.x = lf[F_X + rs * 64 + 32 * rt + l31];
          break;
        case 1:
          sm.cu = __builtin_amdgcn_readfirstlane(__float_as_int(sm.rec[0]));
          sm.po = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sm.rec[1])));
          sm.Ac = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sm.rec[2])));
          sm.ex = __expf((sm.z[0] + sm.z[1]) + sm.b3);
          break;
        case 2:
          sm.se = half_sum32(sm.ex);  // the env's 32 rows; lane 31 holds it
          break;
        case 3: {
          const float se = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm.se), 31));
          sm.p = sm.ex * __builtin_amdgcn_rcpf(se);
          break;
        }
        case 4: {
          sm.pc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm.p), sm.cu & 31));
          if (a.algo == kPPO) {
            // clipped_gradient (rl.h:54-74) through softmax_layer::backward
            const float ratio = sm.pc * __builtin_amdgcn_rcpf(sm.po);
            float ce = a.clip_eps;  // the bounds computed here, not held
            asm volatile("" : "+s"(ce));
            const float clipped = fminf(fmaxf(ratio, 1.0f - ce), 1.0f + ce);
            const float ig = fminf(clipped * sm.Ac, ratio * sm.Ac) * -1.0f;
            sm.gc = ig * __builtin_amdgcn_rcpf(sm.pc);
          }
          break;
        }
        case 5:
          if (a.algo == kPPO) {
            gz = ((l31 == sm.cu ? sm.p : 0.0f) - sm.p * sm.pc) * sm.gc;
          } else {
            // softmax_gradient_log (rl.h:45-52) through softmax-xent
            gz = sm.p * sm.Ac;
            if (l31 == sm.cu) gz -= sm.Ac;
          }
          break;
        default:
          if (ot == 0) {
            if (h == 0) {
              float *gv = lf + F_G + 128 * gpar + 32 * rt + opaque(l31);
              gv[0] = gz;
              gv[64] = gz * sm.x;
            }
            if (acc) accb3 += gz;
          }
          // a look-ahead group past the end: its dW3 / db2 terms vanish
          if (!acc) gz = 0.0f;
      }
    };
    // dW3 / db2 sums of layer-2 value e (units of S2; w3 at the write-out)
    auto dw3_e = [&](const f32x16s &c, int e) {
      const float v = c[e];
      const float gm = v > 0.0f ? gz : 0.0f;
      acc3[e] = fmaf(gm, v, acc3[e]);
      accb2[e] += gm;
    };
    // relu masks of block q as 0 / 0x4000 -> slot ms (2.0 as bf16 for dW2
    // and as f16 for dH1; the factor 2 is taken back at the write-outs)
    auto mask_q = [&](const f32x16s &c, int ms, int q) {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      unsigned m[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) m[u] = c[4 * q + u] > 0.0f ? 1u : 0u;
      const u32x2 mm = {(unsigned)__umul24(m[0] | (m[1] << 16), 0x4000u),
                        (unsigned)__umul24(m[2] | (m[3] << 16), 0x4000u)};
      st4(kImg * ms + mwb[q], __builtin_bit_cast(bf16x4, mm));
    };
    // dW2 += M^T (S_H g (x) H1) of the group whose masks are in slot ms:
    // 4 K-steps of 16 rows, three bf16 MFMAs each; A (mask, transposed) and
    // B (the three parts) one step ahead; task(k) after MFMA k
    auto dw2 = [&](int ms, auto &&task) {
      const int mb = kImg * ms;  // (trM holds L_MK)
      bf16x8 A[4], Bv[4][3];
      auto ldB = [&](int ks) {
        const int ob = 1024 * (ks >> 1) + ((ks & 1) ? rbg1 : rbg0);
        Bv[ks][0] = ld8(ob);
        Bv[ks][1] = ld8(ob + kImg);
        Bv[ks][2] = ld8(ob + 2 * kImg);
      };
      auto ldA = [&](int ks) {
        const int o = mb + 1024 * (kNY * ks + ot);
        A[ks] = ldtr(trM0 + o, trM1 + o);
      };
      ldB(0);
      ldA(0);
      ldB(2);
      ldA(2);
#pragma unroll
      for (int kp = 0; kp < 2; ++kp) {  // K-steps kp (-> accW2), 2 + kp (-> accW2b)
        const int ca = kp, cb = 2 + kp;
        if (kp == 0) {
          ldA(1);
          ldB(1);
          ldA(3);
          ldB(3);
        }
        FENCE();
        accW2 = mfma_bf16(A[ca], Bv[ca][2], accW2);
        FENCE();
        task(6 * kp);
        FENCE();
        accW2b = mfma_bf16(A[cb], Bv[cb][2], accW2b);
        FENCE();
        task(6 * kp + 1);
        FENCE();
        accW2 = mfma_bf16(A[ca], Bv[ca][1], accW2);
        FENCE();
        task(6 * kp + 2);
        FENCE();
        accW2b = mfma_bf16(A[cb], Bv[cb][1], accW2b);
        FENCE();
        task(6 * kp + 3);
        FENCE();
        accW2 = mfma_bf16(A[ca], Bv[ca][0], accW2);
        FENCE();
        task(6 * kp + 4);
        FENCE();
        accW2b = mfma_bf16(A[cb], Bv[cb][0], accW2b);
        FENCE();
        task(6 * kp + 5);
        FENCE();
      }
    };
    // B's VALU in dW2's 12 slots: the softmax stages with the mask blocks
    // beside the first four, then the dW3 / db2 sums, three per slot
    auto b_task = [&](const f32x16s &c, int gi, int gpar, bool acc, int k) {
      if (k < 7) softmax_stage(gi, gpar, acc, k);
      if (k < 4) mask_q(c, gpar, k);
      if (k == 6) {
        dw3_e(c, 0);
        dw3_e(c, 1);
      } else if (k >= 7) {
#pragma unroll
        for (int e = 2 + 3 * (k - 7); e < 5 + 3 * (k - 7); ++e)
          if (e < 16) dw3_e(c, e);
      }
    };
    auto no_task = [](int) {};

    // ---- pipeline prologue (barriers as the vector path's)
    f32x16s c;
    // the staging loads run two periods ahead of their stores (a period is
    // short here: one phase would expose the HBM latency at every store):
    // group g's raw words in rr[g & 1]
    Raw rr[2];
    if (s == 0) {
      stage_store(stage_load(0), 0);
      stage_store(stage_load(1), 1);
      stage_store(stage_load(2), 2);
      rr[1] = stage_load(3);
    }
    __syncthreads();  // P1: rows staged          (vector: L1(0))
    __syncthreads();  // P2
    layer2(c, no_task);
    partials(c);
    __syncthreads();  // P3                       (vector: L1(1))
#pragma unroll
    for (int k = 0; k < 12; ++k) b_task(c, 0, 0, true, k);
    __syncthreads();  // P4
    auto period = [&](int j, auto P) {
      constexpr int par = decltype(P)::value;
      SP4_STAMP(a, j, w, l, 0);
      if (s == 0) rr[par] = stage_load(j + 4);  // (group j + 4: rr[(j + 4) & 1])
      // A(j): layer 2 of group j+1, its partial logits after
      layer2(c, no_task);
      partials(c);
      SP4_STAMP(a, j, w, l, 1);
      __syncthreads();
      SP4_STAMP(a, j, w, l, 2);
      // B(j): dW2 of group j with group j+1's softmax, masks and dW3 / db2
      // sums in its MFMA slots; group j+3's rows (loaded a period ago) staged
      if (s == 0) stage_store(rr[par ^ 1], (j + 3) & 3);
      const bool acc = j + 1 < J;
      dw2(par, [&](int k) { b_task(c, j + 1, 1 - par, acc, k); });
      SP4_STAMP(a, j, w, l, 3);
      __syncthreads();
      SP4_STAMP(a, j, w, l, 4);
    };
    for (int j = 0; j < J; j += 2) {
      period(j, Par<0>{});
      if (j + 1 < J) period(j + 1, Par<1>{});
    }

    // ---- write-out (every entry has exactly one producing lane)
    const float rSH = 0.5f / SH;  // (the masks were 2.0)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int o = 32 * ot + 8 * (e >> 2) + 4 * h + (e & 3);
      slab[PL.oW2() + o * kH + 32 * it2 + l31] = ((accW2[e] + accW2b[e]) * rSH) * w3g[o];
    }
    // dW3 / db2 of o = 32 ot + 8 (e >> 2) + 4 h + (e & 3): sums over the 32
    // lanes (rows) of the half, env B's waves hand theirs to env A's
    float s3[16], s2[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      s3[e] = seg_sum<32>(acc3[e]);
      s2[e] = seg_sum<32>(accb2[e]);
    }
    const float v3 = half_sum32(accb3);  // lane 31 (ot == 0 waves)
    if (rt == 1 && l31 == 0) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int o = 32 * ot + 8 * (e >> 2) + 4 * h + (e & 3);
        cmb[2 * o] = s3[e];
        cmb[2 * o + 1] = s2[e];
      }
    }
    if (rt == 1 && ot == 0 && l == 31) cmb[128] = v3;
    __syncthreads();  // (the vector waves' combine barrier)
    if (rt == 0) {
      if (l31 == 0) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int o = 32 * ot + 8 * (e >> 2) + 4 * h + (e & 3);
          slab[PL.ow3() + o] = (s3[e] + cmb[2 * o]) * (1.0f / S2);
          slab[PL.ob2() + o] = (s2[e] + cmb[2 * o + 1]) * w3g[o];
        }
      }
      if (ot == 0 && l == 31) slab[PL.ob3()] = v3 + cmb[128];
    }
  } else {
    // ======================= vector waves =================================
    const int v = role_idx;
    const int it = v & 1, rt = v >> 1;  // i-tile, env
    const int fi = 32 * it + l31;       // this lane's feature i
    // W2' = S_D diag(w3) W2 as f16 pairs, B operand of dH1: lane column i,
    // K-step ks: k = o = 16 ks + 8 h + e
    f16x8 wd[4][2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int o = 16 * ks + 8 * h + e;
        _Float16 x0, x1;
        split2h((P[PL.oW2() + o * kH + fi] * P[PL.ow3() + o]) * SD, x0, x1);
        wd[ks][0][e] = x0;
        wd[ks][1][e] = x1;
      }
    // the exact f32 chain for g (x) H1 and dW1's relu mask: S_H W1's bin
    // column and S_H (b1 + the item's part)
    const float w1a = P[PL.oW1() + fi * kF0] * SH;
    const float wit = P[PL.oW1() + fi * kF0 + kD];
    const float b1v = P[PL.ob1() + fi];
    const float b1a = (b1v + wit * ((float)a.env.item_a[0] / (float)kCapacity)) * SH;
    const float b1b = (b1v + wit * ((float)a.env.item_b[0] / (float)kCapacity)) * SH;
    auto ia_of = [&](int gi) {
      return __builtin_amdgcn_readfirstlane(
                 __float_as_int(lf[F_REC + 8 * (gi & 3) + 4 * rt + 3])) != 0;
    };
    // the layer-1 image (layer 2's f16-pair operand) from the matrix cores:
    // pre[i][r] = sum_k A[i][k] X[k][r], A = S_H [W1[i][0], b1[i], W1[i][1]
    // item_a / cap, W1[i][1] item_b / cap] in three exact bf16 parts, X =
    // [x, 1, is item_a, is item_b] (exact in bf16); K entries 4..15 zero
    bf16x8 w1p[3];
    {
      const float bv[4] = {P[PL.oW1() + fi * kF0], b1v,
                           wit * ((float)a.env.item_a[0] / (float)kCapacity),
                           wit * ((float)a.env.item_b[0] / (float)kCapacity)};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        __bf16 y0, y1, y2;
        split3(h == 0 && e < 4 ? bv[e] * SH : 0.0f, y0, y1, y2);
        w1p[0][e] = y0;
        w1p[1][e] = y1;
        w1p[2][e] = y2;
      }
    }
    // image stores: the g (x) H1 image (lane row i, values r = 32 rt + 8 q
    // + 4 h ..), the H1 image ([r][column]: lane row r = 32 rt + l31, this
    // wave's features i = 32 it + 8 q + 4 h + u at columns 32 it + 16 h + 8
    // (q >> 1) + 4 (q & 1) + u: whole chunks 2 h, 2 h + 1 of column tile it);
    // dH1's A operand (the mask image read as f16, lane row r)
    int vwb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) vwb[q] = opaque(wr_base(fi, q, h, kNY) + 1024 * rt + L_GH);
    int vwH[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
      vwH[j] = opaque(poff(32 * rt + l31, 32 * it + 16 * h + 8 * j, kNY) + L_H1);
    const int rbm0 = opaque(rd_base(32 * rt + l31, 0, h, kNY) + L_MK),
              rbm1 = opaque(rd_base(32 * rt + l31, 1, h, kNY) + L_MK);
    float w0 = 0.0f, sa = 0.0f, sb = 0.0f;

    // B: layer 1 of group gi -> the H1 image (f16 pairs)
    auto layer1 = [&](int gi) {
      const int sl = gi & 3;
      const bool ia = ia_of(gi);
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const float xv = lf[F_X + sl * 64 + 32 * rt + l31];
      const unsigned d0 = __builtin_bit_cast(unsigned, bf16x2{(__bf16)xv, (__bf16)1.0f});
      const unsigned d1 = ia ? 0x00003F80u : 0x3F800000u;
      const bf16x8 X = __builtin_bit_cast(bf16x8, u32x4{h ? 0u : d0, h ? 0u : d1, 0u, 0u});
      f32x16s pre = mfma_bf16(w1p[2], X, f32x16s{});
      pre = mfma_bf16(w1p[1], X, pre);
      pre = mfma_bf16(w1p[0], X, pre);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        // chunk j: blocks q = 2 j, 2 j + 1
        u32x4 hi, lo;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int q = 2 * j + (p >> 1), u = 2 * (p & 1);
          unsigned h2, l2;
          split2h_x2(relu(pre[4 * q + u]), relu(pre[4 * q + u + 1]), h2, l2);
          hi[p] = h2;
          lo[p] = l2;
        }
        st8h(vwH[j], __builtin_bit_cast(f16x8, hi));
        st8h(vwH[j] + kImg, __builtin_bit_cast(f16x8, lo));
      }
    };
    // x0, x1 -> three bf16 parts each, as bf16 pairs (as spec8)
    auto split3_pair = [](float x0, float x1, unsigned &ph, unsigned &pm, unsigned &pl) {
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      auto cvt = [](float a, float b) {
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
    // A(gi): DH -- S_D dH1 = M (S_D W2') for this wave's features and env,
    // 4 K-steps of two f16 MFMAs (A, the f16 mask image, one step ahead) --
    // with, in the MFMA slots, the group's layer-1 values (hk, kept for B's
    // dW1) and S_H g (x) H1 -> the split image: block q of four rows over
    // four sub-slots, two per MFMA slot.  dh stays in registers for B's dW1.
    auto dh_gh = [&](int gi, int gpar, f32x16s &hk, f32x16s &dh) {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const int mb = kImg * gpar;  // (rbm holds L_MK)
      const float *gv = lf + F_G + 128 * gpar + 32 * rt;
      const float *xv = lf + F_X + (gi & 3) * 64 + 32 * rt;
      const float b1 = ia_of(gi) ? b1a : b1b;
      f16x8 A[4];
      auto ldA = [&](int ks) {
        A[ks] = ld8h(((ks & 1) ? rbm1 : rbm0) + mb + 1024 * (ks >> 1));
      };
      f32x4 ring[3][2];  // [block % 3][x, g]: two blocks ahead
      auto ld2 = [&](int q) {
        ring[q % 3][0] = lds4v(xv + 8 * q + 4 * h);
        ring[q % 3][1] = lds4v(gv + 8 * q + 4 * h);
      };
      ld2(0);
      ld2(1);
      float xx[4];
      unsigned ph[2], pm[2], pl[2];
      auto gh_task = [&](int k) {  // k = 0 .. 15: block q = k / 4
        const int q = k >> 2;
        const f32x4(&o)[2] = ring[q % 3];
        switch (k & 3) {
          case 0:
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const float hv = relu(fmaf(o[0][u], w1a, b1));
              hk[4 * q + u] = hv;
              xx[u] = hv * o[1][u];
            }
            if (q + 2 < 4) ld2(q + 2);
            break;
          case 1:
            split3_pair(xx[0], xx[1], ph[0], pm[0], pl[0]);
            break;
          case 2:
            split3_pair(xx[2], xx[3], ph[1], pm[1], pl[1]);
            break;
          default: {
            st4(vwb[q], __builtin_bit_cast(bf16x4, u32x2{ph[0], ph[1]}));
            st4(vwb[q] + kImg, __builtin_bit_cast(bf16x4, u32x2{pm[0], pm[1]}));
            st4(vwb[q] + 2 * kImg, __builtin_bit_cast(bf16x4, u32x2{pl[0], pl[1]}));
          }
        }
      };
      // (two accumulators, K-steps 0-1 and 2-3, interleaved; summed after)
      f32x16s dh1;
      ldA(0);
      ldA(2);
#pragma unroll
      for (int kp = 0; kp < 2; ++kp) {
        const int ka = kp, kb = 2 + kp;
        if (kp == 0) {
          ldA(1);
          ldA(3);
        }
        FENCE();
        if (kp == 0)
          dh = mfma_f16(A[ka], wd[ka][1], f32x16s{});
        else
          dh = mfma_f16(A[ka], wd[ka][1], dh);
        FENCE();
        gh_task(8 * kp);
        gh_task(8 * kp + 1);
        FENCE();
        if (kp == 0)
          dh1 = mfma_f16(A[kb], wd[kb][1], f32x16s{});
        else
          dh1 = mfma_f16(A[kb], wd[kb][1], dh1);
        FENCE();
        gh_task(8 * kp + 2);
        gh_task(8 * kp + 3);
        FENCE();
        dh = mfma_f16(A[ka], wd[ka][0], dh);
        FENCE();
        gh_task(8 * kp + 4);
        gh_task(8 * kp + 5);
        FENCE();
        dh1 = mfma_f16(A[kb], wd[kb][0], dh1);
        FENCE();
        gh_task(8 * kp + 6);
        gh_task(8 * kp + 7);
        FENCE();
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) dh[e] += dh1[e];
    };
    // B(gi): dW1 / db1 / item sums of group gi: d = relu'(H1) dH1; sums
    // d g x, d g (g, g x staged by the matrix waves), two partial sums each
    auto dw1 = [&](int gi, int gpar, const f32x16s &hk, const f32x16s &dh) {
      const float *gv = lf + F_G + 128 * gpar + 32 * rt;
      float a0[2] = {0.0f, 0.0f}, ag[2] = {0.0f, 0.0f};
      f32x4 g4[4], gx4[4];  // every load issued before the first use
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        g4[q] = lds4v(gv + 8 * q + 4 * h);
        gx4[q] = lds4v(gv + 64 + 8 * q + 4 * h);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float m = hk[4 * q + u] > 0.0f ? dh[4 * q + u] : 0.0f;
          a0[u & 1] = fmaf(m, gx4[q][u], a0[u & 1]);
          ag[u & 1] = fmaf(m, g4[q][u], ag[u & 1]);
        }
      }
      w0 += a0[0] + a0[1];
      const float sg = ag[0] + ag[1];
      if (ia_of(gi))
        sa += sg;
      else
        sb += sg;
    };

    f32x16s hk, dh;
    __syncthreads();  // P1: rows staged
    layer1(0);
    __syncthreads();  // P2                       (matrix: L2(0))
    __syncthreads();  // P3
    layer1(1);
    __syncthreads();  // P4                       (matrix: SM(0))
    auto period = [&](int j, auto P) {
      constexpr int par = decltype(P)::value;
      SP4_STAMP(a, j, w, l, 0);
      dh_gh(j, par, hk, dh);
      SP4_STAMP(a, j, w, l, 1);
      __syncthreads();  // A(j)
      SP4_STAMP(a, j, w, l, 2);
      dw1(j, par, hk, dh);
      layer1(j + 2);
      SP4_STAMP(a, j, w, l, 3);
      __syncthreads();  // B(j)
      SP4_STAMP(a, j, w, l, 4);
    };
    for (int j = 0; j < J; j += 2) {
      period(j, Par<0>{});
      if (j + 1 < J) period(j + 1, Par<1>{});
    }

    // ---- write-out: dW1 / db1 of feature fi (the two lane halves hold row
    // subsets, env B's waves hand theirs to env A's; dH1 was in units of
    // S_D, times the masks' 2)
    float tw0 = w0 + __shfl_xor(w0, 32, kWave);
    float va = sa + __shfl_xor(sa, 32, kWave);
    float vb = sb + __shfl_xor(sb, 32, kWave);
    if (rt == 1 && h == 0) {
      cmb[256 + 3 * fi] = tw0;
      cmb[256 + 3 * fi + 1] = va;
      cmb[256 + 3 * fi + 2] = vb;
    }
    __syncthreads();  // (the matrix waves' combine barrier)
    if (rt == 0 && h == 0) {
      tw0 = (tw0 + cmb[256 + 3 * fi]) * (0.5f / SD);
      va = (va + cmb[256 + 3 * fi + 1]) * (0.5f / SD);
      vb = (vb + cmb[256 + 3 * fi + 2]) * (0.5f / SD);
      slab[PL.oW1() + fi * kF0 + 0] = tw0;
      slab[PL.oW1() + fi * kF0 + kD] = va * ((float)a.env.item_a[0] / (float)kCapacity) +
                                       vb * ((float)a.env.item_b[0] / (float)kCapacity);
      slab[PL.ob1() + fi] = va + vb;
    }
  }
}

}  // namespace sp4

hipError_t launch_policy_train_spec4(const PolicyTrainArgs &a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)sp4::policy_train_spec4_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sp4::kLds);
    attr = true;
  }
  hipLaunchKernelGGL(sp4::policy_train_spec4_kernel, dim3(grid), dim3(sp4::kThreads),
                     sp4::kLds, s, a);
  return hipGetLastError();
}

}  // namespace xh
