// xh_device.h -- device-side building blocks shared by the xylo-hip kernels
// (gfx950 / CDNA4 only: wave64, v_mfma_f32_32x32x2_f32, minstd streams).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xh {

constexpr int kWave = 64;
constexpr int kCapacity = 8;  // bin_packing.h:48 (per dim, all D)

// ------------------------------------------------------------------ RNG ----
// std::minstd_rand0: x <- 16807 x mod (2^31-1) (libstdc++ bits/random.h:1555),
// reduced with the Mersenne identity (no 64-bit division).
__device__ __forceinline__ uint32_t mstd_mulmod(uint32_t x, uint32_t a) {
  uint64_t p = (uint64_t)x * a;
  uint64_t r = (p & 0x7fffffffull) + (p >> 31);
  r = (r & 0x7fffffffull) + (r >> 31);
  return (uint32_t)(r >= 0x7fffffffull ? r - 0x7fffffffull : r);
}
__device__ __forceinline__ uint32_t mstd_next(uint32_t &x) {
  x = mstd_mulmod(x, 16807u);
  return x;
}
// x * a^k mod m: jump a stream k draws ahead.
__device__ __forceinline__ uint32_t mstd_jump(uint32_t x, uint64_t k) {
  uint32_t base = 16807u, acc = 1u;
  while (k) {
    if (k & 1) acc = mstd_mulmod(acc, base);
    base = mstd_mulmod(base, base);
    k >>= 1;
  }
  return mstd_mulmod(x, acc);
}

// std::generate_canonical<double,53>(minstd_rand0): two draws,
// u = ((x1-1) + (x2-1)*R) / double(R*R), R = 2147483646, clamped below 1
// (libstdc++ bits/random.tcc:3348-3380).  No contraction: bit-exact.
__device__ __forceinline__ double canonical(uint32_t &x) {
#pragma clang fp contract(off)
  const double R = 2147483646.0;
  const double R2 = 4611686009837453316.0;  // nearest double to R*R
  double sum = (double)(mstd_next(x) - 1u);
  double hi = (double)(mstd_next(x) - 1u) * R;
  sum = sum + hi;
  double u = sum / R2;
  return u >= 1.0 ? 0x1.fffffffffffffp-1 : u;
}

// ------------------------------------------------------------------ MFMA ---
typedef float f32x16 __attribute__((ext_vector_type(16)));

// D = A(32x2) * B(2x32) + C with A[i=l&31][k=l>>5], B[k=l>>5][j=l&31];
// C/D: col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5).
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Row (m index) held by accumulator register r in lane half h.
__device__ __forceinline__ constexpr int acc_row(int r, int h) {
  return (r & 3) + 8 * (r >> 2) + 4 * h;
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.0f;
  return z;
}

// ----------------------------------------------------------- wave helpers --
__device__ __forceinline__ float wave_shfl(float v, int src) {
  return __shfl(v, src, kWave);
}
__device__ __forceinline__ double wave_shfl_d(double v, int src) {
  return __shfl(v, src, kWave);
}

// The value of lane ^ 32 (v_permlane32_swap, CDNA4): one VALU exchange
// instead of a ds_bpermute round trip through the LDS crossbar.  Inline asm,
// not the builtin: hipcc (ROCm 7.2) sinks the builtin into the branch of a
// `cond ? v : half_swap(v)` select, where half the lanes are inactive and
// the swap reads their unwritten registers (measured: wrong policy
// gradients).  A volatile asm runs exactly where it is written, with every
// lane active; `s_nop 1` is the 2 wait states a VALU write of either operand
// needs before the swap reads it.
__device__ __forceinline__ float half_swap(float v) {
  unsigned a = __float_as_uint(v), b = a;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  // a: lanes 32-63 now hold lanes 0-31's value; b: lanes 0-31 hold 32-63's
  return __uint_as_float((threadIdx.x & 32) ? a : b);
}

// The sums over the four lane groups (rows of 16 lanes) of four values at
// once, for the MFMA C layout's partial dot products (config 2's train
// kernel, policy_split4h_kernels.hip: 0.0700 -> 0.0686 ms per epoch; the
// 8-wave kernels measured slower with it and keep one swap pair per value):
// lane group G returns (v[G] of group 0 + group 1) + (groups 2 + 3) -- the
// bits of two self-swap steps (permlane16 then permlane32) per value, in three
// swaps and three adds instead of eight of each plus the copy each self-swap
// needs.
// v_permlane16_swap exchanges the first operand's odd rows with the second's
// even rows, so after (v0, v1) row 2k holds v0 and row 2k+1 v1, summed over
// rows 2k and 2k+1; v_permlane32_swap (the first operand's upper half with the
// second's lower half) then pairs the two halves.
__device__ __forceinline__ float sum_groups_t(const float (&v)[4]) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[0]), __float_as_uint(v[1]),
                                                  false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[2]), __float_as_uint(v[3]),
                                                  false, false);
  const float s01 = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const float s23 = __uint_as_float(b[0]) + __uint_as_float(b[1]);
  const auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(s01), __float_as_uint(s23),
                                                  false, false);
  return __uint_as_float(c[0]) + __uint_as_float(c[1]);
}
// v + (v of a partner lane) through a DPP lane pattern (a VALU modifier, no
// LDS round trip).
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __int_as_float(
                 __builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over aligned segments of S lanes (S a power of two, S <= 64).  The
// result is bit-identical to the xor butterfly v += shfl_xor(v, o) for
// o = 1, 2, .., S/2: every stage adds the partner's partial sum, and the DPP
// patterns used (quad_perm [1,0,3,2] / [2,3,0,1] = xor 1 / 2, row_half_mirror
// i <-> 7-i, row_mirror i <-> 15-i) pair each lane with a lane holding the
// same partial sum as its xor-4 / xor-8 partner; float addition commutes, so
// every lane of a segment ends with the same bits as the butterfly.  The last
// two stages of a full wave read the four row sums with v_readlane.
template <int S>
__device__ __forceinline__ float seg_sum(float v) {
  if constexpr (S >= 2) v = dpp_add<0xB1>(v);   // quad_perm [1,0,3,2]
  if constexpr (S >= 4) v = dpp_add<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (S >= 8) v = dpp_add<0x141>(v);  // row_half_mirror
  if constexpr (S >= 16) v = dpp_add<0x140>(v); // row_mirror
  if constexpr (S == 32) v += __shfl_xor(v, 16, kWave);
  if constexpr (S == 64) {
    const int b = __float_as_int(v);
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(b, 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(b, 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(b, 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(b, 48));
    v = (r0 + r1) + (r2 + r3);
  }
  return v;
}
// Sum over each lane half (lanes 0-31, 32-63) by DPP only: seg_sum<32>'s
// four in-row stages, then row_bcast15 adds row 0's (row 2's) sum into row 1
// (row 3).  Valid in lanes 16-31 and 48-63, with the bits of the xor
// butterfly (the partner's partial sum is added, float addition commutes).
__device__ __forceinline__ float half_sum32(float v) {
  v = dpp_add<0xB1>(v);
  v = dpp_add<0x4E>(v);
  v = dpp_add<0x141>(v);
  v = dpp_add<0x140>(v);
  // row_bcast15 into rows 1 and 3 only (row_mask 0xA); rows 0 / 2 add 0
  return v + __int_as_float(__builtin_amdgcn_update_dpp(
                 0, __float_as_int(v), 0x142, 0xA, 0xF, false));
}

template <int S>
__device__ __forceinline__ double seg_sum_d(double v) {
#pragma unroll
  for (int o = 1; o < S; o <<= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
// Inclusive prefix sum within aligned segments of S lanes.
template <int S>
__device__ __forceinline__ double seg_scan_d(double v, int lane) {
  const int pos = lane & (S - 1);
#pragma unroll
  for (int o = 1; o < S; o <<= 1) {
    double u = __shfl_up(v, o, kWave);
    if (pos >= o) v += u;
  }
  return v;
}
template <int S>
__device__ __forceinline__ float seg_min(float v) {
#pragma unroll
  for (int o = 1; o < S; o <<= 1) v = fminf(v, __shfl_xor(v, o, kWave));
  return v;
}

// std::discrete_distribution<size_t>(p[0..B)) sampled with canonical u
// (libstdc++ random.tcc:2654-2713): p -> double, normalise by the sum,
// partial sums, last = 1.0, lower_bound(u).  Lane = bin of a B-lane segment
// (`lane` its wave lane).  The tree-ordered sums agree with the sequential
// ones except within rounding of a boundary; there the segment recomputes
// sequentially.  Returns the chosen bin (the same in every lane).
template <int B>
__device__ __forceinline__ int sample_discrete(float p, int lane, double u) {
  const int bin = lane & (B - 1), seg0 = lane - bin;
  const double pd = (double)p;
  const double sd = seg_sum_d<B>(pd);
  double cp = seg_scan_d<B>(pd / sd, lane);
  if (bin == B - 1) cp = 1.0;
  const unsigned long long below = __ballot(cp < u);
  unsigned long long segmask = ~0ull;
  if constexpr (B < 64) segmask = ((1ull << B) - 1ull) << seg0;
  int choice = __popcll(below & segmask);
  const float gap = (float)fabs(cp - u);
  if (seg_min<B>(gap) < 1e-9f) {
    double s2 = 0.0;
    for (int k = 0; k < B; ++k) s2 += (double)__shfl(p, seg0 + k, kWave);
    double acc = 0.0;
    int c2 = B - 1;
    for (int k = 0; k < B; ++k) {
      const double qk = (double)__shfl(p, seg0 + k, kWave) / s2;
      acc = k == 0 ? qk : acc + qk;
      const double cpk = k == B - 1 ? 1.0 : acc;
      if (!(cpk < u) && k < c2) c2 = k;
    }
    choice = c2;
  }
  return choice;
}

// First maximum of v over a B-lane segment (std::ranges::max_element,
// tensor.cc:464-466): ties go to the lowest bin.
template <int B>
__device__ __forceinline__ int seg_argmax_first(float v, int bin) {
  float bv = v;
  int bi = bin;
#pragma unroll
  for (int o = 1; o < B; o <<= 1) {
    const float ov = __shfl_xor(bv, o, kWave);
    const int oi = __shfl_xor(bi, o, kWave);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  return bi;
}

}  // namespace xh
