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

// Sum over aligned segments of S lanes (S a power of two, S <= 64).
template <int S>
__device__ __forceinline__ float seg_sum(float v) {
#pragma unroll
  for (int o = 1; o < S; o <<= 1) v += __shfl_xor(v, o, kWave);
  return v;
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
