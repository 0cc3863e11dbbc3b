// xh_split.h -- f32 GEMMs on the bf16 matrix cores of gfx950 at f32 accuracy.
//
// gfx950 runs f32-input MFMA (v_mfma_f32_32x32x2_f32) at 64 FLOP/clk/SIMD,
// 1/16 of its bf16 rate (v_mfma_f32_32x32x16_bf16: 32x32x16 in 32 cycles).
// An f32 value splits EXACTLY into three bf16 parts,
//     x = hi + mid + lo + e,   hi = bf16(x), mid = bf16(x - hi),
//     lo = bf16(x - hi - mid), |e| <= 2^-24 |x|
// (each difference is exact by Sterbenz; 8 significand bits per part), and a
// product of two bf16 values is exact in f32.  A dot product then is
//     a.b = hi.hi + (hi.mid + mid.hi) + (hi.lo + lo.hi + mid.mid) + d,
//     |d| <= (2^-23 + 2^-22) sum|a_k b_k|
// (the dropped mid.lo + lo.mid + lo.lo and the two e terms), i.e. six bf16
// MFMAs per K=16 slice (192 cycles) in place of eight f32 ones (512 cycles).
// Against an f32 fmaf chain over K terms, whose worst-case error is
// (K-1) 2^-24 sum|a_k b_k|, the bound is tighter from K = 8 on (the MFMA
// adds each instruction's 16 exact products into the f32 accumulator).
//
// Operand images in LDS: [rows][128 x bf16] (256-byte rows), one image per
// part, 16-byte chunks XOR-swizzled so that both the ds_read_b128 row reads
// (an operand whose k runs along the row) and the ds_read_b64_tr_b16
// transposed reads (k runs down the rows) of a 32x32x16 operand are
// bank-conflict-free (cdna_hip_programming.md T10, layout (b)).
#pragma once
#include <hip/hip_runtime.h>

namespace xh {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16s __attribute__((ext_vector_type(16)));

constexpr int kImgRow = 256;  // bytes per image row (128 bf16)

// Byte offset of 16-byte chunk ch (0..15) of row `row`.
__device__ __forceinline__ int img_off(int row, int ch) {
  return kImgRow * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// x -> hi + mid + lo (bf16, round to nearest even); the differences are
// exact in f32.
__device__ __forceinline__ void split3(float x, __bf16 &h, __bf16 &m, __bf16 &l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  const float r2 = r1 - (float)m;
  l = (__bf16)r2;
}

// 32x32x16 bf16 MFMA: lane l (r = l&31, h = l>>5) holds A[r][8h+j] and
// B[8h+j][r] in element j; C/D as the f32 forms (col = l&31, acc_row).
__device__ __forceinline__ f32x16s mfma_bf16(bf16x8 a, bf16x8 b, f32x16s c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// The six products of a split pair into acc (small terms first, the
// hi.hi term last).
__device__ __forceinline__ f32x16s mfma_split6(const bf16x8 (&a)[3],
                                               const bf16x8 (&b)[3],
                                               f32x16s c) {
  c = mfma_bf16(a[1], b[1], c);
  c = mfma_bf16(a[0], b[2], c);
  c = mfma_bf16(a[2], b[0], c);
  c = mfma_bf16(a[0], b[1], c);
  c = mfma_bf16(a[1], b[0], c);
  c = mfma_bf16(a[0], b[0], c);
  return c;
}

// An operand that is exact in bf16 (e.g. a 0/1 mask) times a split one:
// three products, error <= 2^-24 sum|a_k b_k| (the split's e term only).
__device__ __forceinline__ f32x16s mfma_split3(bf16x8 a, const bf16x8 (&b)[3],
                                               f32x16s c) {
  c = mfma_bf16(a, b[2], c);
  c = mfma_bf16(a, b[1], c);
  c = mfma_bf16(a, b[0], c);
  return c;
}

// Row read: the 8 bf16 of chunk ch of row `row` of an image.
__device__ __forceinline__ bf16x8 img_row8(const char *img, int row, int ch) {
  return *reinterpret_cast<const bf16x8 *>(img + img_off(row, ch));
}

// Transposed read of a 32x32x16 operand whose k runs down the image rows:
// lane l gets column c0 + (l&31) of rows k0 + 8h .. k0 + 8h + 7 (h = l>>5),
// element j = row k0 + 8h + j.  c0 is a multiple of 32.  Two
// ds_read_b64_tr_b16: per 16-lane group g, lane 4q+p supplies the address of
// row (k0 + 8h + 4t + q), columns c0 + 16(g&1) + 4p .. +3.  EXEC must be
// full (every lane of the wave executes this).  l = the lane id (a caller
// may pass an opaque copy so the address arithmetic is not hoisted).
__device__ __forceinline__ bf16x8 img_tr8(const char *img, int k0, int c0,
                                          int l = threadIdx.x & 63) {
  const int g = l >> 4, li = l & 15;
  const int q = li >> 2, p = li & 3, h = l >> 5;
  const int ch = (c0 >> 3) + 2 * (g & 1) + (p >> 1);
  const int boff = 8 * (p & 1);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int r0 = k0 + 8 * h + q;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4 *)(img + img_off(r0, ch) + boff));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4 *)(img + img_off(r0 + 4, ch) + boff));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// ---- Immediate-offset addressing of the same images.  The XOR swizzle
// touches only address bits 4-7, so a per-lane base computed once turns every
// read into at most one v_xor plus the ds_read's immediate offset.
__device__ __forceinline__ int img_swz(int row) {
  return ((row & 3) << 2) | ((row >> 2) & 3);
}
// Row reads of row R in lane half h: chunk 2s + h of the row is at
// row_base(R, h) ^ (32 s).
__device__ __forceinline__ int row_base(int R, int h) {
  return kImgRow * R + 16 * (h ^ img_swz(R));
}
__device__ __forceinline__ bf16x8 ld_row(const char *img, int base, int s) {
  return *reinterpret_cast<const bf16x8 *>(img + (base ^ (32 * s)));
}
// Transposed reads (img_tr8's element order): for lane l and half-fragment t,
// row 8h + 4t + q of the K-slice and chunk 2(g&1) + (p>>1) of the column
// tile; the swizzle of rows 16s + .. does not depend on s, and column tile n
// XORs bits 6-7: operand (k0 = 16 s, c0 = 32 n) = tr_base ^ (64 n), + 4096 s.
__device__ __forceinline__ int tr_base(int l, int t) {
  const int g = l >> 4, li = l & 15, q = li >> 2, p = li & 3, h = l >> 5;
  const int cl = 2 * (g & 1) + (p >> 1);
  const int B = 4 * q + (cl ^ (2 * h + t));
  return kImgRow * (8 * h + 4 * t + q) + 16 * B + 8 * (p & 1);
}
// b0 / b1: tr_base(l, 0 / 1) ^ (64 n) of the column tile
__device__ __forceinline__ bf16x8 ld_tr(const char *img, int b0, int b1, int s) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4 *)(img + b0 + 4096 * s));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4 *)(img + b1 + 4096 * s));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// Stores of img_store_split: row R's chunk cg, lane half h's 8 bytes at
// st_base(R, h) ^ (16 cg).
__device__ __forceinline__ int st_base(int R, int h) {
  return kImgRow * R + 16 * img_swz(R) + 8 * h;
}
__device__ __forceinline__ void img_store_split_b(char *img_hi, char *img_mid,
                                                  char *img_lo, int base, int c0,
                                                  const f32x16s &v) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    bf16x4 ph, pm, pl;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      __bf16 a, b, c;
      split3(v[4 * g + u], a, b, c);
      ph[u] = a;
      pm[u] = b;
      pl[u] = c;
    }
    const int off = base ^ (16 * ((c0 >> 3) + g));
    *reinterpret_cast<bf16x4 *>(img_hi + off) = ph;
    *reinterpret_cast<bf16x4 *>(img_mid + off) = pm;
    *reinterpret_cast<bf16x4 *>(img_lo + off) = pl;
  }
}

// Write a 32x32 f32 tile held in MFMA C layout (lane col = image row
// `row`, register j = feature c0 + acc_row(j, h)) as its three bf16 parts
// into three images: registers 4g..4g+3 are 4 consecutive features
// c0 + 8g + 4h .. +3, one 8-byte store per part.
__device__ __forceinline__ void img_store_split(char *img_hi, char *img_mid,
                                                char *img_lo, int row, int c0,
                                                const f32x16s &v) {
  const int h = (threadIdx.x & 63) >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    bf16x4 ph, pm, pl;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      __bf16 a, b, c;
      split3(v[4 * g + u], a, b, c);
      ph[u] = a;
      pm[u] = b;
      pl[u] = c;
    }
    const int off = img_off(row, (c0 >> 3) + g) + 8 * h;
    *reinterpret_cast<bf16x4 *>(img_hi + off) = ph;
    *reinterpret_cast<bf16x4 *>(img_mid + off) = pm;
    *reinterpret_cast<bf16x4 *>(img_lo + off) = pl;
  }
}

// ---- f16 pairs (policy_split8wh / 8x / 4h_kernels.hip, the split
// rollouts): an operand with a bound known before the kernel is scaled by a
// power of two S (|S x| <= 2^14, f16's range ends at 65504) and split EXACTLY
// into two f16 parts,
//     S x = hi + lo + e,  hi = f16(S x), lo = f16(S x - hi)
// (11 significant bits per part, round to nearest; S x - hi is exact).  The
// error e is lo's rounding:
//     |e| <= max(2^-22 |S x|, 2^-25)
// -- relative while lo is a normal f16 (|S x - hi| >= 2^-14, which holds for
// |S x| >= 2^-3, i.e. within 2^17 of the launch's bound), an absolute 2^-25
// (half of f16's subnormal spacing 2^-24) below that.  A product of two f16
// values is exact in f32, so a dot product is
//     (S_a a).(S_b b) = hi.hi + hi.lo + lo.hi + d,
//     |d| <= 3 2^-22 sum|S_a a_k S_b b_k| + 2^-25 sum(|S_a a_k| + |S_b b_k|)
// (the dropped lo.lo and the two e terms, in scaled units):
// three f16 MFMAs per K slice in place of the bf16 split's six, two against
// an operand exact in f16 (a 0/1 mask) in place of three.  f16 and bf16
// MFMAs run at the same rate.  The result is in units of S_a S_b and is
// unscaled exactly (a power of two).  An entry 2^20 below its launch's bound
// keeps about 19 significant bits instead of 24: tests/test_gpu_range.py
// puts parts of the policy 2^20 below the rest and holds the tight gradient
// budget (median <= 1, p99 <= 100 units of u sum|terms|; measured p99 <= 13
// at config 3, <= 50 at config 5).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split2h(float x, _Float16 &hi, _Float16 &lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}
// split2h of (a0 s, a1 s), packed, for a power-of-two s (a s exact in f32):
// hi by v_fma_mixlo / mixhi_f16 (a s + 0 rounded once to f16: the same as
// converting the f32 product), lo as split2h_x2; four instructions per pair,
// writing both halves of each word (no packing afterwards)
__device__ __forceinline__ void split2h_x2s(float a0, float a1, float s, unsigned &hi2,
                                            unsigned &lo2) {
  asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(hi2) : "v"(a0), "v"(s));
  asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(hi2) : "v"(a1), "v"(s));
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(lo2) : "v"(a0), "v"(s), "v"(hi2));
  asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "+v"(lo2)
      : "v"(a1), "v"(s), "v"(hi2));
}
// split2h of two values, packed: hi2 = {hi(x0), hi(x1)} (v_cvt_pk_f16_f32,
// round to nearest), lo2 = {lo(x0), lo(x1)} by v_fma_mixlo / mixhi_f16:
// x * 1 - hi with hi read as f16 (op_sel_hi) is exact in f32 and rounded once
// to f16, the same lo as split2h, in one instruction per value instead of a
// convert back, a subtract and a convert (the compiler does not form the mix
// from the subtract)
__device__ __forceinline__ void split2h_x2(float x0, float x1, unsigned &hi2,
                                           unsigned &lo2) {
  typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
  hi2 = __builtin_bit_cast(unsigned, f16x2_t{(_Float16)x0, (_Float16)x1});
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(lo2) : "v"(x0), "v"(hi2));
  asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "+v"(lo2)
      : "v"(x1), "v"(hi2));
}
// 2^(14 - e) for a maximum m <= 2^e (frexp); e clamped so that products of
// two scales and their inverses stay normal f32
__device__ __forceinline__ float f16_scale_for(float m) {
  int e = 0;
  (void)frexpf(m, &e);
  e = min(max(e, -40), 40);
  return ldexpf(1.0f, 14 - e);
}
__device__ __forceinline__ f32x16s mfma_f16(f16x8 a, f16x8 b, f32x16s c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// acc + f16(half of w) * g in one v_fma_mix_f32 (the f16 operand read from the
// low / high half of w): a relu-mask word's 0 / 0x4000 (2.0) half times g,
// i.e. db2's masked sum 2 g M without a compare or a select
__device__ __forceinline__ float fma_mix_lo(unsigned w, float g, float acc) {
  asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(w), "v"(g));
  return acc;
}
__device__ __forceinline__ float fma_mix_hi(unsigned w, float g, float acc) {
  asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "+v"(acc)
      : "v"(w), "v"(g));
  return acc;
}
// the bits of a bf16 0/1 operand as f16 (1.0 = 0x3F80 -> 0x3C00)
__device__ __forceinline__ f16x8 mask_bf16_to_f16(bf16x8 m) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(f16x8, __builtin_bit_cast(u32x4, m) & 0x3C003C00u);
}
// A 32x32 f32 tile in MFMA C layout (as img_store_split_b), times S, as two
// f16 part images
__device__ __forceinline__ void img_store_h2(char *img_hi, char *img_lo, int base,
                                             int c0, const f32x16s &v, float S) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    f16x4 ph, pl;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      _Float16 a, b;
      split2h(v[4 * g + u] * S, a, b);
      ph[u] = a;
      pl[u] = b;
    }
    const int off = base ^ (16 * ((c0 >> 3) + g));
    *reinterpret_cast<f16x4 *>(img_hi + off) = ph;
    *reinterpret_cast<f16x4 *>(img_lo + off) = pl;
  }
}

// ---- helpers of the split train kernels (variants/policy_split_kernels.hip,
// variants/policy_split128_kernels.hip)
namespace split {

__device__ __forceinline__ float relu(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}
__device__ __forceinline__ float4 lds4(const float *p) {
  return *reinterpret_cast<const float4 *>(p);
}
// 16 f32 of C-layout register order from 4 consecutive-feature quads of an
// LDS vector: register 4g + u = v[c0 + 8g + 4h + u]
__device__ __forceinline__ f32x16s lds_acc16(const float *v, int c0, int h) {
  f32x16s r;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 b = lds4(v + c0 + 8 * g + 4 * h);
    r[4 * g + 0] = b.x;
    r[4 * g + 1] = b.y;
    r[4 * g + 2] = b.z;
    r[4 * g + 3] = b.w;
  }
  return r;
}

}  // namespace split

}  // namespace xh
