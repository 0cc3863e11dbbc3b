// spec8_layout.h -- the LDS image layout of the wave-specialised config-3
// train kernel (policy_spec8_kernels.hip), host + device so that
// tests/test_spec8_layout.py can check every address decomposition and the
// bank-conflict claims exhaustively on the CPU (tests/spec8_layout_check.cc).
//
// An image holds an [X][Y] tile of 16-bit values (X rows a multiple of 16, Y
// columns a multiple of 32) in 1 KB blocks of 4 physical 256-byte rows:
//
//   block  = (x >> 4) (Y / 32) + (y >> 5)
//   row R  = 4 block + (x & 3)
//   chunk  = 4 (a ^ b) + (c ^ a),   a = (x >> 2) & 3, b = x & 3, c = (y >> 3) & 3
//   byte   = 256 R + 16 chunk + 2 (y & 7)
//
// (a bijection: b = R & 3, a = (chunk >> 2) ^ b, c = (chunk & 3) ^ a).  The
// kernel touches its images in four patterns, each conflict-free or at the
// store minimum (tests/spec8_layout_check.cc counts them):
//   * 8-byte stores of 4 consecutive y from an MFMA C layout (lane x, 16
//     lanes x = x0 .. x0 + 15 per store group): 2-way, the minimum for 16
//     lanes of one lane half (a bank-32 store group has 8 slots of 8 bytes);
//   * ds_read_b128 row reads of a 32x32x16 operand (lane x, 8 consecutive y):
//     conflict-free;
//   * ds_read_b64_tr_b16 transposed reads of a 32x32x16 operand whose k runs
//     down x: conflict-free.
// The loop-invariant lane part of every address is computed once; what
// varies over a loop (x or y tiles) is a multiple of 1 KB or of 16 bytes that
// does not meet the XOR, so it folds into the ds instructions' immediates.
#pragma once

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace xh {
namespace sp8 {

// byte offset of element (x, y) of an image with ny = Y / 32 column tiles
__host__ __device__ inline int poff(int x, int y, int ny) {
  const int a = (x >> 2) & 3, b = x & 3, c = (y >> 3) & 3;
  return 1024 * ((x >> 4) * ny + (y >> 5)) + 256 * b + 16 * (4 * (a ^ b) + (c ^ a)) +
         2 * (y & 7);
}

// Stores: lane row x, values y = 32 T + 8 q + 4 h .. +3 (h = lane >> 5) at
// wr_base(x, q, h, ny) + 1024 T (x's 16-row block included).
__host__ __device__ inline int wr_base(int x, int q, int h, int ny) {
  const int a = (x >> 2) & 3, b = x & 3;
  return 1024 * ny * (x >> 4) + 256 * b + 64 * (a ^ b) + 16 * (q ^ a) + 8 * h;
}

// Row reads of a 32x32x16 operand, lane row x, K-step ks (y = 16 ks + 8 h ..
// + 7): rd_base(x, ks & 1, h, ny) + 1024 (ks >> 1).
__host__ __device__ inline int rd_base(int x, int m, int h, int ny) {
  const int a = (x >> 2) & 3, b = x & 3;
  return 1024 * ny * (x >> 4) + 256 * b + 64 * (a ^ b) + 16 * ((2 * m + h) ^ a);
}

// Transposed reads (ds_read_b64_tr_b16) of a 32x32x16 operand whose k runs
// down x: lane l's fragment element e = 4 n + j is x = 16 ks + 8 h + 4 n + j
// of column tile T (y = 32 T + (l & 31)).  Read n: lane 4 q + p of 16-lane
// group g supplies the address of x = 16 ks + 8 h + 4 n + q, y = 32 T +
// 16 (g & 1) + 4 p .. +3, which is tr_base(l, n) + 1024 (ks ny + T).
__host__ __device__ inline int tr_base(int l, int n) {
  const int g = l >> 4, q = (l & 15) >> 2, p = l & 3, h = l >> 5;
  const int a = 2 * h + n, c = 2 * (g & 1) + (p >> 1);
  return 256 * q + 64 * (a ^ q) + 16 * (c ^ a) + 8 * (p & 1);
}

}  // namespace sp8
}  // namespace xh
