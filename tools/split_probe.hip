// split_probe.hip -- checks the bf16-split GEMM building blocks of xh_split.h
// on the device: the 32x32x16 bf16 operand maps through row reads and
// ds_read_b64_tr_b16 transposed reads of the swizzled images (exact integer
// data: every product and sum exact, the result must equal the host's), and
// the accuracy of the six- and nine-product split against a double reference
// beside the f32 MFMA (v_mfma_f32_32x32x2_f32 chain).
//   hipcc --offload-arch=gfx950 -O3 -I dependence_free_rl_amd/csrc \
//         tools/split_probe.hip -o build/split_probe && build/split_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "xh_device.h"
#include "xh_split.h"

using namespace xh;

constexpr int NR = 64, NC = 128;  // each input matrix [64][128] f32

// images: 3 matrices x 3 parts of [64][256 B]
__global__ __launch_bounds__(64) void probe_kernel(const float *W, const float *X,
                                                   const float *Y, float *out,
                                                   int mode) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x, lr = lane & 31, h = lane >> 5;
  char *img[3][3];
  for (int m = 0; m < 3; ++m)
    for (int p = 0; p < 3; ++p) img[m][p] = lds + (m * 3 + p) * NR * kImgRow;
  const float *src[3] = {W, X, Y};
  for (int m = 0; m < 3; ++m)
    for (int e = lane; e < NR * NC; e += 64) {
      const int row = e / NC, col = e % NC;
      __bf16 a, b, c;
      split3(src[m][e], a, b, c);
      const int off = img_off(row, col >> 3) + 2 * (col & 7);
      *reinterpret_cast<__bf16 *>(img[m][0] + off) = a;
      *reinterpret_cast<__bf16 *>(img[m][1] + off) = b;
      *reinterpret_cast<__bf16 *>(img[m][2] + off) = c;
    }
  __syncthreads();
  auto prod = [&](const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16s c) {
    c = mfma_split6(a, b, c);
    if (mode == 9) {
      c = mfma_bf16(a[1], b[2], c);
      c = mfma_bf16(a[2], b[1], c);
      c = mfma_bf16(a[2], b[2], c);
    }
    return c;
  };
  // C1[o][r] = sum_i W[o][i] X[r][i], o in 32..63, r in 32..63
  f32x16s c1 = {};
  for (int s = 0; s < 8; ++s) {
    bf16x8 a[3], b[3];
    for (int p = 0; p < 3; ++p) {
      a[p] = img_row8(img[0][p], 32 + lr, 2 * s + h);
      b[p] = img_row8(img[1][p], 32 + lr, 2 * s + h);
    }
    c1 = prod(a, b, c1);
  }
  // C2[o][i] = sum_r Y[r][o] X[r][i], o in 32..63, i in 64..95
  f32x16s c2 = {};
  for (int s = 0; s < 4; ++s) {
    bf16x8 a[3], b[3];
    for (int p = 0; p < 3; ++p) {
      a[p] = img_tr8(img[2][p], 16 * s, 32);
      b[p] = img_tr8(img[1][p], 16 * s, 64);
    }
    c2 = prod(a, b, c2);
  }
  // C3[i][r] = sum_{o<64} W[o][i] Y[r][o], i in 96..127, r in 32..63
  f32x16s c3 = {};
  for (int s = 0; s < 4; ++s) {
    bf16x8 a[3], b[3];
    for (int p = 0; p < 3; ++p) {
      a[p] = img_tr8(img[0][p], 16 * s, 96);
      b[p] = img_row8(img[2][p], 32 + lr, 2 * s + h);
    }
    c3 = prod(a, b, c3);
  }
  // C1 by the f32 MFMA chain (k = 2s + h), operands from global memory
  f32x16 c4 = zero16();
  for (int s = 0; s < 64; ++s)
    c4 = mfma32(W[(32 + lr) * NC + 2 * s + h], X[(32 + lr) * NC + 2 * s + h], c4);
  // C2 also through img_store_split: X tile (rows 0..31 = C layout col) ->
  // a fresh image, read back by rows: must equal the split of the source
  char *tst[3] = {img[2][0], img[2][1], img[2][2]};  // Y images reused
  __syncthreads();
  f32x16s xv;
  for (int j = 0; j < 16; ++j) xv[j] = X[lr * NC + 32 + acc_row(j, h)];
  img_store_split(tst[0], tst[1], tst[2], lr, 32, xv);
  __syncthreads();
  float rt = 0.0f;  // row 'lane&31' features 32..63 reassembled
  for (int ch = 4; ch < 8; ++ch)
    for (int u = 0; u < 8; ++u) {
      const int off = img_off(lr, ch) + 2 * u;
      const float v = ((float)*reinterpret_cast<__bf16 *>(tst[0] + off) +
                       (float)*reinterpret_cast<__bf16 *>(tst[1] + off)) +
                      (float)*reinterpret_cast<__bf16 *>(tst[2] + off);
      const float x = X[lr * NC + ch * 8 + u];
      rt += fabsf(v - x);
    }
  for (int j = 0; j < 16; ++j) {
    const int row = acc_row(j, h);
    out[0 * 1024 + row * 32 + lr] = c1[j];
    out[1 * 1024 + row * 32 + lr] = c2[j];
    out[2 * 1024 + row * 32 + lr] = c3[j];
    out[3 * 1024 + row * 32 + lr] = c4[j];
  }
  if (h == 0) out[4 * 1024 + lr] = rt;
}

static double urand(unsigned &s) {
  s = s * 1664525u + 1013904223u;
  return ((s >> 8) & 0xffffff) / 16777216.0;
}

int main() {
  std::vector<float> W(NR * NC), X(NR * NC), Y(NR * NC), out(5 * 1024);
  float *dW, *dX, *dY, *dO;
  hipMalloc(&dW, NR * NC * 4);
  hipMalloc(&dX, NR * NC * 4);
  hipMalloc(&dY, NR * NC * 4);
  hipMalloc(&dO, 5 * 1024 * 4);
  const size_t lds = 9 * NR * kImgRow;
  hipFuncSetAttribute((const void *)probe_kernel,
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int fails = 0;
  for (int trial = 0; trial < 3; ++trial) {
    unsigned s = 12345u + trial;
    const bool integer = trial == 0;
    for (int i = 0; i < NR * NC; ++i) {
      if (integer) {
        W[i] = (float)((int)(urand(s) * 17) - 8);
        X[i] = (float)((int)(urand(s) * 13) - 6);
        Y[i] = (float)((int)(urand(s) * 11) - 5);
      } else {  // wide dynamic range, both signs
        const double e = std::pow(2.0, (int)(urand(s) * 20) - 10);
        W[i] = (float)((urand(s) - 0.5) * e);
        X[i] = (float)((urand(s) - 0.5) * std::pow(2.0, (int)(urand(s) * 20) - 10));
        Y[i] = (float)((urand(s) - 0.5) * std::pow(2.0, (int)(urand(s) * 8) - 4));
      }
    }
    hipMemcpy(dW, W.data(), NR * NC * 4, hipMemcpyHostToDevice);
    hipMemcpy(dX, X.data(), NR * NC * 4, hipMemcpyHostToDevice);
    hipMemcpy(dY, Y.data(), NR * NC * 4, hipMemcpyHostToDevice);
    for (int mode : {6, 9}) {
      hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), lds, 0, dW, dX, dY, dO, mode);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("launch failed\n");
        return 2;
      }
      hipMemcpy(out.data(), dO, 5 * 1024 * 4, hipMemcpyDeviceToHost);
      double worst[4] = {0, 0, 0, 0};
      for (int m = 0; m < 32; ++m)
        for (int n = 0; n < 32; ++n) {
          double ref[4] = {0, 0, 0, 0}, mag[4] = {0, 0, 0, 0};
          for (int k = 0; k < NC; ++k) {
            const double t = (double)W[(32 + m) * NC + k] * X[(32 + n) * NC + k];
            ref[0] += t; mag[0] += std::fabs(t);
          }
          for (int r = 0; r < NR; ++r) {
            const double t = (double)Y[r * NC + 32 + m] * X[r * NC + 64 + n];
            ref[1] += t; mag[1] += std::fabs(t);
            const double u = (double)W[r * NC + 96 + m] * Y[(32 + n) * NC + r];
            ref[2] += u; mag[2] += std::fabs(u);
          }
          ref[3] = ref[0]; mag[3] = mag[0];
          for (int t = 0; t < 4; ++t) {
            const double e = std::fabs(out[t * 1024 + m * 32 + n] - ref[t]) /
                             (mag[t] > 0 ? mag[t] : 1.0);
            if (e > worst[t]) worst[t] = e;
          }
        }
      double rt = 0;
      for (int i = 0; i < 32; ++i) rt += out[4 * 1024 + i];
      printf("trial %d (%s) split%d: max |err|/sum|ab| rowread %.3g tr.tr %.3g "
             "tr.row %.3g | f32 MFMA %.3g | store_split roundtrip %.3g\n",
             trial, integer ? "integer" : "random", mode, worst[0], worst[1],
             worst[2], worst[3], rt);
      if (integer && (worst[0] || worst[1] || worst[2] || worst[3] || rt)) ++fails;
      if (!integer && (worst[0] > 1e-6 || worst[1] > 1e-6 || worst[2] > 1e-6 || rt))
        ++fails;
    }
  }
  printf(fails ? "FAIL\n" : "PASS\n");
  return fails ? 1 : 0;
}
