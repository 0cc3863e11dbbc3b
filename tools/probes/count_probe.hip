// Micro-probe: does SQ_INSTS_VALU count v_mfma instructions?  Kernel
// mfma_only issues 1024 v_mfma_f32_16x16x32_bf16 per wave and a loop's few
// scalar instructions; valu_only 1024 v_fma_f32 per wave.  Read both kernels'
// SQ_INSTS_VALU / SQ_INSTS_MFMA from one rocprofv3 --pmc pass:
//   hipcc --offload-arch=gfx950 -O3 tools/probes/count_probe.hip -o build/probe_count
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES -d OUT -- build/probe_count
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mfma_only(float *out) {
  const int l = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(0.01f * (l + j));
    b[j] = (__bf16)(0.02f * (l - j));
  }
  f32x4 acc[4] = {};
  for (int it = 0; it < 64; ++it) {
#pragma unroll
    for (int m = 0; m < 16; ++m)
      acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m & 3], 0, 0, 0);
  }
  const f32x4 s = acc[0] + acc[1] + acc[2] + acc[3];
  if (s[0] == 12345.0f) out[threadIdx.x] = s[1];
}

__global__ __launch_bounds__(256) void valu_only(float *out) {
  float x = 1.0f + 1e-3f * threadIdx.x;
  const float c1 = 1.0001f, c2 = 0.5f;
  for (int it = 0; it < 64; ++it) {
#pragma unroll
    for (int m = 0; m < 16; ++m) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(c1), "v"(c2));
  }
  if (x == 12345.0f) out[threadIdx.x] = x;
}

int main() {
  float *d = nullptr;
  if (hipMalloc(&d, 256 * sizeof(float)) != hipSuccess) return 1;
  hipLaunchKernelGGL(mfma_only, dim3(1024), dim3(256), 0, 0, d);
  hipLaunchKernelGGL(valu_only, dim3(1024), dim3(256), 0, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  // 1024 blocks x 4 waves x 1024 instructions of each kind
  printf("expected per kernel: %d instructions of its kind\n", 1024 * 4 * 1024);
  (void)hipFree(d);
  return 0;
}
