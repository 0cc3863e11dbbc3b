// Micro-probe: does VALU work hide under MFMAs on MI355X?  Per block each
// wave issues 96 v_mfma_f32_16x16x32_bf16 (or 48 v_mfma_f32_32x32x16_bf16:
// the same matrix-pipe cycles) and 96 K independent v_fma_f32, either as an
// MFMA block then a VALU block, or interleaved (1 MFMA : K VALU), at two
// waves per SIMD (512-thread blocks) or one (256).  Prints cycles per block.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/interleave_probe.hip -o build/probe_il
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// an opaque v_fma_f32 (the compiler can neither fold nor move it)
__device__ __forceinline__ void vfma(float &x, float a, float b) {
  asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
}

template <int MODE, int K, int BIG>
__global__ __launch_bounds__(512) void probe(float *out, long long *cyc, int iters) {
  const int l = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.01f * (l + j)); b[j] = (__bf16)(0.02f * (l - j)); }
  f32x4 acc[4] = {};
  f32x16 acc2[2] = {};
  float v[8];
  for (int j = 0; j < 8; ++j) v[j] = 1.0f + 0.001f * (l + j);
  const float c1 = 1.0001f + 1e-9f * l, c2 = 0.5f;
  constexpr int NM = BIG ? 48 : 96;   // MFMAs per block
  constexpr int KV = BIG ? 2 * K : K;  // VALU per MFMA (same VALU per block)
  __syncthreads();
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      if (MODE == 0 || MODE == 2 || MODE == 3) {
        if (BIG)
          acc2[m & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc2[m & 1], 0, 0, 0);
        else
          acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m & 3], 0, 0, 0);
      }
      if (MODE == 3) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < KV; ++k) vfma(v[(m * KV + k) & 7], c1, c2);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (MODE == 1 || MODE == 2) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 96 * K; ++k) vfma(v[k & 7], c1, c2);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
  }
  long long t1 = clock64();
  float s = 0;
  for (int j = 0; j < 8; ++j) s += v[j];
  for (int r = 0; r < 4; ++r) s += acc[r][0] + acc[r][1] + acc[r][2] + acc[r][3];
  for (int r = 0; r < 2; ++r) s += acc2[r][0] + acc2[r][5];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = (t1 - t0) / iters;
}

template <int MODE, int K, int BIG>
void run(const char *name, int threads, float *out, long long *cyc) {
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((probe<MODE, K, BIG>), dim3(256), dim3(threads), 0, 0, out, cyc, 200);
  (void)hipDeviceSynchronize();
  long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-9s %-22s waves/SIMD=%d K=%d  %5lld cycles per block\n",
         BIG ? "32x32x16" : "16x16x32", name, threads / 256, K, c);
}

template <int BIG>
void all(int threads, float *out, long long *cyc) {
  run<0, 1, BIG>("mfma only", threads, out, cyc);
  run<1, 2, BIG>("valu only", threads, out, cyc);
  run<2, 2, BIG>("mfma block then valu", threads, out, cyc);
  run<3, 1, BIG>("interleaved", threads, out, cyc);
  run<3, 2, BIG>("interleaved", threads, out, cyc);
}

int main() {
  float *out;
  long long *cyc;
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&cyc, 8);
  all<0>(512, out, cyc);
  all<1>(512, out, cyc);
  all<0>(256, out, cyc);
  all<1>(256, out, cyc);
  return 0;
}
