// Micro-probe: the cost of a dependent MFMA chain on gfx950.  One wave per
// SIMD (256-thread blocks, one per CU) issues NM v_mfma_f32_32x32x16_f16 per
// iteration into DIST accumulators in turn (DIST = 1: every MFMA reads the
// previous one's result as its C operand; 2, 3, 4: the chain distance), with
// and without FILL independent v_fma_f32 between MFMAs (the VALU "slot" the
// train kernels fill).  Cycles per MFMA tell how much of an MFMA's latency a
// chain of distance DIST exposes (spec4 / spec8 phase design).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/chain_probe.hip -o build/probe_chain
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void vfma(float &x, float a, float b) {
  asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
}

template <int DIST, int NM, int FILL>
__global__ __launch_bounds__(256) void probe(float *out, long long *cyc, int iters) {
  const int l = threadIdx.x & 63;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)(0.01f * (l + j));
    b[j] = (_Float16)(0.02f * (l - j));
  }
  f32x16 acc[4] = {};
  float v[4] = {1.0f, 1.1f, 1.2f, 1.3f};
  const float c1 = 1.0001f + 1e-9f * l, c2 = 0.5f;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      acc[m % DIST] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[m % DIST], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < FILL; ++k) vfma(v[k & 3], c1, c2);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  long long t1 = clock64();
  float s = v[0] + v[1] + v[2] + v[3];
  for (int r = 0; r < 4; ++r) s += acc[r][0] + acc[r][7];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = (t1 - t0) / iters;
}

template <int DIST, int NM, int FILL>
void run(float *out, long long *cyc) {
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((probe<DIST, NM, FILL>), dim3(256), dim3(256), 0, 0, out, cyc, 100);
  (void)hipDeviceSynchronize();
  long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("32x32x16 f16  chain distance %d  %2d VALU between MFMAs: %6lld cycles per %d MFMAs "
         "(%.1f per MFMA)\n", DIST, FILL, c, NM, (double)c / NM);
}

int main() {
  float *out;
  long long *cyc;
  (void)hipMalloc(&out, 256 * 256 * 4);
  (void)hipMalloc(&cyc, 8);
  run<1, 48, 0>(out, cyc);
  run<2, 48, 0>(out, cyc);
  run<3, 48, 0>(out, cyc);
  run<4, 48, 0>(out, cyc);
  run<1, 48, 2>(out, cyc);
  run<2, 48, 2>(out, cyc);
  run<1, 48, 4>(out, cyc);
  run<2, 48, 4>(out, cyc);
  run<4, 48, 4>(out, cyc);
  return 0;
}
