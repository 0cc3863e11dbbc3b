// Micro-probe: an MFMA wave WITH VALU filler between its MFMAs beside a
// VALU-only wave on the same SIMD (waves w and w + 4 share a SIMD,
// tools/probes/simd_probe.hip).  Waves 0-3 issue NM v_mfma_f32_32x32x16_f16
// with F independent v_fma_f32 after each; waves 4-7 issue NV independent
// v_fma_f32 (8 chains); then a barrier.  "both" against "mfma only" / "valu
// only" shows whether the matrix wave's own VALU filler keeps the two waves'
// work from overlapping.  PRIO: s_setprio of the MFMA waves.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/filler_probe.hip -o build/probe_filler
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void vfma(float &x, float a, float b) {
  asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
}

template <int MODE, int NM, int F, int NV, int PRIO>
__global__ __launch_bounds__(512) void probe(float *out, long long *cyc, int iters) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)(0.01f * (l + j));
    b[j] = (_Float16)(0.02f * (l - j));
  }
  f32x16 acc[2] = {};
  float v[8], fv[4];
  for (int j = 0; j < 8; ++j) v[j] = 1.0f + 0.001f * (l + j);
  for (int j = 0; j < 4; ++j) fv[j] = 1.0f + 0.002f * (l + j);
  const float c1 = 1.0001f + 1e-9f * l, c2 = 0.5f;
  const bool mw = w < 4;
  if (mw && PRIO) __builtin_amdgcn_s_setprio(PRIO);
  __syncthreads();
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (mw && (MODE & 1)) {
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[m & 1], 0, 0, 0);
#pragma unroll
        for (int f = 0; f < F; ++f) vfma(fv[f & 3], c1, c2);
      }
    }
    if (!mw && (MODE & 2)) {
#pragma unroll
      for (int k = 0; k < NV; ++k) vfma(v[k & 7], c1, c2);
    }
    __syncthreads();
  }
  long long t1 = clock64();
  float s = 0;
  for (int j = 0; j < 8; ++j) s += v[j];
  for (int j = 0; j < 4; ++j) s += fv[j];
  for (int r = 0; r < 2; ++r) s += acc[r][0] + acc[r][5];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = (t1 - t0) / iters;
}

template <int MODE, int NM, int F, int NV, int PRIO>
long long run(float *out, long long *cyc) {
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((probe<MODE, NM, F, NV, PRIO>), dim3(256), dim3(512), 0, 0, out, cyc, 200);
  (void)hipDeviceSynchronize();
  long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  return c;
}

template <int NM, int F, int NV, int PRIO>
void set(float *out, long long *cyc) {
  const long long m = run<1, NM, F, NV, PRIO>(out, cyc);
  const long long v = run<2, NM, F, NV, PRIO>(out, cyc);
  const long long b = run<3, NM, F, NV, PRIO>(out, cyc);
  printf("NM=%2d filler=%d per MFMA, NV=%3d, prio %d: mfma wave %5lld  valu wave %5lld  both %5lld"
         "  (max %5lld, sum %5lld)\n", NM, F, NV, PRIO, m, v, b, m > v ? m : v, m + v);
}

int main() {
  float *out;
  long long *cyc;
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&cyc, 8);
  set<32, 0, 256, 0>(out, cyc);
  set<32, 1, 256, 0>(out, cyc);
  set<32, 2, 256, 0>(out, cyc);
  set<32, 4, 256, 0>(out, cyc);
  set<32, 2, 256, 3>(out, cyc);
  set<32, 4, 256, 3>(out, cyc);
  set<32, 2, 128, 0>(out, cyc);
  set<32, 4, 128, 0>(out, cyc);
  set<32, 8, 128, 0>(out, cyc);
  set<32, 0, 512, 0>(out, cyc);
  set<32, 2, 512, 0>(out, cyc);
  return 0;
}
