// Micro-probe: which SIMD each wave of a 512-thread workgroup runs on
// (HW_REG_HW_ID: SIMD_ID bits 5:4, CU_ID 11:8), over many workgroups, and
// the dependent-VALU latency (one chain of v_fma_f32 vs 2, 4, 8 chains).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/simd_probe.hip -o build/probe_simd
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(512) void hwid(unsigned *out) {
  __shared__ char pad[100 * 1024];  // one workgroup per CU, as the train kernel
  pad[threadIdx.x] = 0;
  const unsigned id = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = id + pad[0];
}

template <int CH>
__global__ void chain(float *out, long long *cyc, int iters) {
  float v[CH];
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 0.001f + c;
  const float a = 1.0001f, b = 0.5f;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 64 / CH; ++k)
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(a), "v"(b));
  }
  long long t1 = clock64();
  float s = 0;
  for (int c = 0; c < CH; ++c) s += v[c];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = (t1 - t0) / iters;
}

template <int CH>
void run(float *out, long long *cyc) {
  hipLaunchKernelGGL(chain<CH>, dim3(1), dim3(64), 0, 0, out, cyc, 1000);
  (void)hipDeviceSynchronize();
  long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("one wave, 64 v_fma_f32 as %d independent chain(s): %lld cycles (%.2f per fma)\n", CH, c,
         c / 64.0);
}

int main() {
  const int G = 512;
  unsigned *d;
  (void)hipMalloc(&d, G * 8 * 4);
  hipLaunchKernelGGL(hwid, dim3(G), dim3(512), 0, 0, d);
  std::vector<unsigned> h(G * 8);
  (void)hipMemcpy(h.data(), d, G * 8 * 4, hipMemcpyDeviceToHost);
  std::map<std::vector<int>, int> patterns;  // SIMD of waves 0..7
  for (int b = 0; b < G; ++b) {
    std::vector<int> p(8);
    for (int w = 0; w < 8; ++w) p[w] = (h[b * 8 + w] >> 4) & 3;
    patterns[p]++;
  }
  printf("SIMD id of waves 0..7 (workgroups with that pattern):\n");
  for (auto &kv : patterns) {
    for (int w = 0; w < 8; ++w) printf("%d ", kv.first[w]);
    printf(" x%d\n", kv.second);
  }
  float *out;
  long long *cyc;
  (void)hipMalloc(&out, 64 * 4);
  (void)hipMalloc(&cyc, 8);
  run<1>(out, cyc);
  run<2>(out, cyc);
  run<4>(out, cyc);
  run<8>(out, cyc);
  return 0;
}
