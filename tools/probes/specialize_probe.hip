// Micro-probe: wave specialisation on one SIMD.  A 512-thread block puts two
// waves on each SIMD (wave w on SIMD w % 4).  Waves 0-3 issue only MFMAs
// (NM per iteration, independent accumulators), waves 4-7 only independent
// v_fma_f32 (NV per iteration), then every wave meets at a barrier.  If the
// matrix pipe and the vector issue of one SIMD overlap across its two waves,
// "both" costs about max(mfma only, valu only) cycles per iteration, not
// their sum.  Also with LDS operand reads in the MFMA waves and LDS stores in
// the VALU waves (the traffic of a producer / consumer train epoch).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/specialize_probe.hip -o build/probe_sp
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void vfma(float &x, float a, float b) {
  asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
}
__device__ __forceinline__ void vpkfma(float2 &x, float2 a, float2 b) {
  asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
}

// MODE bit 0: MFMA waves work, bit 1: VALU waves work, bit 2: LDS traffic,
// bit 3: packed VALU (v_pk_fma_f32, NV / 2 of them)
template <int MODE, int NM, int NV, int BIG>
__global__ __launch_bounds__(512) void probe(float *out, long long *cyc, int iters) {
  __shared__ __attribute__((aligned(16))) char lds[64 * 1024];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(0.01f * (l + j));
    b[j] = (__bf16)(0.02f * (l - j));
  }
  f32x4 acc[4] = {};
  f32x16 acc2[2] = {};
  float v[8];
  float2 pv[4];
  for (int j = 0; j < 8; ++j) v[j] = 1.0f + 0.001f * (l + j);
  for (int j = 0; j < 4; ++j) pv[j] = float2{v[2 * j], v[2 * j + 1]};
  const float c1 = 1.0001f + 1e-9f * l, c2 = 0.5f;
  for (int i = threadIdx.x; i < 64 * 1024 / 4; i += 512) ((float *)lds)[i] = 0.001f * i;
  __syncthreads();
  const bool mw = w < 4;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (mw && (MODE & 1)) {
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        if (MODE & 4) {  // one ds_read_b128 operand per MFMA
          b = *(const bf16x8 *)(lds + ((m * 1024 + l * 16) & 0xffff));
        }
        if (BIG)
          acc2[m & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc2[m & 1], 0, 0, 0);
        else
          acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m & 3], 0, 0, 0);
      }
    }
    if (!mw && (MODE & 2)) {
      __builtin_amdgcn_sched_barrier(0);
      if (MODE & 8) {
#pragma unroll
        for (int k = 0; k < NV / 2; ++k) vpkfma(pv[k & 3], float2{c1, c1}, float2{c2, c2});
      } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          vfma(v[k & 7], c1, c2);
          if ((MODE & 4) && (k & 15) == 15)  // one ds_write_b64 per 16 VALU
            *(float2 *)(lds + 32768 + (((k >> 4) * 512 + l * 8) & 0x7fff)) =
                float2{v[0], v[1]};
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
  }
  long long t1 = clock64();
  float s = 0;
  for (int j = 0; j < 8; ++j) s += v[j];
  for (int j = 0; j < 4; ++j) s += pv[j].x + pv[j].y;
  for (int r = 0; r < 4; ++r) s += acc[r][0] + acc[r][1] + acc[r][2] + acc[r][3];
  for (int r = 0; r < 2; ++r) s += acc2[r][0] + acc2[r][5];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = (t1 - t0) / iters;
}

template <int MODE, int NM, int NV, int BIG>
void run(const char *name, float *out, long long *cyc) {
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((probe<MODE, NM, NV, BIG>), dim3(256), dim3(512), 0, 0, out,
                       cyc, 200);
  (void)hipDeviceSynchronize();
  long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-9s NM=%3d NV=%4d %-34s %6lld cycles per iteration\n",
         BIG ? "32x32x16" : "16x16x32", NM, NV, name, c);
}

template <int NM, int NV, int BIG>
void set(float *out, long long *cyc) {
  run<1, NM, NV, BIG>("mfma waves only", out, cyc);
  run<2, NM, NV, BIG>("valu waves only", out, cyc);
  run<3, NM, NV, BIG>("both", out, cyc);
  run<10, NM, NV, BIG>("valu waves only, packed", out, cyc);
  run<11, NM, NV, BIG>("both, packed valu", out, cyc);
  run<7, NM, NV, BIG>("both + LDS reads / stores", out, cyc);
}

int main() {
  float *out;
  long long *cyc;
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&cyc, 8);
  // 32 x 32-cycle MFMAs = 1024 cycles of matrix pipe per SIMD per iteration
  set<32, 128, 1>(out, cyc);
  set<32, 192, 1>(out, cyc);
  set<32, 256, 1>(out, cyc);
  set<32, 384, 1>(out, cyc);
  // the same pipe cycles as 64 x 16-cycle MFMAs
  set<64, 128, 0>(out, cyc);
  set<64, 256, 0>(out, cyc);
  return 0;
}
