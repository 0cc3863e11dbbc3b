// FETCH_SIZE / WRITE_SIZE calibration for the access widths the train and
// rollout kernels use (MI355X_MICROARCH.md §HBM: only 16-B/lane streaming
// reads are calibrated, at x2).  Each kernel streams a 1 GiB buffer once
// (past the 256 MiB Infinity Cache) with one access width and writes one
// float per wave; rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) per kernel
// gives the counter / bytes ratio:
//   hipcc --offload-arch=gfx950 -O3 tools/probes/fetch_probe.hip -o build/probe_fetch
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d out -- ./build/probe_fetch
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename V>
__global__ void read_width(const V *in, float *out, size_t n) {
  float s = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const V v = in[i];
    const unsigned char *b = reinterpret_cast<const unsigned char *>(&v);
    s += (float)b[0];
  }
  if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = s;
}

// 4-byte per-lane scattered-row stores like the slab write-out
__global__ void write_f32(float *out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = (float)i;
}

struct b2 { char x, y; };
struct b16 { int4 v; };

int main() {
  const size_t bytes = 1ull << 30;
  char *buf;
  float *out, *wbuf;
  hipMalloc(&buf, bytes);
  hipMemset(buf, 1, bytes);
  hipMalloc(&out, 1 << 24);
  hipMalloc(&wbuf, 256ull << 20);
  const dim3 grid(2048), block(256);
  hipLaunchKernelGGL(read_width<char>, grid, block, 0, 0, (const char *)buf, out, bytes);
  hipLaunchKernelGGL(read_width<b2>, grid, block, 0, 0, (const b2 *)buf, out, bytes / 2);
  hipLaunchKernelGGL(read_width<int>, grid, block, 0, 0, (const int *)buf, out, bytes / 4);
  hipLaunchKernelGGL(read_width<b16>, grid, block, 0, 0, (const b16 *)buf, out, bytes / 16);
  hipLaunchKernelGGL(write_f32, grid, block, 0, 0, wbuf, (256ull << 20) / 4);
  hipDeviceSynchronize();
  printf("read 1 GiB with 1 / 2 / 4 / 16-byte lanes; wrote 256 MiB with 4-byte lanes\n");
  return 0;
}
