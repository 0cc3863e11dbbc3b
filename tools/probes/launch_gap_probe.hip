// launch_gap_probe.hip -- the idle time between dependent kernels in one
// stream on gfx950, launched one by one vs replayed from a hipGraph.
// A chain of NK kernels, each a grid of 256 workgroups that reads the
// previous kernel's output (`bytes` per kernel) and writes its own; the
// chain's wall time minus the sum of the kernels' own durations (measured
// alone) is the gap.  hipcc --offload-arch=gfx950 -O3 launch_gap_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                        \
      return 1;                                                             \
    }                                                                       \
  } while (0)

__global__ void step_kernel(const float *in, float *out, long n, int spin) {
  const long i0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  float acc = 0.0f;
  for (long i = i0; i < n; i += (long)gridDim.x * blockDim.x) acc += in[i];
  for (int s = 0; s < spin; ++s) acc = acc * 0.999f + 1.0f;  // work per thread
  for (long i = i0; i < n; i += (long)gridDim.x * blockDim.x) out[i] = acc;
}

int main() {
  const int NK = 16, reps = 20;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (long bytes : {4096L, 1L << 20, 16L << 20}) {
    for (int spin : {0, 2000}) {
      const long n = bytes / 4;
      std::vector<float *> buf(NK + 1);
      for (auto &b : buf) {
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(b, 0, bytes));
      }
      auto chain = [&]() {
        for (int k = 0; k < NK; ++k)
          hipLaunchKernelGGL(step_kernel, dim3(256), dim3(256), 0, s, buf[k], buf[k + 1], n, spin);
      };
      // one kernel alone (average over reps, events around each)
      float one = 0.0f;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(step_kernel, dim3(256), dim3(256), 0, s, buf[0], buf[1], n, spin);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0) one += ms / (reps - 1);
      }
      // the chain, launched
      chain();
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r) chain();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms_launch;
      CK(hipEventElapsedTime(&ms_launch, e0, e1));
      // the chain, captured once and replayed
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      chain();
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms_graph;
      CK(hipEventElapsedTime(&ms_graph, e0, e1));
      const double per = 1e3 / (reps * NK);
      printf("bytes %9ld spin %5d: kernel alone %7.2f us | launched %7.2f us/kernel (gap %6.2f) | graph %7.2f us/kernel (gap %6.2f)\n",
             bytes, spin, one * 1e3, ms_launch * per, ms_launch * per - one * 1e3,
             ms_graph * per, ms_graph * per - one * 1e3);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      for (auto &b : buf) CK(hipFree(b));
    }
  }
  return 0;
}
