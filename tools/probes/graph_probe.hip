// graph_probe.hip -- is a hipGraph replay of a chain of small dependent
// kernels faster than launching them one by one on a stream (the iteration of
// a small config is ~18 launches, each followed by a ~3.5 us gap)?
//   hipcc --offload-arch=gfx950 -O2 tools/probes/graph_probe.hip -o build/probe_graph
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void work(float *p, int n, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = p[i];
  for (int k = 0; k < iters; ++k) v = v * 0.999f + 0.001f;
  p[i] = v;
}

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                \
      return 1;                                                          \
    }                                                                    \
  } while (0)

int main() {
  const int n = 1 << 20, kLaunches = 18, kReps = 200;
  float *p = nullptr;
  CK(hipMalloc(&p, n * 4));
  CK(hipMemset(p, 0, n * 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int iters : {1, 64, 512}) {
    auto chain = [&]() {
      for (int k = 0; k < kLaunches; ++k)
        hipLaunchKernelGGL(work, dim3(n / 256), dim3(256), 0, s, p, n, iters);
    };
    // one kernel alone (device time by events)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    chain();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < kReps; ++r)
      hipLaunchKernelGGL(work, dim3(n / 256), dim3(256), 0, s, p, n, iters);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float one = 0.0f;
    CK(hipEventElapsedTime(&one, e0, e1));
    // stream launches
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < kReps; ++r) chain();
    CK(hipStreamSynchronize(s));
    auto t1 = std::chrono::steady_clock::now();
    // graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    chain();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    auto t2 = std::chrono::steady_clock::now();
    for (int r = 0; r < kReps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    auto t3 = std::chrono::steady_clock::now();
    const double us_stream = std::chrono::duration<double, std::micro>(t1 - t0).count() / kReps;
    const double us_graph = std::chrono::duration<double, std::micro>(t3 - t2).count() / kReps;
    const double k_us = one * 1e3 / kReps;
    std::printf("iters %3d: kernel %.2f us; chain of %d: stream %.1f us (gap %.2f), "
                "graph %.1f us (gap %.2f)\n",
                iters, k_us, kLaunches, us_stream, us_stream / kLaunches - k_us, us_graph,
                us_graph / kLaunches - k_us);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipFree(p));
  return 0;
}
