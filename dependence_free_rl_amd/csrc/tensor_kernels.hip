// tensor_kernels.hip -- xylo/tensor.{h,cc}'s vector / matrix arithmetic on
// the device, for the drop-in tensor type's device-resident tensors and its
// large host operations (include/xylo_compat/xylo/tensor.h; C ABI
// xh_tensor_*, include/xylo_hip.h).  Reference: tensor.cc:209-317 (matrix and
// vector functions), :338-398 (the compound operators), :427-470 (dot / sum /
// mean / variance / max / argmax).
//
// Elementwise maps: HBM-bound, 16-byte lanes (float4) when the operands are
// 16-byte aligned, a grid-stride loop sized to a few waves per CU.
// Reductions: one pass of per-workgroup partials in double (a fixed grid for a
// given n, so the result is bit-identical run to run), a wave64 shuffle tree
// inside each workgroup, then a one-workgroup finish in the same order.
// Transpose: 64 x 64 tiles through LDS (row stride 65: conflict-free column
// reads).  The GEMMs run on the Dense f32-MFMA GEMM (dense_kernels.hip).
#include <cfloat>

#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {
namespace tensor {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 2048;  // 8 workgroups per CU at 256 CUs

__device__ __forceinline__ float map1(int op, float x, float y, float s) {
  switch (op) {
    case kTensorAdd: return x + y;
    case kTensorMinus: return x - y;
    case kTensorMultiply: return x * y;
    case kTensorDivide: return x / y;
    case kTensorAddS: return x + s;
    case kTensorMinusS: return x - s;
    case kTensorMultiplyS: return x * s;
    case kTensorDivideS: return x / s;
    case kTensorAbs: return fabsf(x);
    case kTensorSin: return sinf(x);
    case kTensorExp: return expf(x);
    case kTensorLog: return logf(x);
    case kTensorSqrt: return sqrtf(x);
    case kTensorFill: return s;
    case kTensorRMinusS: return s - x;
    case kTensorRDivideS: return s / x;
  }
  return x;
}

// out[i] = op(a[i], b[i], s): OP a compile-time constant, VEC = float4 lanes
template <int OP, bool VEC>
__global__ __launch_bounds__(kThreads) void map_kernel(const float *a,
                                                        const float *b, float s,
                                                        float *out, long n) {
  const long stride = (long)gridDim.x * kThreads;
  long i = (long)blockIdx.x * kThreads + threadIdx.x;
  if constexpr (VEC) {
    const long n4 = n >> 2;
    for (; i < n4; i += stride) {
      float4 x = OP == kTensorFill ? float4{0, 0, 0, 0}
                                   : reinterpret_cast<const float4 *>(a)[i];
      float4 y = (OP <= kTensorDivide) ? reinterpret_cast<const float4 *>(b)[i]
                                       : float4{0, 0, 0, 0};
      float4 r;
      r.x = map1(OP, x.x, y.x, s);
      r.y = map1(OP, x.y, y.y, s);
      r.z = map1(OP, x.z, y.z, s);
      r.w = map1(OP, x.w, y.w, s);
      reinterpret_cast<float4 *>(out)[i] = r;
    }
    // the tail (n % 4 elements), one thread each
    const long t = (n4 << 2) + (long)blockIdx.x * kThreads + threadIdx.x;
    if (t < n && t < (n4 << 2) + 4)
      out[t] = map1(OP, OP == kTensorFill ? 0.0f : a[t],
                    OP <= kTensorDivide ? b[t] : 0.0f, s);
  } else {
    for (; i < n; i += stride)
      out[i] = map1(OP, OP == kTensorFill ? 0.0f : a[i],
                    OP <= kTensorDivide ? b[i] : 0.0f, s);
  }
}

static unsigned map_blocks(long n, bool vec) {
  const long work = vec ? (n + 3) / 4 : n;
  long b = (work + kThreads - 1) / kThreads;
  if (b < 1) b = 1;
  return (unsigned)(b > kMaxBlocks ? kMaxBlocks : b);
}

template <int OP>
static hipError_t map_op(const float *a, const float *b, float s, float *out,
                         long n, hipStream_t st) {
  const auto al = [](const void *p) {
    return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  };
  const bool vec = al(a) && al(b) && al(out);
  if (vec)
    hipLaunchKernelGGL((map_kernel<OP, true>), dim3(map_blocks(n, true)),
                       dim3(kThreads), 0, st, a, b, s, out, n);
  else
    hipLaunchKernelGGL((map_kernel<OP, false>), dim3(map_blocks(n, false)),
                       dim3(kThreads), 0, st, a, b, s, out, n);
  return hipGetLastError();
}

// ------------------------------------------------------------ reductions --
// Partial of a workgroup: value (double sums, or the max) and, for argmax,
// the first index of it.
struct Part {
  double v;
  long i;
};

// an empty max / argmax partial (no candidate element seen yet)
constexpr long kNoIndex = 0x7fffffffffffffffL;

__device__ __forceinline__ Part combine(int op, Part x, Part y) {
  if (op == kTensorMax || op == kTensorArgmax) {
    // max_element keeps the first of equal maxima (tensor.cc:462-466); an
    // empty side never wins, whatever its value (-inf elements are
    // candidates like any other)
    if (y.i == kNoIndex) return x;
    if (x.i == kNoIndex) return y;
    if (y.v > x.v || (y.v == x.v && y.i < x.i)) return y;
    return x;
  }
  return Part{x.v + y.v, 0};
}

__device__ __forceinline__ Part wave_reduce(int op, Part p) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    Part q;
    q.v = __shfl_xor(p.v, off, 64);
    q.i = __shfl_xor(p.i, off, 64);
    p = combine(op, p, q);
  }
  return p;
}

__device__ __forceinline__ Part block_reduce(int op, Part p) {
  __shared__ double sv[kThreads / 64];
  __shared__ long si[kThreads / 64];
  p = wave_reduce(op, p);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = p.v;
    si[w] = p.i;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 1; k < kThreads / 64; ++k) p = combine(op, p, Part{sv[k], si[k]});
  return p;
}

__device__ __forceinline__ Part identity(int op) {
  return (op == kTensorMax || op == kTensorArgmax) ? Part{-DBL_MAX, kNoIndex}
                                                   : Part{0.0, 0};
}

// per-workgroup partials of op over a[0, n) (b: dot's second operand, s:
// the mean of the squared deviations)
__global__ __launch_bounds__(kThreads) void reduce_kernel(int op, const float *a,
                                                          const float *b, float s,
                                                          long n, Part *part) {
  Part p = identity(op);
  const long stride = (long)gridDim.x * kThreads;
  for (long i = (long)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const float x = a[i];
    Part q;
    switch (op) {
      case kTensorSum: q = Part{(double)x, 0}; break;
      case kTensorDot: q = Part{(double)x * (double)b[i], 0}; break;
      case kTensorSqDev: {
        const double d = (double)x - (double)s;
        q = Part{d * d, 0};
        break;
      }
      // max_element's scan (`if (*largest < *it) largest = it`) never moves
      // onto a NaN: NaN elements are no candidates (a NaN at index 0 is
      // reduce_finish_kernel's case)
      default: q = x != x ? identity(op) : Part{(double)x, i}; break;
    }
    p = combine(op, p, q);
  }
  p = block_reduce(op, p);
  if (threadIdx.x == 0) part[blockIdx.x] = p;
}

__global__ __launch_bounds__(kThreads) void reduce_finish_kernel(int op,
                                                                 const float *a,
                                                                 const Part *part,
                                                                 int nparts,
                                                                 Part *out) {
  Part p = identity(op);
  for (int k = threadIdx.x; k < nparts; k += kThreads) p = combine(op, p, part[k]);
  p = block_reduce(op, p);
  if (threadIdx.x == 0) {
    if (op == kTensorMax || op == kTensorArgmax) {
      // max_element stays on element 0 when it is NaN (no element compares
      // greater), and when every element is NaN: index 0, value a[0]
      const float a0 = a[0];
      if (a0 != a0 || p.i == kNoIndex) p = Part{(double)a0, 0};
    }
    *out = p;
  }
}

// ------------------------------------------------------------- transpose --
constexpr int kTile = 64;
__global__ __launch_bounds__(kThreads) void transpose_kernel(const float *in,
                                                             float *out, int rows,
                                                             int cols) {
  __shared__ float t[kTile][kTile + 1];
  const int r0 = blockIdx.y * kTile, c0 = blockIdx.x * kTile;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll 4
  for (int k = ty; k < kTile; k += kThreads / 64) {
    const int r = r0 + k, c = c0 + tx;
    if (r < rows && c < cols) t[k][tx] = in[(size_t)r * cols + c];
  }
  __syncthreads();
#pragma unroll 4
  for (int k = ty; k < kTile; k += kThreads / 64) {
    const int c = c0 + k, r = r0 + tx;  // out[c][r] = in[r][c]
    if (r < rows && c < cols) out[(size_t)c * rows + r] = t[tx][k];
  }
}

}  // namespace tensor

hipError_t launch_tensor_map(int op, const float *a, const float *b, float s,
                             float *out, long n, hipStream_t st) {
  using namespace tensor;
  if (n <= 0) return hipSuccess;
  switch (op) {
#define XH_MAP_CASE(OP) \
  case OP: return map_op<OP>(a, b, s, out, n, st);
    XH_MAP_CASE(kTensorAdd)
    XH_MAP_CASE(kTensorMinus)
    XH_MAP_CASE(kTensorMultiply)
    XH_MAP_CASE(kTensorDivide)
    XH_MAP_CASE(kTensorAddS)
    XH_MAP_CASE(kTensorMinusS)
    XH_MAP_CASE(kTensorMultiplyS)
    XH_MAP_CASE(kTensorDivideS)
    XH_MAP_CASE(kTensorAbs)
    XH_MAP_CASE(kTensorSin)
    XH_MAP_CASE(kTensorExp)
    XH_MAP_CASE(kTensorLog)
    XH_MAP_CASE(kTensorSqrt)
    XH_MAP_CASE(kTensorFill)
    XH_MAP_CASE(kTensorRMinusS)
    XH_MAP_CASE(kTensorRDivideS)
#undef XH_MAP_CASE
  }
  return hipErrorInvalidValue;
}

int tensor_reduce_parts(long n) {
  long b = (n + tensor::kThreads * 8 - 1) / (tensor::kThreads * 8);
  if (b < 1) b = 1;
  return (int)(b > tensor::kMaxBlocks ? tensor::kMaxBlocks : b);
}

// scratch: tensor_reduce_parts(n) + 1 partial records (16 bytes each); the
// result (value, index) lands in the last one
hipError_t launch_tensor_reduce(int op, const float *a, const float *b, float s,
                                long n, void *scratch, hipStream_t st) {
  using namespace tensor;
  const int parts = tensor_reduce_parts(n);
  Part *p = reinterpret_cast<Part *>(scratch);
  hipLaunchKernelGGL(reduce_kernel, dim3(parts), dim3(kThreads), 0, st, op, a, b,
                     s, n, p);
  hipLaunchKernelGGL(reduce_finish_kernel, dim3(1), dim3(kThreads), 0, st, op, a,
                     p, parts, p + parts);
  return hipGetLastError();
}

hipError_t launch_tensor_transpose(const float *in, float *out, int rows,
                                   int cols, hipStream_t st) {
  using namespace tensor;
  if (rows <= 0 || cols <= 0) return hipSuccess;
  dim3 grid((cols + kTile - 1) / kTile, (rows + kTile - 1) / kTile);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(kThreads), 0, st, in, out, rows,
                     cols);
  return hipGetLastError();
}

}  // namespace xh
