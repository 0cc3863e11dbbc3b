// tensor_api.cpp -- the C ABI behind the drop-in xylo/tensor.h
// (include/xylo_compat/xylo/tensor.h; include/xylo_hip.h "tensor"):
// device memory for tensors created with on_device = true (the reference's
// gpu_alloc / gpu_dealloc stubs, tensor.cc:38-39), copies, elementwise maps,
// reductions, transposes and the two GEMMs (tensor.cc:209-317, 427-466).
// Every call is synchronous on the context's stream.  Maps take device
// arrays; reductions, GEMMs and transposes take device arrays (on_device = 1)
// or host arrays, which are staged through device memory for the call.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>

#include "xh_host.h"
#include "xh_kernels.h"

using namespace xh::host;

namespace {

// device memory of this process (a device array argument must be one)
bool is_device(const void *p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky query error
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

int need_device(const void *p, const char *what, const char *arg) {
  if (p && !is_device(p))
    return fail(XH_ERR_INVALID, "%s: %s is not device memory (on_device "
                "tensors only)", what, arg);
  return XH_OK;
}

// A device scratch block freed with the call.
struct Scratch {
  void *p = nullptr;
  ~Scratch() {
    if (p) (void)hipFree(p);
  }
  int alloc(size_t bytes) {
    if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess)
      return fail(XH_ERR_HIP, "tensor scratch of %zu bytes", bytes);
    return XH_OK;
  }
};

int launched(hipError_t e, const char *what) {
  return e == hipSuccess ? XH_OK
                         : fail(XH_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

}  // namespace

extern "C" {

int xh_tensor_alloc(xh_ctx *ctx, size_t n, float **out) {
  return guard([&]() -> int {
    if (!ctx || !out) return fail(XH_ERR_INVALID, "tensor_alloc: null arg");
    *out = nullptr;
    if (n == 0) return XH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMalloc((void **)out, n * sizeof(float)));
    // zero-filled on the context's stream (a null-stream memset is not
    // ordered before its next copy or kernel)
    const hipError_t e = hipMemsetAsync(*out, 0, n * sizeof(float), ctx->stream);
    if (e != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess) {
      (void)hipFree(*out);
      *out = nullptr;
      return fail(XH_ERR_HIP, "tensor_alloc: zero fill: %s", hipGetErrorString(e));
    }
    return XH_OK;
  });
}

int xh_tensor_free(xh_ctx *ctx, float *p) {
  return guard([&]() -> int {
    if (!ctx) return fail(XH_ERR_INVALID, "tensor_free: null ctx");
    if (!p) return XH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipStreamSynchronize(ctx->stream));  // no kernel still reads it
    HIPCHK(hipFree(p));
    return XH_OK;
  });
}

int xh_tensor_copy(xh_ctx *ctx, float *dst, const float *src, size_t n,
                   int kind) {
  return guard([&]() -> int {
    if (!ctx || (n && (!dst || !src)))
      return fail(XH_ERR_INVALID, "tensor_copy: null arg");
    if (kind < XH_COPY_H2D || kind > XH_COPY_D2D)
      return fail(XH_ERR_INVALID, "tensor_copy: kind %d", kind);
    if (!n) return XH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    if (kind != XH_COPY_D2H) CHK(need_device(dst, "tensor_copy", "dst"));
    if (kind != XH_COPY_H2D) CHK(need_device(src, "tensor_copy", "src"));
    const hipMemcpyKind k = kind == XH_COPY_H2D   ? hipMemcpyHostToDevice
                            : kind == XH_COPY_D2H ? hipMemcpyDeviceToHost
                                                  : hipMemcpyDeviceToDevice;
    HIPCHK(hipMemcpyAsync(dst, src, n * sizeof(float), k, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return XH_OK;
  });
}

int xh_tensor_map(xh_ctx *ctx, int op, const float *a, const float *b,
                  float scalar, float *out, size_t n) {
  return guard([&]() -> int {
    if (!ctx) return fail(XH_ERR_INVALID, "tensor_map: null ctx");
    if (op < XH_T_ADD || op > XH_T_RDIVIDE_S)
      return fail(XH_ERR_INVALID, "tensor_map: op %d", op);
    if (!n) return XH_OK;
    const bool binary = op <= XH_T_DIVIDE, unary = op != XH_T_FILL;
    if (!out || (unary && !a) || (binary && !b))
      return fail(XH_ERR_INVALID, "tensor_map: null operand");
    HIPCHK(hipSetDevice(ctx->device));
    CHK(need_device(out, "tensor_map", "out"));
    if (unary) CHK(need_device(a, "tensor_map", "a"));
    if (binary) CHK(need_device(b, "tensor_map", "b"));
    CHK(launched(xh::launch_tensor_map(op, a, binary ? b : nullptr, scalar, out,
                                       (long)n, ctx->stream),
                 "tensor_map"));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return XH_OK;
  });
}

int xh_tensor_reduce(xh_ctx *ctx, int op, const float *a, const float *b,
                     float scalar, size_t n, int on_device, double *value,
                     int64_t *index) {
  return guard([&]() -> int {
    if (!ctx || !value) return fail(XH_ERR_INVALID, "tensor_reduce: null arg");
    if (op < XH_R_SUM || op > XH_R_ARGMAX)
      return fail(XH_ERR_INVALID, "tensor_reduce: op %d", op);
    if (!n && (op == XH_R_MAX || op == XH_R_ARGMAX))
      return fail(XH_ERR_INVALID, "tensor_reduce: max / argmax of nothing");
    if (n && (!a || (op == XH_R_DOT && !b)))
      return fail(XH_ERR_INVALID, "tensor_reduce: null operand");
    *value = 0.0;
    if (index) *index = 0;
    if (!n) return XH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int parts = xh::tensor_reduce_parts((long)n);
    const size_t pbytes = (size_t)(parts + 1) * 16;
    const size_t abytes = on_device ? 0 : n * sizeof(float);
    const size_t bbytes = on_device || op != XH_R_DOT ? 0 : n * sizeof(float);
    Scratch sc;
    CHK(sc.alloc(pbytes + abytes + bbytes));
    char *base = static_cast<char *>(sc.p);
    const float *da = a, *db = op == XH_R_DOT ? b : nullptr;
    if (on_device) {
      CHK(need_device(a, "tensor_reduce", "a"));
      if (db) CHK(need_device(db, "tensor_reduce", "b"));
    } else {  // host arrays, staged
      HIPCHK(hipMemcpyAsync(base + pbytes, a, abytes, hipMemcpyHostToDevice, s));
      da = reinterpret_cast<const float *>(base + pbytes);
      if (db) {
        HIPCHK(hipMemcpyAsync(base + pbytes + abytes, b, bbytes,
                              hipMemcpyHostToDevice, s));
        db = reinterpret_cast<const float *>(base + pbytes + abytes);
      }
    }
    CHK(launched(xh::launch_tensor_reduce(op, da, db, scalar, (long)n, base, s),
                 "tensor_reduce"));
    struct {
      double v;
      int64_t i;
    } res{};
    HIPCHK(copy_to_host(&res, base + (size_t)parts * 16, 16, s));
    *value = res.v;
    if (index) *index = res.i;
    return XH_OK;
  });
}

int xh_tensor_gemm(xh_ctx *ctx, int layout, const float *a, const float *b,
                   float *out, int m, int n, int k, int on_device) {
  return guard([&]() -> int {
    if (!ctx || (m > 0 && n > 0 && (!a || !b || !out)))
      return fail(XH_ERR_INVALID, "tensor_gemm: null arg");
    if (layout != XH_GEMM_NT && layout != XH_GEMM_NN)
      return fail(XH_ERR_INVALID, "tensor_gemm: layout %d", layout);
    if (m < 0 || n < 0 || k < 0)
      return fail(XH_ERR_INVALID, "tensor_gemm: %d x %d x %d", m, n, k);
    if (!m || !n) return XH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t na = (size_t)m * k, nb = (size_t)n * k, nc = (size_t)m * n;
    const float *da = a, *db = b;
    float *dc = out;
    Scratch sc;
    if (on_device) {
      CHK(need_device(a, "tensor_gemm", "a"));
      CHK(need_device(b, "tensor_gemm", "b"));
      CHK(need_device(out, "tensor_gemm", "out"));
    } else {
      CHK(sc.alloc((na + nb + nc) * sizeof(float)));
      float *p = static_cast<float *>(sc.p);
      HIPCHK(hipMemcpyAsync(p, a, na * 4, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(p + na, b, nb * 4, hipMemcpyHostToDevice, s));
      da = p;
      db = p + na;
      dc = p + na + nb;
    }
    CHK(launched(xh::launch_tensor_gemm(layout == XH_GEMM_NT, da, db, dc, m, n,
                                        k, s),
                 "tensor_gemm"));
    if (!on_device) HIPCHK(copy_to_host(out, dc, nc * 4, s));
    HIPCHK(hipStreamSynchronize(s));
    return XH_OK;
  });
}

int xh_tensor_transpose(xh_ctx *ctx, const float *in, float *out, int rows,
                        int cols, int on_device) {
  return guard([&]() -> int {
    if (!ctx || (rows > 0 && cols > 0 && (!in || !out)))
      return fail(XH_ERR_INVALID, "tensor_transpose: null arg");
    if (rows < 0 || cols < 0)
      return fail(XH_ERR_INVALID, "tensor_transpose: %d x %d", rows, cols);
    if (!rows || !cols) return XH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t nel = (size_t)rows * cols;
    const float *di = in;
    float *dout = out;
    Scratch sc;
    if (on_device) {
      CHK(need_device(in, "tensor_transpose", "in"));
      CHK(need_device(out, "tensor_transpose", "out"));
    } else {
      CHK(sc.alloc(2 * nel * sizeof(float)));
      float *p = static_cast<float *>(sc.p);
      HIPCHK(hipMemcpyAsync(p, in, nel * 4, hipMemcpyHostToDevice, s));
      di = p;
      dout = p + nel;
    }
    CHK(launched(xh::launch_tensor_transpose(di, dout, rows, cols, s),
                 "tensor_transpose"));
    if (!on_device) HIPCHK(copy_to_host(out, dout, nel * 4, s));
    HIPCHK(hipStreamSynchronize(s));
    return XH_OK;
  });
}

}  // extern "C"
