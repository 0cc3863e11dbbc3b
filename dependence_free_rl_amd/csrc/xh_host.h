// xh_host.h -- internal helpers of the C ABI's host runtime (xylo_hip.cpp,
// model_api.cpp): the error slot behind xh_last_error, status macros, the
// exception guard, stream-ordered copies and the context struct.
#ifndef XH_HOST_H_
#define XH_HOST_H_

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <exception>
#include <string>

#include "../../include/xylo_hip.h"

struct xh_ctx {
  int device = 0, rank = 0, world = 1;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  int trainers = 0;      // live trainers on this context
  bool closing = false;  // xh_ctx_destroy called while trainers were alive
  int fault = 0;         // xh_ctx_inject_fault (test hook): pending fault
};

namespace xh {
namespace host {

// the message of the last failing call on this thread (xh_last_error)
inline thread_local std::string g_err;

inline int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                                         \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess)                                                 \
      return fail(XH_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #x,     \
                  hipGetErrorString(e_));                                 \
  } while (0)

#define RCCLCHK(x)                                                        \
  do {                                                                    \
    ncclResult_t r_ = (x);                                                \
    if (r_ != ncclSuccess)                                                \
      return fail(XH_ERR_RCCL, "%s:%d %s: %s", __FILE__, __LINE__, #x,    \
                  ncclGetErrorString(r_));                                \
  } while (0)

#define CHK(x)                   \
  do {                           \
    int s_ = (x);                \
    if (s_ != XH_OK) return s_;  \
  } while (0)

// No exception may cross the ABI.
template <class F>
int guard(F &&f) {
  try {
    return f();
  } catch (const std::exception &e) {
    return fail(XH_ERR_INVALID, "exception: %s", e.what());
  } catch (...) {
    return fail(XH_ERR_INVALID, "unknown exception");
  }
}

// Copies between the device and caller (pageable) host memory, ordered on
// the context's stream and waited for before returning (the caller may free
// or read its buffer right after).  Not hipMemcpy: the stream is
// non-blocking, so a null-stream H2D copy of pageable memory, which returns
// once the bytes are staged, is not ordered before the next kernel on it --
// measured: parameters read stale by the first rollout kernel, intermittently.
inline hipError_t copy_to_host(void *host, const void *dev, size_t n,
                               hipStream_t s) {
  const hipError_t e = hipMemcpyAsync(host, dev, n, hipMemcpyDeviceToHost, s);
  return e != hipSuccess ? e : hipStreamSynchronize(s);
}
inline hipError_t copy_to_device(void *dev, const void *host, size_t n,
                                 hipStream_t s) {
  const hipError_t e = hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, s);
  return e != hipSuccess ? e : hipStreamSynchronize(s);
}

inline int copy_ok(hipError_t e) {
  return e == hipSuccess ? XH_OK
                         : fail(XH_ERR_HIP, "copy: %s", hipGetErrorString(e));
}

}  // namespace host
}  // namespace xh

#endif  // XH_HOST_H_
