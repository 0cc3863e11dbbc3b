// xylo/tensor.h (xylo-hip drop-in layer): the reference's tensor type and
// its arithmetic (xylo/tensor.h:15-523, xylo/tensor.cc:16-557), with device
// memory behind the memory_blob's on_device bit.
//
// The same vocabulary as the reference: tensor<N> / tensor_view<N> (vector,
// matrix, vector_view, matrix_view), memory_blob, array<N>, the free
// functions in namespace xylo (transpose / matmul_transposed / matmul into an
// output, add / minus / multiply / divide, abs / sin / exp / log / sqrt,
// view / flatten / fold / slice / borrow_vector) and the ones the reference
// declares at global scope (the returning transpose / matmul_transposed /
// matmul, the compound and arithmetic operators, dot / sum / mean /
// variance / stddev / coef_variance / max / argmax / discrete_distribution /
// normal_distribution / uniform_distribution, operator==).  Shape checks
// throw xeno::error as tensor.cc:41-69 does.
//
// Where the arithmetic runs:
// * tensors created with on_device = true live in HBM (tensor.cc:38-39's
//   gpu_alloc / gpu_dealloc stubs made real through xh_tensor_alloc); every
//   operation on them runs on the device (xh_tensor_map / reduce / gemm /
//   transpose: tensor_kernels.hip, the Dense f32-MFMA GEMM).  Mixing a device
//   and a host operand throws.  Element access (operator[] to a float,
//   iteration) needs host memory, as the reference's "TODO: Has to be on CPU"
//   says; xylo::to_host / to_device copy between the two (extensions).
// * on host tensors, the GEMMs from kGemmDeviceMacs multiply-adds and the
//   reductions from kReduceDeviceFloats elements go to the device (a
//   transfer of the operands is cheaper than the host loop there); smaller
//   ones and every elementwise map (memory-bound: a PCIe round trip costs
//   more than the loop) run the reference's host loops.  XYLO_HIP_DEVICE_MIN
//   = k overrides both thresholds (0: every eligible host operation on the
//   device).
//
// Differences from the reference, all on paths where it has undefined or
// broken behaviour: fresh tensors are zero-filled (posix_memalign leaves
// them uninitialised, tensor.cc:19-27); assigning a matrix (tensor<N>, N >= 2) copies values
// into fresh storage instead of aliasing the other tensor's memory (the
// reference's implicit assignment shares the pointer and frees it twice);
// memory_blob's copy assignment makes a borrowed alias; the destructor frees
// device memory only on the device (tensor.cc:94-102 calls both gpu_dealloc
// and free on it); operator* / operator/ of matrices are defined (declared
// but never defined in tensor.cc).  Extensions: default-constructible
// (empty) vector / matrix, move construction, view constructors from a
// pointer and shape, num_rows / num_cols on a matrix, to_host / to_device.
#ifndef XYLO_HIP_COMPAT_TENSOR_H_
#define XYLO_HIP_COMPAT_TENSOR_H_

#include <algorithm>
#include <array>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <functional>
#include <initializer_list>
#include <numeric>
#include <random>
#include <ranges>
#include <span>
#include <sstream>
#include <string>
#include <utility>

#include <xeno/exception.h>
#include <xeno/string.h>
#include <xylo_hip.h>

namespace xylo {

namespace detail {
// Deferred device work that must happen before anybody else draws from the
// global engine (set by the device session, apps/bin_packing/bin_packing.h).
inline void (*&engine_flush_hook())() {
  static void (*hook)() = nullptr;
  return hook;
}
inline std::default_random_engine &raw_generator() {
  // tensor.cc:71-72 seeds with wall-clock seconds; XYLO_SEED pins it.
  static std::default_random_engine g([] {
    const char *s = std::getenv("XYLO_SEED");
    return s ? (unsigned long)std::strtoul(s, nullptr, 10)
             : (unsigned long)std::time(nullptr);
  }());
  return g;
}

// The process-wide device context (XYLO_HIP_DEVICE picks the GPU), created
// on first use: a program whose tensors stay small and on the host never
// touches the device.
inline xh_ctx *hip_context() {
  struct holder {
    xh_ctx *h = nullptr;
    holder() {
      const char *d = std::getenv("XYLO_HIP_DEVICE");
      if (xh_ctx_create(d ? std::atoi(d) : 0, 0, 1, nullptr, &h) != XH_OK)
        throw xeno::error(std::string("xylo-hip: xh_ctx_create: ") +
                          xh_last_error());
    }
    ~holder() { xh_ctx_destroy(h); }
  };
  static holder c;
  return c.h;
}
inline void hip_check(int status, const char *what) {
  if (status != XH_OK)
    throw xeno::error(std::string("xylo-hip: ") + what + ": " + xh_last_error());
}

// host operations of at least this much work go to the device
constexpr std::size_t kGemmDeviceMacs = std::size_t(1) << 22;
constexpr std::size_t kReduceDeviceFloats = std::size_t(1) << 20;
inline std::size_t device_min(std::size_t dflt) {
  static const long over = [] {
    const char *s = std::getenv("XYLO_HIP_DEVICE_MIN");
    return s ? std::atol(s) : -1L;
  }();
  return over >= 0 ? std::size_t(over) : dflt;
}

// fresh tensors hold zeros (the reference leaves them uninitialised)
inline float *host_alloc(std::size_t n) {
  if (n == 0) return nullptr;
  // 64-byte aligned (the reference aligns to 32 for its AVX dot, tensor.cc:24)
  const std::size_t bytes = (n * sizeof(float) + 63) & ~std::size_t(63);
  void *p = std::aligned_alloc(64, bytes);
  if (!p) throw std::bad_alloc();
  std::memset(p, 0, bytes);
  return static_cast<float *>(p);
}
inline float *device_alloc(std::size_t n) {
  float *p = nullptr;
  hip_check(xh_tensor_alloc(hip_context(), n, &p), "tensor on_device alloc");
  return p;
}
inline void device_free(float *p) {
  if (p) (void)xh_tensor_free(hip_context(), p);
}
// n floats between host / device arrays
inline void copy_floats(float *dst, bool dst_dev, const float *src,
                        bool src_dev, std::size_t n) {
  if (!n || dst == src) return;
  if (!dst_dev && !src_dev) {
    std::memmove(dst, src, n * sizeof(float));
    return;
  }
  const int kind = dst_dev && src_dev ? XH_COPY_D2D
                   : dst_dev          ? XH_COPY_H2D
                                      : XH_COPY_D2H;
  hip_check(xh_tensor_copy(hip_context(), dst, src, n, kind), "tensor copy");
}
inline void device_map(int op, const float *a, const float *b, float s,
                       float *out, std::size_t n) {
  hip_check(xh_tensor_map(hip_context(), op, a, b, s, out, n), "tensor map");
}
inline double device_reduce(int op, const float *a, const float *b, float s,
                            std::size_t n, bool dev, int64_t *index = nullptr) {
  double v = 0;
  hip_check(xh_tensor_reduce(hip_context(), op, a, b, s, n, dev ? 1 : 0, &v,
                             index),
            "tensor reduction");
  return v;
}
}  // namespace detail

// The one global engine (std::default_random_engine = minstd_rand0,
// tensor.cc:71-75).  Any access first runs deferred device rollouts /
// evaluations, so the draws happen in the reference's order.
inline std::default_random_engine &default_generator() {
  if (auto h = detail::engine_flush_hook()) h();
  return detail::raw_generator();
}

// tensor.h:19-33
template <std::size_t N> class array {
 public:
  array(std::initializer_list<std::size_t> l) {
    std::copy(l.begin(), l.end(), content_.begin());
  }
  template <std::ranges::range R> array(R &&r) {
    std::copy(r.begin(), r.end(), content_.begin());
  }
  using content_t = std::array<std::size_t, N>;
  const content_t &get_content() const { return content_; }

 private:
  content_t content_{};
};

// tensor.h:35-67: an owned or borrowed float array, the on_device and
// borrowed flags in the address's two top bits.
class memory_blob {
 public:
  explicit memory_blob(std::size_t size = 0, bool on_device = false)
      : u_{on_device ? detail::device_alloc(size) : detail::host_alloc(size)} {
    if (on_device) set_on_device();
  }
  explicit memory_blob(float *addr, bool on_device = false) : u_{addr} {
    set_borrowed();
    if (on_device) set_on_device();
  }
  memory_blob(memory_blob &&other) noexcept { std::swap(u_, other.u_); }
  memory_blob(const memory_blob &) = delete;
  ~memory_blob() { release(); }

  // an alias of other's memory (borrowed: this blob never frees it)
  void operator=(const memory_blob &other) {
    if (this == &other) return;
    release();
    u_.val = other.u_.val | borrowed_mask;
  }
  void operator=(memory_blob &&other) noexcept { std::swap(u_, other.u_); }

  void set_on_device() { u_.val |= on_device_mask; }
  bool on_device() const { return u_.val & on_device_mask; }
  void set_borrowed() { u_.val |= borrowed_mask; }
  bool borrowed() const { return u_.val & borrowed_mask; }

  float *addr() const {
    auto r = u_;
    r.val &= addr_mask;
    return r.addr;
  }

 private:
  void release() {
    if (borrowed() || !addr()) return;
    if (on_device())
      detail::device_free(addr());
    else
      std::free(addr());
    u_.val = 0;
  }
  static constexpr uint64_t borrowed_pos = 62;
  static constexpr uint64_t addr_mask = uint64_t(-1) & ~(0x3ull << 62);
  static constexpr uint64_t on_device_mask = 1ull << 63;
  static constexpr uint64_t borrowed_mask = 1ull << borrowed_pos;
  union {
    float *addr;
    uint64_t val = 0;
  } u_;
};

template <std::size_t N> class tensor_view;
template <std::size_t N> class tensor;

namespace detail {
template <std::size_t N>
std::size_t volume(const std::array<std::size_t, N> &s) {
  return std::accumulate(s.begin(), s.end(), std::size_t(1),
                         std::multiplies<std::size_t>{});
}
template <class T1, class T2>
void check_shape_equal(const T1 &a, const T2 &b) {
  if (a.shape() != b.shape()) throw xeno::error("different tensor shapes.");
}
// both operands on the host, or both on the device; true = device
template <class T1, class T2>
bool same_place(const T1 &a, const T2 &b) {
  if (a.on_device() != b.on_device())
    throw xeno::error("xylo-hip: an operation mixes a host and a device tensor");
  return a.on_device();
}
}  // namespace detail

// tensor.h:69-113
template <std::size_t N> class tensor {
 public:
  tensor() { shape_.fill(0); }  // extension: an empty tensor
  explicit tensor(std::array<std::size_t, N> shape, bool on_device = false)
      : shape_(shape), memory_blob_{detail::volume(shape), on_device} {}
  explicit tensor(std::initializer_list<std::size_t> shape,
                  bool on_device = false)
      : memory_blob_(std::accumulate(shape.begin(), shape.end(), std::size_t(1),
                                     std::multiplies<std::size_t>{}),
                     on_device) {
    shape_.fill(1);
    std::copy(shape.begin(), shape.end(), shape_.begin());
  }
  tensor(const tensor &other)
      : shape_{other.shape()}, memory_blob_{other.size(), other.on_device()} {
    detail::copy_floats(data(), on_device(), other.data(), other.on_device(),
                        size());
  }
  tensor(tensor &&other) noexcept
      : shape_{other.shape_}, memory_blob_(std::move(other.memory_blob_)) {
    other.shape_.fill(0);
  }
  explicit tensor(const tensor_view<N> &view);
  // values into fresh storage (the reference's implicit assignment aliases)
  tensor &operator=(const tensor &other) {
    if (this != &other) {
      tensor t(other);
      swap(t);
    }
    return *this;
  }
  tensor &operator=(tensor &&other) noexcept {
    swap(other);
    return *this;
  }

  std::size_t rank() const { return N; }
  std::size_t size() const { return detail::volume(shape_); }
  float *data() const { return memory_blob_.addr(); }
  bool on_device() const { return memory_blob_.on_device(); }
  std::array<std::size_t, N> shape() const { return shape_; }
  std::size_t num_rows() const requires(N == 2) { return shape_[0]; }
  std::size_t num_cols() const requires(N == 2) { return shape_[1]; }

  tensor_view<N - 1> operator[](std::size_t i) const {
    std::array<std::size_t, N - 1> s;
    std::copy(shape_.begin() + 1, shape_.end(), s.begin());
    return tensor_view<N - 1>(data() + i * detail::volume(s), s, on_device());
  }

  void swap(tensor &o) noexcept {
    std::swap(shape_, o.shape_);
    std::swap(memory_blob_, o.memory_blob_);
  }

 private:
  std::array<std::size_t, N> shape_;
  memory_blob memory_blob_;
};

// tensor.h:115-171
template <> class tensor<1> {
 public:
  using value_type = float;
  using iterator = float *;
  using const_iterator = const float *;
  tensor() : shape_{0} {}  // extension: an empty vector
  explicit tensor(std::array<std::size_t, 1> shape, bool on_device = false)
      : shape_(shape), memory_blob_{shape[0], on_device} {}
  explicit tensor(std::size_t size, bool on_device = false)
      : shape_{size}, memory_blob_{size, on_device} {}
  explicit tensor(std::initializer_list<std::size_t> shape,
                  bool on_device = false)
      : memory_blob_(std::accumulate(shape.begin(), shape.end(), std::size_t(1),
                                     std::multiplies<std::size_t>{}),
                     on_device) {
    shape_[0] = shape.size() ? *shape.begin() : 1;
  }
  tensor(const tensor &other)
      : shape_{other.shape()}, memory_blob_{other.size(), other.on_device()} {
    detail::copy_floats(data(), on_device(), other.data(), other.on_device(),
                        size());
  }
  tensor(tensor &&other) noexcept
      : shape_{other.shape_}, memory_blob_(std::move(other.memory_blob_)) {
    other.shape_[0] = 0;
  }
  explicit tensor(tensor_view<1> view);

  void operator=(float val);
  void operator=(tensor_view<1> other);
  void operator=(const tensor<1> &other);

  std::size_t rank() const { return 1; }
  std::size_t size() const { return shape_[0]; }

  iterator begin() noexcept { return memory_blob_.addr(); }
  iterator end() noexcept { return memory_blob_.addr() + size(); }
  const_iterator begin() const noexcept { return memory_blob_.addr(); }
  const_iterator end() const noexcept { return memory_blob_.addr() + size(); }

  float *data() const { return memory_blob_.addr(); }
  bool on_device() const { return memory_blob_.on_device(); }
  std::array<std::size_t, 1> shape() const { return shape_; }

  // host memory (tensor.h:159-166)
  float operator[](std::size_t i) const { return *(data() + i); }
  float &operator[](std::size_t i) { return *(data() + i); }

  void swap(tensor &o) noexcept {
    std::swap(shape_, o.shape_);
    std::swap(memory_blob_, o.memory_blob_);
  }

 private:
  std::array<std::size_t, 1> shape_;
  memory_blob memory_blob_;
};

// tensor.h:173-210
template <std::size_t N> class tensor_view {
 public:
  tensor_view(const tensor<N> &t)
      : shape_(t.shape()), memory_blob_(t.data(), t.on_device()) {}
  tensor_view(const tensor_view<N> &other)
      : shape_(other.shape()), memory_blob_(other.data(), other.on_device()) {}
  // extension: a view of n-dimensional data at addr
  tensor_view(float *addr, const std::array<std::size_t, N> &shape,
              bool on_device = false)
      : shape_(shape), memory_blob_(addr, on_device) {}
  std::size_t rank() const { return N; }
  std::size_t size() const { return detail::volume(shape_); }
  float *data() const { return memory_blob_.addr(); }
  bool on_device() const { return memory_blob_.on_device(); }
  std::array<std::size_t, N> shape() const { return shape_; }
  tensor_view<1> flatten() const;
  tensor_view<N - 1> operator[](std::size_t i) const {
    std::array<std::size_t, N - 1> s;
    std::copy(shape_.begin() + 1, shape_.end(), s.begin());
    return tensor_view<N - 1>(data() + i * detail::volume(s), s, on_device());
  }

 private:
  std::array<std::size_t, N> shape_;
  memory_blob memory_blob_;
};

// Matrix view, tensor.h:212-250
template <> class tensor_view<2> {
 public:
  class iterator;
  using value_type = tensor<1>;

  tensor_view(const tensor<2> &m)
      : shape_(m.shape()), memory_blob_{m.data(), m.on_device()} {}
  tensor_view(const tensor_view<2> &other)
      : shape_(other.shape()), memory_blob_{other.data(), other.on_device()} {}
  // extensions: rows x cols floats at addr
  tensor_view(float *addr, const std::array<std::size_t, 2> &shape,
              bool on_device = false)
      : shape_(shape), memory_blob_{addr, on_device} {}
  tensor_view(float *addr, std::size_t rows, std::size_t cols,
              bool on_device = false)
      : shape_{rows, cols}, memory_blob_{addr, on_device} {}
  // a view is not re-seated (tensor.h:245: its blob is const)
  tensor_view &operator=(const tensor_view &) = delete;

  std::size_t rank() const { return 2; }
  std::size_t size() const { return shape_[0] * shape_[1]; }
  float *data() const { return memory_blob_.addr(); }
  bool on_device() const { return memory_blob_.on_device(); }

  iterator begin() const noexcept;
  iterator end() const noexcept;

  std::array<std::size_t, 2> shape() const { return shape_; }
  std::size_t num_rows() const { return shape_[0]; }
  std::size_t num_cols() const { return shape_[1]; }

  tensor_view<1> operator[](std::size_t i) const;
  tensor_view<1> flatten() const;

 private:
  std::array<std::size_t, 2> shape_;
  const memory_blob memory_blob_;
};

// Vector view, tensor.h:252-319
template <> class tensor_view<1> {
 public:
  using value_type = float;
  using iterator = float *;
  using const_iterator = const float *;

  tensor_view(const tensor<1> &v)
      : shape_(v.shape()), memory_blob_{v.data(), v.on_device()} {}
  tensor_view(const tensor_view<1> &other)
      : shape_(other.shape()), memory_blob_{other.data(), other.on_device()} {}
  // extensions: n floats at addr
  tensor_view(float *addr, const std::array<std::size_t, 1> &shape,
              bool on_device = false)
      : shape_(shape), memory_blob_{addr, on_device} {}
  tensor_view(float *addr, std::size_t n, bool on_device = false)
      : shape_{n}, memory_blob_{addr, on_device} {}

  std::size_t rank() const { return 1; }
  std::size_t size() const { return shape_[0]; }
  float *data() const { return memory_blob_.addr(); }
  bool borrowed() const { return memory_blob_.borrowed(); }
  bool on_device() const { return memory_blob_.on_device(); }

  iterator begin() noexcept { return memory_blob_.addr(); }
  iterator end() noexcept { return memory_blob_.addr() + size(); }
  const_iterator begin() const noexcept { return memory_blob_.addr(); }
  const_iterator end() const noexcept { return memory_blob_.addr() + size(); }

  float operator[](uint64_t i) const { return *(begin() + i); }
  float &operator[](uint64_t i) { return *(begin() + i); }

  std::array<std::size_t, 1> shape() const { return shape_; }

  void operator=(float val);
  void operator=(const tensor_view<1> &v);

  float dot(tensor_view<1> v) const;
  float sum() const;
  float mean() const;
  float variance() const;
  float stddev() const;
  float coef_variance() const;
  float max() const;
  std::size_t argmax() const;

  void normal_distribution(float mean, float stddev);
  void uniform_distribution(float lower, float upper);

  tensor_view<1> slice(std::size_t pos, std::size_t size) const {
    return tensor_view<1>(memory_blob_.addr() + pos,
                          std::array<std::size_t, 1>{size}, on_device());
  }
  tensor_view<1> flatten() const { return *this; }

  template <std::size_t N>
  tensor_view<N> fold(std::array<std::size_t, N> shape) const {
    return tensor_view<N>{memory_blob_.addr(), shape, on_device()};
  }
  tensor_view<2> fold(std::size_t num_rows, std::size_t num_cols) const {
    return tensor_view<2>{memory_blob_.addr(),
                          std::array<std::size_t, 2>{num_rows, num_cols},
                          on_device()};
  }

 private:
  std::array<std::size_t, 1> shape_;
  const memory_blob memory_blob_;
};

inline tensor_view<1> borrow_vector(std::span<float> s, bool on_device = false) {
  return tensor_view<1>(s.data(), std::array<std::size_t, 1>{s.size()},
                        on_device);
}

using vector = tensor<1>;
using matrix = tensor<2>;
using vector_view = tensor_view<1>;
using matrix_view = tensor_view<2>;

inline vector_view matrix_view::flatten() const {
  return vector_view{memory_blob_.addr(), std::array<std::size_t, 1>{size()},
                     on_device()};
}
template <std::size_t N> inline vector_view tensor_view<N>::flatten() const {
  return vector_view{memory_blob_.addr(), std::array<std::size_t, 1>{size()},
                     on_device()};
}
inline vector_view matrix_view::operator[](std::size_t i) const {
  return flatten().slice(i * num_cols(), num_cols());
}

class matrix_view::iterator {
 public:
  vector_view operator*() { return m_[idx_]; }
  bool operator!=(const iterator &other) { return idx_ != other.idx_; }
  void operator++() { ++idx_; }

 private:
  iterator(tensor_view<2> m, std::size_t idx) : m_(m), idx_(idx) {}
  matrix_view m_;
  std::size_t idx_;
  friend matrix_view;
};
inline matrix_view::iterator matrix_view::begin() const noexcept {
  return iterator(*this, 0);
}
inline matrix_view::iterator matrix_view::end() const noexcept {
  return iterator(*this, num_rows());
}

// ------------------------------------------------ construction / assignment
template <std::size_t N>
tensor<N>::tensor(const tensor_view<N> &tv)
    : shape_{tv.shape()}, memory_blob_{tv.size(), tv.on_device()} {
  detail::copy_floats(data(), on_device(), tv.data(), tv.on_device(), size());
}
inline vector::tensor(vector_view view)
    : shape_{view.shape()}, memory_blob_{view.size(), view.on_device()} {
  detail::copy_floats(data(), on_device(), view.data(), view.on_device(),
                      size());
}
namespace detail {
inline void fill(vector_view v, float val) {
  if (v.on_device())
    device_map(XH_T_FILL, nullptr, nullptr, val, v.data(), v.size());
  else
    std::fill(v.data(), v.data() + v.size(), val);
}
// values of src into dst, shapes equal (tensor.cc:129-136, 153-156)
inline void assign(vector_view dst, vector_view src) {
  check_shape_equal(dst, src);
  copy_floats(dst.data(), dst.on_device(), src.data(), src.on_device(),
              dst.size());
}
}  // namespace detail
inline void vector::operator=(float val) { detail::fill(*this, val); }
inline void vector::operator=(vector_view other) { detail::assign(*this, other); }
inline void vector::operator=(const vector &other) {
  detail::assign(*this, other);
}
inline void vector_view::operator=(float val) { detail::fill(*this, val); }
inline void vector_view::operator=(const vector_view &v) {
  detail::assign(*this, v);
}

// Extensions: copies of a tensor in host / device memory.
template <std::size_t N> tensor<N> to_host(const tensor_view<N> &t) {
  tensor<N> out(t.shape(), false);
  detail::copy_floats(out.data(), false, t.data(), t.on_device(), t.size());
  return out;
}
template <std::size_t N> tensor<N> to_device(const tensor_view<N> &t) {
  tensor<N> out(t.shape(), true);
  detail::copy_floats(out.data(), true, t.data(), t.on_device(), t.size());
  return out;
}
inline vector to_host(const vector &t) { return to_host<1>(vector_view(t)); }
inline vector to_device(const vector &t) { return to_device<1>(vector_view(t)); }
inline matrix to_host(const matrix &t) { return to_host<2>(matrix_view(t)); }
inline matrix to_device(const matrix &t) { return to_device<2>(matrix_view(t)); }

// ------------------------------------------------------------- kernels --
namespace detail {
// out = op(in1, in2, s) elementwise (tensor.cc:256-317)
inline void map(int op, vector_view in1, const vector_view *in2, float s,
                vector_view out) {
  check_shape_equal(in1, out);
  if (in2) check_shape_equal(in1, *in2);
  const bool dev = same_place(in1, out);
  if (in2) same_place(in1, *in2);
  const std::size_t n = in1.size();
  const float *a = in1.data(), *b = in2 ? in2->data() : nullptr;
  float *o = out.data();
  if (dev) {
    device_map(op, a, b, s, o, n);
    return;
  }
  switch (op) {
    case XH_T_ADD: std::transform(a, a + n, b, o, std::plus{}); break;
    case XH_T_MINUS: std::transform(a, a + n, b, o, std::minus{}); break;
    case XH_T_MULTIPLY: std::transform(a, a + n, b, o, std::multiplies{}); break;
    case XH_T_DIVIDE: std::transform(a, a + n, b, o, std::divides{}); break;
    case XH_T_ADD_S:
      std::transform(a, a + n, o, [s](float x) { return x + s; });
      break;
    case XH_T_MINUS_S:
      std::transform(a, a + n, o, [s](float x) { return x - s; });
      break;
    case XH_T_MULTIPLY_S:
      std::transform(a, a + n, o, [s](float x) { return x * s; });
      break;
    case XH_T_DIVIDE_S:
      std::transform(a, a + n, o, [s](float x) { return x / s; });
      break;
    case XH_T_ABS: std::transform(a, a + n, o, ::fabsf); break;
    case XH_T_SIN: std::transform(a, a + n, o, ::sinf); break;
    case XH_T_EXP: std::transform(a, a + n, o, ::expf); break;
    case XH_T_LOG: std::transform(a, a + n, o, ::logf); break;
    case XH_T_SQRT: std::transform(a, a + n, o, ::sqrtf); break;
    case XH_T_RMINUS_S:
      std::transform(a, a + n, o, [s](float x) { return s - x; });
      break;
    case XH_T_RDIVIDE_S:
      std::transform(a, a + n, o, [s](float x) { return s / x; });
      break;
  }
}
// the compound operators: v1 op= v2 / scalar (tensor.cc:371-398)
inline void map_inplace(int op, vector_view v, const vector_view *v2, float s) {
  map(op, v, v2, s, v);
}

// Host float reductions in 32 interleaved partial sums, combined pairwise:
// the shape of the reference's own reductions, which its -O3 -ffast-math
// -mavx build vectorises into partial sums (8 lanes x 4 accumulators), not
// the strictly sequential order std::accumulate names (tensor.cc:166, 437,
// 450; its dot runs 8-wide _mm256_dp_ps blocks, :400-418).
template <class F> float blocked_sum(std::size_t n, F term) {
  constexpr std::size_t L = 32;
  float acc[L] = {};
  std::size_t i = 0;
  for (; i + L <= n; i += L)
    for (std::size_t j = 0; j < L; ++j) acc[j] += term(i + j);
  for (std::size_t j = 0; i < n; ++i, ++j) acc[j] += term(i);
  for (std::size_t w = L / 2; w >= 1; w /= 2)
    for (std::size_t j = 0; j < w; ++j) acc[j] += acc[j + w];
  return acc[0];
}

inline bool reduce_on_device(vector_view v) {
  return v.on_device() || v.size() >= device_min(kReduceDeviceFloats);
}
inline float sum(vector_view v) {
  if (v.size() == 0) return 0.0f;
  if (reduce_on_device(v))
    return (float)device_reduce(XH_R_SUM, v.data(), nullptr, 0.0f, v.size(),
                                v.on_device());
  const float *p = v.data();
  return blocked_sum(v.size(), [p](std::size_t i) { return p[i]; });
}
inline float dot(vector_view a, vector_view b) {
  check_shape_equal(a, b);
  const bool dev = same_place(a, b);
  if (dev || a.size() >= device_min(kReduceDeviceFloats))
    return (float)device_reduce(XH_R_DOT, a.data(), b.data(), 0.0f, a.size(),
                                dev);
  const float *x = a.data(), *y = b.data();
  return blocked_sum(a.size(), [x, y](std::size_t i) { return x[i] * y[i]; });
}
inline float mean(vector_view v) { return sum(v) / v.size(); }
inline float variance(vector_view v) {
  if (v.size() == 0) return 0.0f;
  const float m = mean(v);
  if (reduce_on_device(v))
    return (float)device_reduce(XH_R_SQDEV, v.data(), nullptr, m, v.size(),
                                v.on_device()) /
           v.size();
  const float *p = v.data();
  return blocked_sum(v.size(),
                     [p, m](std::size_t i) {
                       const float d = p[i] - m;
                       return d * d;
                     }) /
         v.size();
}
inline float stddev(vector_view v) { return ::sqrtf(variance(v)); }
inline float coef_variance(vector_view v) {
  const float m = mean(v), sd = stddev(v);
  if (m == 0.0f && sd == 0.0f) return 0.0f;
  return m / sd;
}
inline float max(vector_view v) {
  if (v.size() == 0) throw xeno::error("max of an empty vector");
  if (reduce_on_device(v))
    return (float)device_reduce(XH_R_MAX, v.data(), nullptr, 0.0f, v.size(),
                                v.on_device());
  return *std::max_element(v.data(), v.data() + v.size());
}
inline std::size_t argmax(vector_view v) {
  if (v.size() == 0) return 0;  // distance(begin, max_element) of an empty range
  if (reduce_on_device(v)) {
    int64_t i = 0;
    device_reduce(XH_R_ARGMAX, v.data(), nullptr, 0.0f, v.size(),
                  v.on_device(), &i);
    return (std::size_t)i;
  }
  return std::size_t(std::max_element(v.data(), v.data() + v.size()) - v.data());
}

// the engine's draws land on the host, in order; a device vector gets them
// by one copy (the same values as a host vector)
template <class Dist> void draw(vector_view v, Dist dist) {
  auto &gen = default_generator();
  if (!v.on_device()) {
    for (float *p = v.data(); p != v.data() + v.size(); ++p) *p = dist(gen);
    return;
  }
  vector h(v.size());
  for (float &x : h) x = dist(gen);
  copy_floats(v.data(), true, h.data(), false, v.size());
}

inline void check_transpose_shapes(matrix_view m1, matrix_view m2) {
  if (m1.num_cols() != m2.num_rows() || m1.num_rows() != m2.num_cols())
    throw xeno::error("wrong shapes for transpose");
}
inline void check_matmul_shapes(matrix_view m1, matrix_view m2) {
  if (m1.num_cols() != m2.num_cols())
    throw xeno::error(xeno::string::strcat(
        "wrong shapes for matmul: ", m1.num_rows(), 'x', m1.num_cols(),
        " vs. ", m2.num_cols(), 'x', m2.num_rows()));
}
inline bool gemm_on_device(bool dev, std::size_t m, std::size_t n,
                           std::size_t k) {
  return dev || m * n * k >= device_min(kGemmDeviceMacs);
}
inline void gemm(int layout, matrix_view a, matrix_view b, matrix_view out,
                 std::size_t n, std::size_t k, bool dev) {
  hip_check(xh_tensor_gemm(hip_context(), layout, a.data(), b.data(),
                           out.data(), int(a.num_rows()), int(n), int(k),
                           dev ? 1 : 0),
            "tensor matmul");
}
}  // namespace detail

inline float vector_view::dot(vector_view v) const {
  return detail::dot(*this, v);
}
inline float vector_view::sum() const { return detail::sum(*this); }
inline float vector_view::mean() const { return detail::mean(*this); }
inline float vector_view::variance() const { return detail::variance(*this); }
inline float vector_view::stddev() const { return detail::stddev(*this); }
inline float vector_view::coef_variance() const {
  return detail::coef_variance(*this);
}
inline float vector_view::max() const { return detail::max(*this); }
inline std::size_t vector_view::argmax() const { return detail::argmax(*this); }
inline void vector_view::normal_distribution(float mean, float stddev) {
  detail::draw(*this, std::normal_distribution<float>{mean, stddev});
}
inline void vector_view::uniform_distribution(float lower, float upper) {
  detail::draw(*this, std::uniform_real_distribution<float>{lower, upper});
}

// ---------------------------------------------- global matrix functions --
// tensor.cc:209-216
inline void transpose(matrix_view in, matrix_view out) {
  detail::check_transpose_shapes(in, out);
  const bool dev = detail::same_place(in, out);
  if (dev || in.size() >= detail::device_min(detail::kGemmDeviceMacs)) {
    detail::hip_check(xh_tensor_transpose(detail::hip_context(), in.data(),
                                          out.data(), int(in.num_rows()),
                                          int(in.num_cols()), dev ? 1 : 0),
                      "tensor transpose");
    return;
  }
  const std::size_t r = in.num_rows(), c = in.num_cols();
  const float *pi = in.data();
  float *po = out.data();
  for (std::size_t i = 0; i < r; ++i)
    for (std::size_t j = 0; j < c; ++j) po[j * r + i] = pi[i * c + j];
}
// tensor.cc:218-227: out[i][j] = dot(in1[i], in2[j])
inline void matmul_transposed(matrix_view in1, const matrix_view in2,
                              matrix_view out) {
  detail::check_matmul_shapes(in1, in2);
  const std::size_t m = in1.num_rows(), n = in2.num_rows(), k = in1.num_cols();
  if (out.num_rows() != m || out.num_cols() != n)
    throw xeno::error("wrong output shape for matmul");
  const bool dev = detail::same_place(in1, in2);
  detail::same_place(in1, out);
  if (detail::gemm_on_device(dev, m, n, k)) {
    detail::gemm(XH_GEMM_NT, in1, in2, out, n, k, dev);
    return;
  }
  const float *a = in1.data(), *b = in2.data();
  float *o = out.data();
  for (std::size_t i = 0; i < m; ++i)
    for (std::size_t j = 0; j < n; ++j)
      o[i * n + j] = std::inner_product(a + i * k, a + (i + 1) * k, b + j * k,
                                        0.0f);
}
// tensor.cc:228-230: in1 x in2 (in2 is [k][n])
inline void matmul(matrix_view in1, matrix_view in2, matrix_view out) {
  if (in1.num_cols() != in2.num_rows())
    throw xeno::error(xeno::string::strcat(
        "wrong shapes for matmul: ", in1.num_rows(), 'x', in1.num_cols(),
        " vs. ", in2.num_rows(), 'x', in2.num_cols()));
  const std::size_t m = in1.num_rows(), n = in2.num_cols(), k = in1.num_cols();
  if (out.num_rows() != m || out.num_cols() != n)
    throw xeno::error("wrong output shape for matmul");
  const bool dev = detail::same_place(in1, in2);
  detail::same_place(in1, out);
  if (detail::gemm_on_device(dev, m, n, k)) {
    detail::gemm(XH_GEMM_NN, in1, in2, out, n, k, dev);
    return;
  }
  // the reference's order: dot products against the transposed in2
  tensor<2> t(std::array<std::size_t, 2>{n, k});
  transpose(in2, t);
  const float *a = in1.data(), *b = t.data();
  float *o = out.data();
  for (std::size_t i = 0; i < m; ++i)
    for (std::size_t j = 0; j < n; ++j)
      o[i * n + j] = std::inner_product(a + i * k, a + (i + 1) * k, b + j * k,
                                        0.0f);
}

// ---------------------------------------------- global vector functions --
// tensor.cc:256-317 (out may be one of the inputs)
inline void add(vector_view in1, vector_view in2, vector_view out) {
  detail::map(XH_T_ADD, in1, &in2, 0.0f, out);
}
inline void add(vector_view in, float scalar, vector_view out) {
  detail::map(XH_T_ADD_S, in, nullptr, scalar, out);
}
inline void minus(vector_view in1, vector_view in2, vector_view out) {
  detail::map(XH_T_MINUS, in1, &in2, 0.0f, out);
}
inline void minus(vector_view in, float scalar, vector_view out) {
  detail::map(XH_T_MINUS_S, in, nullptr, scalar, out);
}
inline void multiply(vector_view in1, vector_view in2, vector_view out) {
  detail::map(XH_T_MULTIPLY, in1, &in2, 0.0f, out);
}
inline void multiply(vector_view in, float scalar, vector_view out) {
  detail::map(XH_T_MULTIPLY_S, in, nullptr, scalar, out);
}
inline void divide(vector_view in1, vector_view in2, vector_view out) {
  detail::map(XH_T_DIVIDE, in1, &in2, 0.0f, out);
}
inline void divide(vector_view in, float scalar, vector_view out) {
  detail::map(XH_T_DIVIDE_S, in, nullptr, scalar, out);
}
inline void abs(vector_view in, vector_view out) {
  detail::map(XH_T_ABS, in, nullptr, 0.0f, out);
}
inline void sin(vector_view in, vector_view out) {
  detail::map(XH_T_SIN, in, nullptr, 0.0f, out);
}
inline void exp(vector_view in, vector_view out) {
  detail::map(XH_T_EXP, in, nullptr, 0.0f, out);
}
inline void log(vector_view in, vector_view out) {
  detail::map(XH_T_LOG, in, nullptr, 0.0f, out);
}
inline void sqrt(vector_view in, vector_view out) {
  detail::map(XH_T_SQRT, in, nullptr, 0.0f, out);
}
// tensor.cc:232-251
inline void add(matrix_view in1, matrix_view in2, matrix_view out) {
  detail::check_shape_equal(in1, in2);
  detail::check_shape_equal(in1, out);
  add(in1.flatten(), in2.flatten(), out.flatten());
}
inline void minus(matrix_view in1, matrix_view in2, matrix_view out) {
  detail::check_shape_equal(in1, in2);
  detail::check_shape_equal(in1, out);
  minus(in1.flatten(), in2.flatten(), out.flatten());
}
inline void multiply(matrix_view in1, matrix_view in2, matrix_view out) {
  detail::check_shape_equal(in1, in2);
  detail::check_shape_equal(in1, out);
  multiply(in1.flatten(), in2.flatten(), out.flatten());
}
inline void divide(matrix_view in1, matrix_view in2, matrix_view out) {
  detail::check_shape_equal(in1, in2);
  detail::check_shape_equal(in1, out);
  divide(in1.flatten(), in2.flatten(), out.flatten());
}

// tensor.h:396-422
template <std::size_t N> tensor_view<N> view(tensor<N> t) {
  // (the reference takes t by value and returns a view of the copy)
  tensor_view<N> tv(t);
  return tv;
}
template <std::size_t N> vector_view flatten(tensor_view<N> t) {
  return t.flatten();
}
template <std::size_t N> vector_view flatten(const tensor<N> &t) {
  tensor_view<N> v(t);
  return v.flatten();
}
template <std::size_t N>
tensor_view<N> fold(vector_view v, const xylo::array<N> &shape) {
  return v.fold(shape.get_content());
}
inline vector_view slice(vector_view v, std::size_t pos, std::size_t size) {
  return v.slice(pos, size);
}
inline matrix_view slice(matrix_view v, std::size_t pos, std::size_t size) {
  return matrix_view(v.data() + pos * v.num_cols(),
                     std::array<std::size_t, 2>{size, v.num_cols()},
                     v.on_device());
}

}  // namespace xylo

// ===================================== the reference's global functions ==
// tensor.h:433-487, tensor.cc:321-557
inline xylo::matrix transpose(xylo::matrix_view in) {
  xylo::matrix out(std::array<std::size_t, 2>{in.num_cols(), in.num_rows()},
                   in.on_device());
  xylo::transpose(in, out);
  return out;
}
inline xylo::matrix matmul_transposed(xylo::matrix_view in1,
                                      xylo::matrix_view in2) {
  xylo::matrix out(std::array<std::size_t, 2>{in1.num_rows(), in2.num_rows()},
                   in1.on_device());
  xylo::matmul_transposed(in1, in2, out);
  return out;
}
inline xylo::matrix matmul(xylo::matrix_view in1, xylo::matrix_view in2) {
  xylo::matrix out(std::array<std::size_t, 2>{in1.num_rows(), in2.num_cols()},
                   in1.on_device());
  xylo::matmul(in1, in2, out);
  return out;
}

inline void operator+=(xylo::vector_view v, float val) {
  xylo::detail::map_inplace(XH_T_ADD_S, v, nullptr, val);
}
inline void operator+=(xylo::vector_view v1, xylo::vector_view v2) {
  xylo::detail::map_inplace(XH_T_ADD, v1, &v2, 0.0f);
}
// v -= s and v /= s leave s - v and s / v, as the reference's do: its
// std::bind_front(std::minus{}, val) puts the scalar first (tensor.cc:
// 378-380, 392-394; the matrix forms flatten to these, :343, :353)
inline void operator-=(xylo::vector_view v, float val) {
  xylo::detail::map_inplace(XH_T_RMINUS_S, v, nullptr, val);
}
inline void operator-=(xylo::vector_view v1, xylo::vector_view v2) {
  xylo::detail::map_inplace(XH_T_MINUS, v1, &v2, 0.0f);
}
inline void operator*=(xylo::vector_view v, float val) {
  xylo::detail::map_inplace(XH_T_MULTIPLY_S, v, nullptr, val);
}
inline void operator*=(xylo::vector_view v1, xylo::vector_view v2) {
  xylo::detail::map_inplace(XH_T_MULTIPLY, v1, &v2, 0.0f);
}
inline void operator/=(xylo::vector_view v, float val) {
  xylo::detail::map_inplace(XH_T_RDIVIDE_S, v, nullptr, val);
}
inline void operator/=(xylo::vector_view v1, xylo::vector_view v2) {
  xylo::detail::map_inplace(XH_T_DIVIDE, v1, &v2, 0.0f);
}

inline void operator+=(xylo::matrix_view m, float val) { m.flatten() += val; }
inline void operator+=(xylo::matrix_view m1, xylo::matrix_view m2) {
  xylo::detail::check_shape_equal(m1, m2);
  m1.flatten() += m2.flatten();
}
inline void operator-=(xylo::matrix_view m, float val) { m.flatten() -= val; }
inline void operator-=(xylo::matrix_view m1, xylo::matrix_view m2) {
  xylo::detail::check_shape_equal(m1, m2);
  m1.flatten() -= m2.flatten();
}
inline void operator*=(xylo::matrix_view m, float val) { m.flatten() *= val; }
inline void operator*=(xylo::matrix_view m1, xylo::matrix_view m2) {
  xylo::detail::check_shape_equal(m1, m2);
  m1.flatten() *= m2.flatten();
}
inline void operator/=(xylo::matrix_view m, float val) { m.flatten() /= val; }
inline void operator/=(xylo::matrix_view m1, xylo::matrix_view m2) {
  xylo::detail::check_shape_equal(m1, m2);
  m1.flatten() /= m2.flatten();
}

namespace xylo::detail {
template <class F>
matrix elementwise(matrix_view in1, matrix_view in2, F f) {
  matrix out(std::array<std::size_t, 2>{in1.num_rows(), in1.num_cols()},
             in1.on_device());
  f(in1, in2, out);
  return out;
}
template <class F>
vector elementwise(vector_view in, F f) {
  vector out(std::array<std::size_t, 1>{in.size()}, in.on_device());
  f(out);
  return out;
}
}  // namespace xylo::detail

inline xylo::matrix operator+(xylo::matrix_view a, xylo::matrix_view b) {
  return xylo::detail::elementwise(
      a, b, [](auto x, auto y, xylo::matrix_view o) { xylo::add(x, y, o); });
}
inline xylo::matrix operator-(xylo::matrix_view a, xylo::matrix_view b) {
  return xylo::detail::elementwise(
      a, b, [](auto x, auto y, xylo::matrix_view o) { xylo::minus(x, y, o); });
}
inline xylo::matrix operator*(xylo::matrix_view a, xylo::matrix_view b) {
  return xylo::detail::elementwise(
      a, b, [](auto x, auto y, xylo::matrix_view o) { xylo::multiply(x, y, o); });
}
inline xylo::matrix operator/(xylo::matrix_view a, xylo::matrix_view b) {
  return xylo::detail::elementwise(
      a, b, [](auto x, auto y, xylo::matrix_view o) { xylo::divide(x, y, o); });
}

inline float dot(xylo::vector_view v1, xylo::vector_view v2) {
  return xylo::detail::dot(v1, v2);
}
inline float sum(xylo::vector_view v) { return xylo::detail::sum(v); }
inline float mean(xylo::vector_view v) { return xylo::detail::mean(v); }
inline float variance(xylo::vector_view v) { return xylo::detail::variance(v); }
inline float stddev(xylo::vector_view v) { return xylo::detail::stddev(v); }
inline float coef_variance(xylo::vector_view v) {
  return xylo::detail::coef_variance(v);
}
inline float max(xylo::vector_view v) { return xylo::detail::max(v); }
inline std::size_t argmax(xylo::vector_view v) { return xylo::detail::argmax(v); }
// tensor.cc:467-470: the libstdc++ distribution on the global engine (a
// device vector's probabilities are read back first)
inline std::size_t discrete_distribution(xylo::vector_view v) {
  if (v.on_device()) {
    const xylo::vector h = xylo::to_host<1>(v);
    std::discrete_distribution<std::size_t> dist{h.begin(), h.end()};
    return dist(xylo::default_generator());
  }
  std::discrete_distribution<std::size_t> dist{v.begin(), v.end()};
  return dist(xylo::default_generator());
}
inline void normal_distribution(float mean, float stddev, xylo::vector_view v) {
  v.normal_distribution(mean, stddev);
}
inline void uniform_distribution(float lower, float higher,
                                 xylo::vector_view v) {
  v.uniform_distribution(lower, higher);
}

// tensor.cc:483-491: sizes, then the bytes
inline bool operator==(xylo::vector_view in1, xylo::vector_view in2) {
  if (in1.size() != in2.size()) return false;
  if (in1.data() == in2.data()) return true;
  if (in1.on_device() || in2.on_device()) {
    const xylo::vector a = xylo::to_host<1>(in1), b = xylo::to_host<1>(in2);
    return std::memcmp(a.data(), b.data(), a.size() * sizeof(float)) == 0;
  }
  return std::memcmp(in1.data(), in2.data(), in1.size() * sizeof(float)) == 0;
}

inline xylo::vector operator+(xylo::vector_view a, xylo::vector_view b) {
  return xylo::detail::elementwise(a, [&](xylo::vector_view o) { xylo::add(a, b, o); });
}
inline xylo::vector operator+(xylo::vector_view a, float s) {
  return xylo::detail::elementwise(a, [&](xylo::vector_view o) { xylo::add(a, s, o); });
}
inline xylo::vector operator-(xylo::vector_view a, xylo::vector_view b) {
  return xylo::detail::elementwise(a, [&](xylo::vector_view o) { xylo::minus(a, b, o); });
}
inline xylo::vector operator-(xylo::vector_view a, float s) {
  return xylo::detail::elementwise(a, [&](xylo::vector_view o) { xylo::minus(a, s, o); });
}
inline xylo::vector operator*(xylo::vector_view a, xylo::vector_view b) {
  return xylo::detail::elementwise(
      a, [&](xylo::vector_view o) { xylo::multiply(a, b, o); });
}
inline xylo::vector operator*(xylo::vector_view a, float s) {
  return xylo::detail::elementwise(
      a, [&](xylo::vector_view o) { xylo::multiply(a, s, o); });
}
inline xylo::vector operator/(xylo::vector_view a, xylo::vector_view b) {
  return xylo::detail::elementwise(a, [&](xylo::vector_view o) { xylo::divide(a, b, o); });
}
inline xylo::vector operator/(xylo::vector_view a, float s) {
  return xylo::detail::elementwise(a, [&](xylo::vector_view o) { xylo::divide(a, s, o); });
}
inline xylo::vector abs(xylo::vector_view in) {
  return xylo::detail::elementwise(in, [&](xylo::vector_view o) { xylo::abs(in, o); });
}
inline xylo::vector sin(xylo::vector_view in) {
  return xylo::detail::elementwise(in, [&](xylo::vector_view o) { xylo::sin(in, o); });
}
inline xylo::vector exp(xylo::vector_view in) {
  return xylo::detail::elementwise(in, [&](xylo::vector_view o) { xylo::exp(in, o); });
}
inline xylo::vector log(xylo::vector_view in) {
  return xylo::detail::elementwise(in, [&](xylo::vector_view o) { xylo::log(in, o); });
}
inline xylo::vector sqrt(xylo::vector_view in) {
  return xylo::detail::elementwise(in, [&](xylo::vector_view o) { xylo::sqrt(in, o); });
}

// tensor.h:489-523 (a device tensor prints its host copy)
namespace xeno::string {
inline std::string streamable(xylo::vector_view v) {
  if (v.on_device()) return streamable(xylo::vector_view(xylo::to_host<1>(v)));
  std::stringstream out;
  bool first = true;
  out << "[";
  for (float f : v) {
    if (!first) out << ',';
    first = false;
    out << f;
  }
  out << "]";
  return out.str();
}
inline std::string streamable(xylo::matrix_view m) {
  if (m.on_device()) return streamable(xylo::matrix_view(xylo::to_host<2>(m)));
  std::stringstream out;
  bool first = true;
  out << "[";
  for (xylo::vector_view v : m) {
    if (!first) out << '\n';
    first = false;
    out << streamable(v);
  }
  out << "]";
  return out.str();
}
template <std::size_t N> std::string streamable(const xylo::tensor<N> &t) {
  return streamable(xylo::tensor_view<N>(t));
}
}  // namespace xeno::string

#endif  // XYLO_HIP_COMPAT_TENSOR_H_
