// xylo/tensor.h (xylo-hip drop-in layer) -- host containers only.
//
// Replaces the host-side vocabulary of xylo/tensor.h that the learner / agent
// API and the apps/bin_packing drivers use: owning `vector` / `matrix`,
// borrowing `vector_view` / `matrix_view`, fold / flatten / slice /
// borrow_vector, the global engine `default_generator()` (tensor.cc:71-75) and
// the three sampling helpers (tensor.cc:464-476).  There is no host tensor
// arithmetic here: every Dense / softmax / loss computation of the path runs
// in the HIP kernels behind include/xylo_hip.h.
#ifndef XYLO_HIP_COMPAT_TENSOR_H_
#define XYLO_HIP_COMPAT_TENSOR_H_

#include <algorithm>
#include <array>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <ctime>
#include <initializer_list>
#include <random>
#include <span>
#include <vector>

#include <xeno/exception.h>

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
}  // namespace detail

// The one global engine (std::default_random_engine = minstd_rand0).  Any
// access first runs deferred device rollouts / evaluations, so the draws
// happen in the reference's order.
inline std::default_random_engine &default_generator() {
  if (auto h = detail::engine_flush_hook()) h();
  return detail::raw_generator();
}

class vector_view;
class matrix_view;

class vector_view {
 public:
  vector_view() = default;
  vector_view(float *p, std::size_t n) : p_(p), n_(n) {}
  vector_view(std::span<float> s) : p_(s.data()), n_(s.size()) {}

  std::size_t size() const { return n_; }
  float *data() const { return p_; }
  float *begin() const { return p_; }
  float *end() const { return p_ + n_; }
  float &operator[](std::size_t i) const { return p_[i]; }

  // Assignment copies values (views alias, tensors own), as in the reference.
  const vector_view &operator=(float v) const {
    std::fill(p_, p_ + n_, v);
    return *this;
  }
  const vector_view &operator=(const vector_view &o) const {
    if (o.n_ != n_) throw xeno::error("vector_view: size mismatch");
    std::copy(o.p_, o.p_ + n_, p_);
    return *this;
  }
  vector_view &operator=(const vector_view &o) {
    static_cast<const vector_view &>(*this) = o;
    return *this;
  }

  template <std::size_t N>
  matrix_view fold(std::array<std::size_t, N> shape) const;

 private:
  float *p_ = nullptr;
  std::size_t n_ = 0;
};

class vector {
 public:
  vector() = default;
  explicit vector(std::size_t n) : d_(n) {}
  vector(std::initializer_list<std::size_t> shape) {
    std::size_t n = 1;
    for (std::size_t s : shape) n *= s;
    d_.assign(shape.size() ? n : 0, 0.0f);
  }
  vector(vector_view v) : d_(v.begin(), v.end()) {}

  std::size_t size() const { return d_.size(); }
  float *data() { return d_.data(); }
  const float *data() const { return d_.data(); }
  float *begin() { return d_.data(); }
  float *end() { return d_.data() + d_.size(); }
  const float *begin() const { return d_.data(); }
  const float *end() const { return d_.data() + d_.size(); }
  float &operator[](std::size_t i) { return d_[i]; }
  float operator[](std::size_t i) const { return d_[i]; }

  operator vector_view() { return {d_.data(), d_.size()}; }
  operator vector_view() const {
    return {const_cast<float *>(d_.data()), d_.size()};
  }
  vector &operator=(float v) {
    std::fill(d_.begin(), d_.end(), v);
    return *this;
  }
  vector &operator=(vector_view v) {
    d_.assign(v.begin(), v.end());
    return *this;
  }

 private:
  std::vector<float> d_;
};

class matrix_view {
 public:
  matrix_view() = default;
  matrix_view(float *p, std::size_t rows, std::size_t cols)
      : p_(p), r_(rows), c_(cols) {}

  std::size_t num_rows() const { return r_; }
  std::size_t num_cols() const { return c_; }
  vector_view operator[](std::size_t i) const { return {p_ + i * c_, c_}; }
  vector_view flatten() const { return {p_, r_ * c_}; }

  class iterator {
   public:
    iterator(const matrix_view *m, std::size_t i) : m_(m), i_(i) {}
    vector_view operator*() const { return (*m_)[i_]; }
    iterator &operator++() {
      ++i_;
      return *this;
    }
    bool operator!=(const iterator &o) const { return i_ != o.i_; }

   private:
    const matrix_view *m_;
    std::size_t i_;
  };
  iterator begin() const { return {this, 0}; }
  iterator end() const { return {this, r_}; }

 private:
  float *p_ = nullptr;
  std::size_t r_ = 0, c_ = 0;
};

class matrix {
 public:
  matrix() = default;
  matrix(std::initializer_list<std::size_t> shape) {
    auto it = shape.begin();
    r_ = shape.size() > 0 ? *it++ : 0;
    c_ = shape.size() > 1 ? *it : 1;
    d_.assign(r_ * c_, 0.0f);
  }
  matrix(matrix_view m)
      : d_(m.flatten().begin(), m.flatten().end()), r_(m.num_rows()),
        c_(m.num_cols()) {}

  std::size_t num_rows() const { return r_; }
  std::size_t num_cols() const { return c_; }
  vector_view operator[](std::size_t i) { return {d_.data() + i * c_, c_}; }
  operator matrix_view() { return {d_.data(), r_, c_}; }
  operator matrix_view() const {
    return {const_cast<float *>(d_.data()), r_, c_};
  }

 private:
  std::vector<float> d_;
  std::size_t r_ = 0, c_ = 0;
};

template <std::size_t N>
matrix_view vector_view::fold(std::array<std::size_t, N> shape) const {
  static_assert(N == 2, "fold<2> only");
  if (shape[0] * shape[1] != n_) throw xeno::error("fold: size mismatch");
  return {p_, shape[0], shape[1]};
}

template <std::size_t N>
inline matrix_view fold(vector_view v, std::array<std::size_t, N> shape) {
  return v.fold<N>(shape);
}
inline vector_view flatten(matrix_view m) { return m.flatten(); }
inline vector_view slice(vector_view v, std::size_t offset, std::size_t n) {
  if (offset + n > v.size()) throw xeno::error("slice out of range");
  return {v.data() + offset, n};
}
inline vector_view borrow_vector(std::span<float> s, bool on_device = false) {
  if (on_device) throw xeno::error("borrow_vector: host spans only");
  return {s.data(), s.size()};
}

// tensor.cc:464-476 -- the same libstdc++ distributions on the same engine.
inline std::size_t argmax(vector_view v) {
  return std::size_t(std::max_element(v.begin(), v.end()) - v.begin());
}
inline std::size_t discrete_distribution(vector_view v) {
  std::discrete_distribution<std::size_t> dist{v.begin(), v.end()};
  return dist(default_generator());
}
inline void normal_distribution(float mean, float stddev, vector_view v) {
  std::normal_distribution<float> dist{mean, stddev};
  auto &gen = default_generator();
  for (float &x : v) x = dist(gen);
}

}  // namespace xylo

#endif  // XYLO_HIP_COMPAT_TENSOR_H_
