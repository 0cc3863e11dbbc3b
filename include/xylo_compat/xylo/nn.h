// xylo/nn.h (xylo-hip drop-in layer): model / layer / optimizer *descriptions*.
//
// Same class names, constructors and flat parameter layout as the reference
// (nn.h:12-18 init, :60-194 Dense layers, :350-431 activations / heads,
// :467-542 model, :589-698 optimizers).  Layers own their parameters on the
// host exactly as model::parameters() lays them out ([A(out x in), b(out)] per
// Dense layer, activations contribute nothing), and are initialised from the
// global engine with the reference's schemes, so a seeded run starts from the
// reference's weights.  The arithmetic (eval / forward / gradient / optimizer
// step) is not on the host: a model is executed by the HIP kernels of
// include/xylo_hip.h when a device learner or policy uses it (model::eval
// through xh_model_eval), and the device copy of the parameters is pulled
// back lazily by parameters().
#ifndef XYLO_HIP_COMPAT_NN_H_
#define XYLO_HIP_COMPAT_NN_H_

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <fstream>
#include <functional>
#include <memory>
#include <span>
#include <string>
#include <string_view>
#include <vector>

#include <xeno/exception.h>
#include <xeno/logging.h>
#include <xeno/string.h>
#include <xylo/tensor.h>
#include <xylo_hip.h>

namespace xylo {

namespace detail {
// The process-wide device context (XYLO_HIP_DEVICE picks the GPU).
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
}  // namespace detail

inline void normal_initialize(std::size_t, vector_view v) {
  normal_distribution(0, 0.01, v);
}
inline void he_initialize(std::size_t fan_in, vector_view v) {
  normal_distribution(0, ::sqrtf(2.0f / fan_in), v);
}

enum class layer_kind { full, conv1d_1, relu, softmax, softmax_xent };

class layer {
 public:
  explicit layer(std::string_view name = "") : name_(name) {}
  virtual ~layer() = default;
  virtual vector_view parameters() const = 0;
  virtual layer_kind kind() const = 0;
  virtual std::size_t input_size() const { return 0; }
  virtual std::size_t output_size() const { return 0; }
  std::string_view name() { return name_; }

 protected:
  std::string name_;
};

namespace detail {
// [A(out x in), b(out)] with A drawn by `init`, b = 0 (nn.h:63-69, 116-124).
class dense_base : public layer {
 public:
  dense_base(std::size_t in, std::size_t out, std::string_view name,
             void (*init)(std::size_t, vector_view))
      : layer(name), in_(in), out_(out), p_((in + 1) * out) {
    init(in, vector_view(p_.data(), in * out));
    std::fill(p_.begin() + in * out, p_.end(), 0.0f);
  }
  vector_view parameters() const override {
    return {const_cast<float *>(p_.data()), p_.size()};
  }
  std::size_t input_size() const override { return in_; }
  std::size_t output_size() const override { return out_; }

 private:
  std::size_t in_, out_;
  std::vector<float> p_;
};
}  // namespace detail

// full_layer = matmul_layer: Dense over the whole row, normal(0, 0.01) init.
class matmul_layer : public detail::dense_base {
 public:
  matmul_layer(std::size_t input_size, std::size_t output_size,
               std::string_view name = "")
      : dense_base(input_size, output_size, name, normal_initialize) {}
  layer_kind kind() const override { return layer_kind::full; }
};
using full_layer = matmul_layer;

// Per-point Dense (the per-bin policy layer), He init.
class convolution1d_1_layer : public detail::dense_base {
 public:
  convolution1d_1_layer(std::size_t input_channels,
                        std::size_t output_channels, std::string_view name = "")
      : dense_base(input_channels, output_channels, name, he_initialize) {}
  layer_kind kind() const override { return layer_kind::conv1d_1; }
};

class activation_layer : public layer {
 public:
  explicit activation_layer(std::string_view name = "") : layer(name) {}
  vector_view parameters() const override { return {}; }
};

class relu_activation : public activation_layer {
 public:
  explicit relu_activation(std::string_view name = "")
      : activation_layer(name) {}
  layer_kind kind() const override { return layer_kind::relu; }
};

class softmax_layer : public layer {
 public:
  explicit softmax_layer(std::string_view name = "") : layer(name) {}
  vector_view parameters() const override { return {}; }
  layer_kind kind() const override { return layer_kind::softmax; }
};

class softmax_cross_entropy_layer : public softmax_layer {
 public:
  explicit softmax_cross_entropy_layer(std::string_view name = "")
      : softmax_layer(name) {}
  layer_kind kind() const override { return layer_kind::softmax_xent; }
};

class model {
 public:
  void add_layer(std::unique_ptr<layer> &&l) { layers_.emplace_back(std::move(l)); }

  std::span<std::unique_ptr<layer>> layers() { return layers_; }
  std::span<const std::unique_ptr<layer>> layers() const { return layers_; }

  std::size_t parameter_size() const {
    std::size_t n = 0;
    for (const auto &l : layers_) n += l->parameters().size();
    return n;
  }

  // nn.h:490-508.  parameters() first pulls a newer device copy, if any.
  vector parameters() {
    sync_from_device();
    vector out({parameter_size()});
    std::size_t off = 0;
    for (const auto &l : layers_) {
      vector_view p = l->parameters();
      std::copy(p.begin(), p.end(), out.begin() + off);
      off += p.size();
    }
    return out;
  }
  void set_parameters(vector_view v) {
    if (v.size() < parameter_size())
      throw xeno::error(xeno::string::strcat("set_parameters: ", v.size(),
                                             " values for ", parameter_size()));
    std::size_t off = 0;
    for (const auto &l : layers_) {
      vector_view p = l->parameters();
      std::copy(v.begin() + off, v.begin() + off + p.size(), p.begin());
      off += p.size();
    }
    device_newer_ = false;
    ++host_version_;
  }

  // nn.h:473-479, on the device (xh_model_eval): the layer chain's forward
  // over the rows of x with the current parameters (a newer device copy is
  // pulled first).
  matrix eval(matrix_view x) const {
    auto *self = const_cast<model *>(this);
    self->sync_from_device();
    std::vector<xh_layer> ls;
    std::size_t width = x.num_cols(), widest = width;
    for (const auto &l : layers_) {
      xh_layer d{0, int(l->input_size()), int(l->output_size())};
      switch (l->kind()) {
        case layer_kind::full:
          d.kind = XH_LAYER_FULL;
          width = l->output_size();
          break;
        case layer_kind::conv1d_1:
          d.kind = XH_LAYER_CONV1D_1;
          width = l->input_size() ? width / l->input_size() * l->output_size()
                                  : width;
          break;
        case layer_kind::relu: d.kind = XH_LAYER_RELU; break;
        case layer_kind::softmax: d.kind = XH_LAYER_SOFTMAX; break;
        case layer_kind::softmax_xent: d.kind = XH_LAYER_SOFTMAX_XENT; break;
      }
      widest = std::max(widest, width);
      ls.push_back(d);
    }
    std::vector<float> p;
    p.reserve(parameter_size());
    for (const auto &l : layers_) {
      vector_view v = l->parameters();
      p.insert(p.end(), v.begin(), v.end());
    }
    std::vector<float> out(x.num_rows() * widest);
    int oc = 0;
    if (xh_model_eval(detail::hip_context(), ls.data(), int(ls.size()),
                      p.data(), p.size(), x.flatten().data(),
                      int(x.num_rows()), int(x.num_cols()), out.data(),
                      out.size(), &oc) != XH_OK)
      throw xeno::error(std::string("xylo-hip: model::eval: ") +
                        xh_last_error());
    return matrix(matrix_view(out.data(), x.num_rows(), std::size_t(oc)));
  }

  // ---- device binding (used by the device session) ----------------------
  // `pull` copies the device parameters into the given host span.
  void bind_device(const void *owner,
                   std::function<void(std::span<float>)> pull) {
    owner_ = owner;
    pull_ = std::move(pull);
  }
  void mark_device_newer(const void *owner) {
    if (owner_ == owner) device_newer_ = true;
  }
  void unbind_device(const void *owner) {
    if (owner_ != owner) return;
    sync_from_device();
    owner_ = nullptr;
    pull_ = nullptr;
  }
  const void *device_owner() const { return owner_; }
  // Cache slot for device resources tied to this model's lifetime.
  std::shared_ptr<void> device_slot;
  std::uint64_t host_version() const { return host_version_; }
  void sync_from_device() {
    if (!device_newer_ || !pull_) return;
    std::vector<float> buf(parameter_size());
    pull_(buf);
    std::size_t off = 0;
    for (const auto &l : layers_) {
      vector_view p = l->parameters();
      std::copy(buf.begin() + off, buf.begin() + off + p.size(), p.begin());
      off += p.size();
    }
    device_newer_ = false;
  }

 private:
  std::vector<std::unique_ptr<layer>> layers_;
  const void *owner_ = nullptr;
  std::function<void(std::span<float>)> pull_;
  bool device_newer_ = false;
  std::uint64_t host_version_ = 0;
};

// Writes model::parameters() as raw float32, the `weights.NN` format
// deep_agent.cc maps (xeno::sys::mmap<float>).
inline void save_parameters(model &m, const std::string &path) {
  vector p = m.parameters();
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char *>(p.data()), p.size() * sizeof(float));
  if (!f) throw xeno::error("save_parameters: cannot write " + path);
}

// Optimizers (nn.h:589-698): descriptions the device learner applies.
enum class optimizer_kind { sgd, momentum, adam };

class optimizer {
 public:
  optimizer(model &m, float rate) : model_(m), rate_(rate) {}
  virtual ~optimizer() = default;
  void set_rate(float rate) { rate_ = rate; }
  float rate() const { return rate_; }
  model &target() { return model_; }
  virtual optimizer_kind kind() const = 0;
  virtual float weight_decay() const { return 0.0f; }
  virtual float beta1() const { return 0.0f; }
  virtual float beta2() const { return 0.0f; }

 private:
  model &model_;
  float rate_;
};

// p * (1 - wd) - lr * g (nn.h:616-628)
class sgd_optimizer : public optimizer {
 public:
  sgd_optimizer(model &m, float rate, float weight_decay = 0.0f)
      : optimizer(m, rate), weight_decay_(weight_decay) {}
  optimizer_kind kind() const override { return optimizer_kind::sgd; }
  float weight_decay() const override { return weight_decay_; }

 private:
  float weight_decay_;
};

// v = 0.9 v + g; p -= lr v (nn.h:630-657)
class momentum_optimizer : public optimizer {
 public:
  momentum_optimizer(model &m, float rate) : optimizer(m, rate) {}
  optimizer_kind kind() const override { return optimizer_kind::momentum; }
  float beta1() const override { return 0.9f; }
};

// nn.h:659-698
class adam_optimizer : public optimizer {
 public:
  adam_optimizer(model &m, float rate, float beta1 = 0.9, float beta2 = 0.999)
      : optimizer(m, rate), beta1_(beta1), beta2_(beta2) {}
  optimizer_kind kind() const override { return optimizer_kind::adam; }
  float beta1() const override { return beta1_; }
  float beta2() const override { return beta2_; }

 private:
  float beta1_, beta2_;
};

}  // namespace xylo

#endif  // XYLO_HIP_COMPAT_NN_H_
