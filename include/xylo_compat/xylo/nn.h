// xylo/nn.h (xylo-hip drop-in layer): layers, models, losses, optimizers.
//
// Same class names, constructors, public members and flat parameter layout as
// the reference (nn.h:12-18 init, :20-33 layer, :60-194 Dense layers,
// :340-431 activations / heads, :467-528 model, :531-574 losses, :577-698
// optimizers).  Layers own their parameters on the host exactly as
// model::parameters() lays them out ([A(out x in), b(out)] per Dense layer,
// activations contribute nothing), and are initialised from the global
// engine with the reference's schemes, so a seeded run starts from the
// reference's weights.  The arithmetic is not on the host: layer::forward /
// backward / gradient, model::eval / forward / gradient and the library
// optimizers' next_parameters run the HIP kernels of include/xylo_hip.h
// (xh_model_eval / xh_model_forward / xh_model_gradient / xh_layer_* /
// xh_optimizer_apply); a fused device learner (policy_gradient.h) trains
// the model on the device, and its parameters are pulled back lazily by
// parameters().  A layer class of the caller's own (kind() == custom) runs
// its own host forward / backward / gradient inside the same model.
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

inline void normal_initialize(std::size_t, vector_view v) {
  normal_distribution(0, 0.01, v);
}
inline void he_initialize(std::size_t fan_in, vector_view v) {
  normal_distribution(0, ::sqrtf(2.0f / fan_in), v);
}

// Which built-in layer a `layer` is (the device kernels' vocabulary); a
// layer class of the caller's own is `custom` and brings its own forward /
// backward / gradient, as in the reference.
enum class layer_kind { full, conv1d_1, relu, softmax, softmax_xent, custom };

namespace detail {
// a non-null pointer for empty parameter arrays (the ABI rejects null)
inline float *nonnull(float *p) {
  static float dummy = 0.0f;
  return p ? p : &dummy;
}
}  // namespace detail

// nn.h:20-33.  The built-in layers' forward / backward / gradient run on the
// device, one layer per call (xh_model_eval, xh_layer_backward,
// xh_layer_gradient); model::forward / gradient batch a whole chain of them
// into one call each.
class layer {
 public:
  explicit layer(std::string_view name = "") : name_(name) {}
  virtual ~layer() = default;
  virtual matrix forward(matrix_view input);
  virtual matrix backward(matrix_view input, matrix_view backprop);
  virtual vector gradient(matrix_view input, matrix_view backprop);
  virtual vector_view parameters() const = 0;
  virtual layer_kind kind() const { return layer_kind::custom; }
  virtual std::size_t input_size() const { return 0; }
  virtual std::size_t output_size() const { return 0; }
  std::string_view name() { return name_; }

  // the ABI description of a built-in layer
  xh_layer describe() const {
    xh_layer d{0, int(input_size()), int(output_size())};
    switch (kind()) {
      case layer_kind::full: d.kind = XH_LAYER_FULL; break;
      case layer_kind::conv1d_1: d.kind = XH_LAYER_CONV1D_1; break;
      case layer_kind::relu: d.kind = XH_LAYER_RELU; break;
      case layer_kind::softmax: d.kind = XH_LAYER_SOFTMAX; break;
      case layer_kind::softmax_xent: d.kind = XH_LAYER_SOFTMAX_XENT; break;
      case layer_kind::custom:
        throw xeno::error("xylo-hip: a custom layer has no device description");
    }
    return d;
  }
  // output columns of this layer on `cols` input columns
  std::size_t output_cols(std::size_t cols) const {
    switch (kind()) {
      case layer_kind::full: return output_size();
      case layer_kind::conv1d_1:
        return input_size() ? cols / input_size() * output_size() : cols;
      default: return cols;
    }
  }

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
  vector_view parameters() const override {
    return vector_view(nullptr, std::size_t(0));
  }
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
  vector_view parameters() const override {
    return vector_view(nullptr, std::size_t(0));
  }
  layer_kind kind() const override { return layer_kind::softmax; }
};

class softmax_cross_entropy_layer : public softmax_layer {
 public:
  explicit softmax_cross_entropy_layer(std::string_view name = "")
      : softmax_layer(name) {}
  layer_kind kind() const override { return layer_kind::softmax_xent; }
};

inline matrix layer::forward(matrix_view input) {
  if (kind() == layer_kind::custom)
    throw xeno::error("xylo-hip: a custom layer implements forward()");
  const std::size_t rows = input.num_rows(), oc = output_cols(input.num_cols());
  matrix result({rows, oc});
  if (!rows) return result;
  const xh_layer d = describe();
  vector_view p = parameters();
  std::vector<float> out(rows * oc);
  int got = 0;
  detail::hip_check(
      xh_model_eval(detail::hip_context(), &d, 1, detail::nonnull(p.data()),
                    p.size(), input.flatten().data(), int(rows),
                    int(input.num_cols()), out.data(), out.size(), &got),
      "layer::forward");
  return matrix(matrix_view(out.data(), rows, std::size_t(got)));
}

inline matrix layer::backward(matrix_view input, matrix_view backprop) {
  if (kind() == layer_kind::custom)
    throw xeno::error("xylo-hip: a custom layer implements backward()");
  const std::size_t rows = input.num_rows();
  matrix result({rows, input.num_cols()});
  if (!rows) return result;
  const xh_layer d = describe();
  vector_view p = parameters();
  detail::hip_check(
      xh_layer_backward(detail::hip_context(), &d, detail::nonnull(p.data()),
                        p.size(), input.flatten().data(), int(rows),
                        int(input.num_cols()), backprop.flatten().data(),
                        int(backprop.num_cols()),
                        matrix_view(result).flatten().data()),
      "layer::backward");
  return result;
}

inline vector layer::gradient(matrix_view input, matrix_view backprop) {
  if (kind() == layer_kind::custom)
    throw xeno::error("xylo-hip: a custom layer implements gradient()");
  const std::size_t n = parameters().size();
  vector result({n});
  if (!n || !input.num_rows()) return result;
  const xh_layer d = describe();
  detail::hip_check(
      xh_layer_gradient(detail::hip_context(), &d, input.flatten().data(),
                        int(input.num_rows()), int(input.num_cols()),
                        backprop.flatten().data(), int(backprop.num_cols()),
                        result.data(), n),
      "layer::gradient");
  return result;
}

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

  // every layer a built-in one: the chain runs as one device call
  bool device_chain() const {
    for (const auto &l : layers_)
      if (l->kind() == layer_kind::custom) return false;
    return !layers_.empty();
  }

  // nn.h:473-479, on the device (xh_model_eval): the layer chain's forward
  // over the rows of x with the current parameters (a newer device copy is
  // pulled first).  A chain with a custom layer runs layer by layer.
  matrix eval(matrix_view x) const {
    auto *self = const_cast<model *>(this);
    self->sync_from_device();
    if (!device_chain() || !x.num_rows()) {
      matrix cur(x);
      for (const auto &l : layers_) cur = l->forward(cur);
      return cur;
    }
    std::vector<xh_layer> ls;
    std::size_t width = x.num_cols(), widest = width;
    for (const auto &l : layers_) {
      ls.push_back(l->describe());
      width = l->output_cols(width);
      widest = std::max(widest, width);
    }
    const std::vector<float> p = flat_parameters();
    std::vector<float> out(x.num_rows() * widest);
    int oc = 0;
    detail::hip_check(
        xh_model_eval(detail::hip_context(), ls.data(), int(ls.size()),
                      detail::nonnull(const_cast<float *>(p.data())), p.size(),
                      x.flatten().data(), int(x.num_rows()), int(x.num_cols()),
                      out.data(), out.size(), &oc),
        "model::eval");
    return matrix(matrix_view(out.data(), x.num_rows(), std::size_t(oc)));
  }

  // nn.h:481-488: the batch and every layer's output (xh_model_forward: the
  // whole chain in one device call).
  std::vector<matrix> forward(matrix_view batch) const {
    auto *self = const_cast<model *>(this);
    self->sync_from_device();
    std::vector<matrix> input;
    input.emplace_back(batch);
    if (!device_chain() || !batch.num_rows()) {
      for (std::size_t i = 0; i < layers_.size(); ++i)
        input.emplace_back(layers_[i]->forward(input[i]));
      return input;
    }
    std::vector<xh_layer> ls;
    std::vector<std::size_t> w{batch.num_cols()};
    std::size_t total = batch.num_cols();
    for (const auto &l : layers_) {
      ls.push_back(l->describe());
      w.push_back(l->output_cols(w.back()));
      total += w.back();
    }
    const std::size_t rows = batch.num_rows();
    const std::vector<float> p = flat_parameters();
    std::vector<float> acts(rows * total);
    std::vector<int> got(ls.size() + 1);
    detail::hip_check(
        xh_model_forward(detail::hip_context(), ls.data(), int(ls.size()),
                         detail::nonnull(const_cast<float *>(p.data())),
                         p.size(), batch.flatten().data(), int(rows),
                         int(batch.num_cols()), acts.data(), acts.size(),
                         got.data()),
        "model::forward");
    std::size_t off = rows * w[0];
    for (std::size_t l = 1; l < w.size(); ++l) {
      input.emplace_back(matrix_view(acts.data() + off, rows, w[l]));
      off += rows * w[l];
    }
    return input;
  }

  // nn.h:510-528: backpropagate `target` (dL/d output) through the layers;
  // input = forward()'s matrices without the output.  One device call
  // (xh_model_gradient) for a built-in chain.
  vector gradient(const std::vector<matrix> &input, const matrix &target) const {
    if (input.size() < layers_.size())
      throw xeno::error("model::gradient: one input matrix per layer");
    // a fused device learn() may hold newer parameters than the layers
    const_cast<model *>(this)->sync_from_device();
    vector result({parameter_size()});
    const std::size_t rows = layers_.empty() ? 0 : input[0].num_rows();
    // every input of the chain and the target: rows x the chain's widths
    // (the device call reads them by these sizes)
    if (!layers_.empty()) {
      std::size_t w = input[0].num_cols();
      for (std::size_t i = 0; i < layers_.size(); ++i) {
        if (input[i].num_rows() != rows || input[i].num_cols() != w)
          throw xeno::error(xeno::string::strcat(
              "model::gradient: input ", i, " is ", input[i].num_rows(), 'x',
              input[i].num_cols(), ", expected ", rows, 'x', w));
        w = layers_[i]->output_cols(w);
      }
      if (target.num_rows() != rows || target.num_cols() != w)
        throw xeno::error(xeno::string::strcat(
            "model::gradient: target is ", target.num_rows(), 'x',
            target.num_cols(), ", expected ", rows, 'x', w));
    }
    if (!device_chain() || !rows) {
      matrix backprop = target;
      std::size_t off = result.size();
      for (std::size_t i = layers_.size(); i-- > 0;) {
        const std::size_t n = layers_[i]->parameters().size();
        vector g = layers_[i]->gradient(input[i], backprop);
        std::copy(g.begin(), g.begin() + std::min(n, g.size()),
                  result.begin() + (off - n));
        off -= n;
        if (i > 0) backprop = layers_[i]->backward(input[i], backprop);
      }
      return result;
    }
    std::vector<xh_layer> ls;
    std::vector<float> flat;
    for (std::size_t i = 0; i < layers_.size(); ++i) {
      ls.push_back(layers_[i]->describe());
      vector_view v = matrix_view(input[i]).flatten();
      flat.insert(flat.end(), v.begin(), v.end());
    }
    const std::vector<float> p = flat_parameters();
    detail::hip_check(
        xh_model_gradient(detail::hip_context(), ls.data(), int(ls.size()),
                          detail::nonnull(const_cast<float *>(p.data())),
                          p.size(), flat.data(), int(rows),
                          int(input[0].num_cols()),
                          matrix_view(target).flatten().data(),
                          int(target.num_cols()),
                          detail::nonnull(result.data())),
        "model::gradient");
    return result;
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
  // the layers' parameters, concatenated (no device pull)
  std::vector<float> flat_parameters() const {
    std::vector<float> p;
    p.reserve(parameter_size());
    for (const auto &l : layers_) {
      vector_view v = l->parameters();
      p.insert(p.end(), v.begin(), v.end());
    }
    return p;
  }
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

// ------------------------------------------------------------- losses ----
// output, external info per batch (e.g. label): nn.h:531-533
using loss_grad_func = std::function<matrix(matrix_view)>;
using loss_func = std::function<float(matrix_view)>;

// nn.h:535-537: output - label as a column
inline matrix square_loss_grad(vector_view label, matrix_view output) {
  if (output.num_cols() != 1 || output.num_rows() != label.size())
    throw xeno::error("square_loss_grad: output is not one column per label");
  matrix result(output);
  for (std::size_t i = 0; i < label.size(); ++i) result[i][0] -= label[i];
  return result;
}

// nn.h:539-543: mean squared difference
inline float square_loss(vector_view label, matrix_view output) {
  vector_view o = output.flatten();
  if (o.size() != label.size())
    throw xeno::error("square_loss: size mismatch");
  std::vector<float> diff(o.size());
  for (std::size_t i = 0; i < o.size(); ++i) diff[i] = o[i] - label[i];
  float dot = 0.0f;
  for (float d : diff) dot += d * d;
  return dot / label.size();
}

// nn.h:560-570: output - one_hot(labels)
template <typename T>
matrix softmax_cross_entropy_loss_grad(std::span<const T> labels,
                                       std::size_t category_size,
                                       matrix_view output) {
  (void)category_size;
  matrix result(output);
  for (std::size_t i = 0; i < labels.size(); ++i) result[i][labels[i]] -= 1;
  return result;
}

// nn.h:572-574: output - truth
inline matrix softmax_cross_entropy_loss_grad(matrix_view truth,
                                              matrix_view output) {
  if (truth.num_rows() != output.num_rows() ||
      truth.num_cols() != output.num_cols())
    throw xeno::error("softmax_cross_entropy_loss_grad: shape mismatch");
  matrix result(output);
  for (std::size_t i = 0; i < output.num_rows(); ++i)
    for (std::size_t j = 0; j < output.num_cols(); ++j)
      result[i][j] -= truth[i][j];
  return result;
}

// --------------------------------------------------------- optimizers ----
// nn.h:577-698.  step() is the reference's (forward, loss gradient,
// gradient, next_parameters) on the device-backed model; the library's
// optimizers compute next_parameters on the device (xh_optimizer_apply) with
// their state (velocity, moments, step) held here.  When a device learner
// trains the model (the fused learners of policy_gradient.h), it reads the
// description (kind, rate, weight decay, betas) and keeps its own state on
// the device instead.
enum class optimizer_kind { sgd, momentum, adam, custom };

class optimizer {
 public:
  optimizer(model &m, float rate) : model_(m), rate_(rate) {}
  virtual ~optimizer() = default;
  void set_rate(float rate) { rate_ = rate; }
  float rate() const { return rate_; }
  model &target() { return model_; }
  virtual optimizer_kind kind() const { return optimizer_kind::custom; }
  virtual float weight_decay() const { return 0.0f; }
  virtual float beta1() const { return 0.0f; }
  virtual float beta2() const { return 0.0f; }

  // nn.h:594-605
  void step(matrix_view input, const loss_grad_func &loss_grad) {
    std::vector<matrix> inputs = model_.forward(input);
    matrix output = inputs.back();
    inputs.pop_back();
    matrix target = loss_grad(output);
    vector gradient = model_.gradient(inputs, target);
    vector parameters = next_parameters(model_.parameters(), gradient, rate_);
    model_.set_parameters(parameters);
  }

 protected:
  virtual vector next_parameters(const vector &parameters,
                                 const vector &gradient, float rate) = 0;

  // the device update of the library's optimizers
  static vector device_update(int kind, const vector &parameters,
                              const vector &gradient, float rate, float wd,
                              float beta1, float beta2, float t, vector *m,
                              vector *v) {
    if (gradient.size() != parameters.size())
      throw xeno::error("optimizer: gradient / parameter size mismatch");
    vector p = parameters;
    detail::hip_check(
        xh_optimizer_apply(detail::hip_context(), kind, rate, wd, beta1, beta2,
                           t, detail::nonnull(p.data()),
                           detail::nonnull(const_cast<float *>(gradient.data())),
                           m ? m->data() : nullptr, v ? v->data() : nullptr,
                           p.size()),
        "optimizer::next_parameters");
    return p;
  }

 private:
  model &model_;
  float rate_;
};

// p * (1 - wd) - g * lr (nn.h:616-628)
class sgd_optimizer : public optimizer {
 public:
  sgd_optimizer(model &m, float rate, float weight_decay = 0.0f)
      : optimizer(m, rate), weight_decay_(weight_decay) {}
  optimizer_kind kind() const override { return optimizer_kind::sgd; }
  float weight_decay() const override { return weight_decay_; }

 protected:
  vector next_parameters(const vector &parameters, const vector &gradient,
                         float rate) override {
    return device_update(XH_OPT_SGD, parameters, gradient, rate, weight_decay_,
                         0.0f, 0.0f, 1.0f, nullptr, nullptr);
  }

  float weight_decay_;
};

// v = 0.9 v + g; p -= lr v (nn.h:630-657)
class momentum_optimizer : public optimizer {
 public:
  momentum_optimizer(model &m, float rate) : optimizer(m, rate) {}
  optimizer_kind kind() const override { return optimizer_kind::momentum; }
  float beta1() const override { return 0.9f; }

 protected:
  vector next_parameters(const vector &parameters, const vector &gradient,
                         float rate) override {
    if (velocity_.size() != parameters.size()) {  // zeros, on first use
      vector z({parameters.size()});
      z = 0.0f;
      velocity_.swap(z);
    }
    return device_update(XH_OPT_MOMENTUM, parameters, gradient, rate, 0.0f,
                         0.9f, 0.0f, 1.0f, &velocity_, nullptr);
  }

 private:
  vector velocity_;
};

// nn.h:659-698: moments, bias-corrected with t = 1, 2, ...
class adam_optimizer : public optimizer {
 public:
  adam_optimizer(model &m, float rate, float beta1 = 0.9, float beta2 = 0.999)
      : optimizer(m, rate), beta1_(beta1), beta2_(beta2) {}
  optimizer_kind kind() const override { return optimizer_kind::adam; }
  float beta1() const override { return beta1_; }
  float beta2() const override { return beta2_; }

 protected:
  vector next_parameters(const vector &parameters, const vector &gradient,
                         float rate) override {
    if (first_moment_.size() != parameters.size()) {
      vector z1({parameters.size()}), z2({parameters.size()});
      z1 = 0.0f;
      z2 = 0.0f;
      first_moment_.swap(z1);
      second_moment_.swap(z2);
    }
    vector p = device_update(XH_OPT_ADAM, parameters, gradient, rate, 0.0f,
                             beta1_, beta2_, t_, &first_moment_,
                             &second_moment_);
    t_ += 1;
    return p;
  }

 private:
  float beta1_, beta2_;
  float t_ = 1;
  vector first_moment_, second_moment_;
};

}  // namespace xylo

#endif  // XYLO_HIP_COMPAT_NN_H_
