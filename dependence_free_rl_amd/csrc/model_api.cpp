// model_api.cpp -- the reference's generic training API on the device
// (include/xylo_hip.h, "layer / model / optimizer / loss"): model::eval /
// forward / gradient, layer::backward / gradient, the discrete-action loss
// gradients and optimizer::next_parameters, for callers that assemble a
// learner from those pieces (the drop-in layer's xylo::model, optimizer and
// loss functions).  Each call is synchronous on the context's stream, with
// host arrays in and out; its device buffers live for the call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "xh_host.h"
#include "xh_kernels.h"

using namespace xh::host;

namespace {

// A validated layer chain over `cols` input features: per-layer widths
// (w[0] = cols), parameter offsets and the total parameter count.
struct Chain {
  std::vector<xh::ModelLayer> layers;
  std::vector<int> width;      // nlayers + 1
  std::vector<size_t> poff;    // nlayers + 1 (poff[nl] = parameter count)
};

int dense_params(const xh_layer &L) {
  return L.kind == XH_LAYER_FULL || L.kind == XH_LAYER_CONV1D_1
             ? L.out * L.in + L.out
             : 0;
}

int check_layer(const xh_layer &L, int c, int l, const char *what, int *out_c) {
  switch (L.kind) {
    case XH_LAYER_FULL:
    case XH_LAYER_CONV1D_1:
      if (L.in < 1 || L.out < 1 ||
          (L.kind == XH_LAYER_FULL ? c != L.in : c % L.in != 0))
        return fail(XH_ERR_INVALID, "%s: layer %d (%d -> %d) on %d features",
                    what, l, L.in, L.out, c);
      *out_c = L.kind == XH_LAYER_FULL ? L.out : c / L.in * L.out;
      return XH_OK;
    case XH_LAYER_RELU:
    case XH_LAYER_SOFTMAX:
    case XH_LAYER_SOFTMAX_XENT:
      *out_c = c;
      return XH_OK;
    default:
      return fail(XH_ERR_INVALID, "%s: layer %d kind %d", what, l, L.kind);
  }
}

int make_chain(const xh_layer *layers, int nlayers, int cols, size_t nparams,
               const char *what, Chain *ch) {
  if (!layers || nlayers < 1) return fail(XH_ERR_INVALID, "%s: no layers", what);
  ch->layers.resize((size_t)nlayers);
  ch->width.assign((size_t)nlayers + 1, cols);
  ch->poff.assign((size_t)nlayers + 1, 0);
  int c = cols;
  for (int l = 0; l < nlayers; ++l) {
    const xh_layer &L = layers[l];
    ch->layers[l] = xh::ModelLayer{L.kind, L.in, L.out};
    CHK(check_layer(L, c, l, what, &c));
    ch->width[l + 1] = c;
    ch->poff[l + 1] = ch->poff[l] + (size_t)dense_params(L);
  }
  if (ch->poff[nlayers] != nparams)
    return fail(XH_ERR_INVALID, "%s: %zu parameters, the layers need %zu", what,
                nparams, ch->poff[nlayers]);
  return XH_OK;
}

// One device allocation carved into float regions; freed with the call.
struct Scratch {
  float *base = nullptr;
  ~Scratch() {
    if (base) (void)hipFree(base);
  }
  int alloc(size_t floats) {
    if (hipMalloc((void **)&base, sizeof(float) * std::max<size_t>(floats, 1)) !=
        hipSuccess)
      return fail(XH_ERR_HIP, "allocating %zu floats", floats);
    return XH_OK;
  }
};

int upload(float *dev, const float *host, size_t n, hipStream_t s) {
  return n ? copy_ok(copy_to_device(dev, host, n * 4, s)) : XH_OK;
}
int download(float *host, const float *dev, size_t n, hipStream_t s) {
  return n ? copy_ok(copy_to_host(host, dev, n * 4, s)) : XH_OK;
}
int launched(hipError_t e, const char *what) {
  return e == hipSuccess ? XH_OK
                         : fail(XH_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

}  // namespace

// ---------------------------------------------------------- model::eval --
int xh_model_eval(xh_ctx *ctx, const xh_layer *layers, int nlayers,
                  const float *params, size_t nparams, const float *x,
                  int rows, int cols, float *out, size_t out_cap,
                  int *out_cols) {
  return guard([&]() -> int {
    if (!ctx || !layers || nlayers < 1 || !params || !x || !out || !out_cols)
      return fail(XH_ERR_INVALID, "model_eval: null arg");
    if (rows < 1 || cols < 1)
      return fail(XH_ERR_INVALID, "model_eval: %d x %d input", rows, cols);
    Chain ch;
    CHK(make_chain(layers, nlayers, cols, nparams, "model_eval", &ch));
    const int c = ch.width[nlayers];
    const size_t widest = *std::max_element(ch.width.begin(), ch.width.end());
    if ((size_t)rows * c > out_cap)
      return fail(XH_ERR_INVALID, "model_eval: output needs %zu floats, "
                  "capacity %zu", (size_t)rows * c, out_cap);
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t act = (size_t)rows * widest;
    HIPCHK(hipStreamSynchronize(s));
    Scratch sc;
    CHK(sc.alloc(nparams + 3 * act));
    float *dp = sc.base, *dx = dp + nparams, *da = dx + act, *db = da + act;
    CHK(upload(dp, params, nparams, s));
    CHK(upload(dx, x, (size_t)rows * cols, s));
    const float *res = nullptr;
    int oc = 0;
    CHK(launched(xh::model_forward(ch.layers.data(), nlayers, dp, dx, rows, cols,
                                   da, db, &res, &oc, s),
                 "model_eval"));
    CHK(download(out, res, (size_t)rows * oc, s));
    *out_cols = oc;
    return XH_OK;
  });
}

// -------------------------------------------------------- model::forward --
int xh_model_forward(xh_ctx *ctx, const xh_layer *layers, int nlayers,
                     const float *params, size_t nparams, const float *x,
                     int rows, int cols, float *acts, size_t acts_cap,
                     int *widths) {
  return guard([&]() -> int {
    if (!ctx || !params || !x || !acts || !widths)
      return fail(XH_ERR_INVALID, "model_forward: null arg");
    if (rows < 1 || cols < 1)
      return fail(XH_ERR_INVALID, "model_forward: %d x %d input", rows, cols);
    Chain ch;
    CHK(make_chain(layers, nlayers, cols, nparams, "model_forward", &ch));
    std::vector<size_t> aoff((size_t)nlayers + 2, 0);
    for (int l = 0; l <= nlayers; ++l)
      aoff[l + 1] = aoff[l] + (size_t)rows * ch.width[l];
    if (aoff[nlayers + 1] > acts_cap)
      return fail(XH_ERR_INVALID, "model_forward: activations need %zu floats, "
                  "capacity %zu", aoff[nlayers + 1], acts_cap);
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    HIPCHK(hipStreamSynchronize(s));
    Scratch sc;
    CHK(sc.alloc(nparams + aoff[nlayers + 1]));
    float *dp = sc.base, *da = dp + nparams;
    CHK(upload(dp, params, nparams, s));
    CHK(upload(da, x, (size_t)rows * cols, s));
    for (int l = 0; l < nlayers; ++l)
      CHK(launched(xh::layer_forward(ch.layers[l], dp + ch.poff[l], da + aoff[l],
                                     rows, ch.width[l], da + aoff[l + 1], s),
                   "model_forward"));
    CHK(download(acts, da, aoff[nlayers + 1], s));
    for (int l = 0; l <= nlayers; ++l) widths[l] = ch.width[l];
    return XH_OK;
  });
}

// ------------------------------------------------------- model::gradient --
int xh_model_gradient(xh_ctx *ctx, const xh_layer *layers, int nlayers,
                      const float *params, size_t nparams, const float *inputs,
                      int rows, int cols, const float *target, int target_cols,
                      float *grad) {
  return guard([&]() -> int {
    if (!ctx || !inputs || !target || (nparams && (!params || !grad)))
      return fail(XH_ERR_INVALID, "model_gradient: null arg");
    if (rows < 1 || cols < 1)
      return fail(XH_ERR_INVALID, "model_gradient: %d x %d input", rows, cols);
    Chain ch;
    CHK(make_chain(layers, nlayers, cols, nparams, "model_gradient", &ch));
    if (target_cols != ch.width[nlayers])
      return fail(XH_ERR_INVALID, "model_gradient: target has %d columns, the "
                  "output %d", target_cols, ch.width[nlayers]);
    std::vector<size_t> aoff((size_t)nlayers + 1, 0);
    for (int l = 0; l < nlayers; ++l)
      aoff[l + 1] = aoff[l] + (size_t)rows * ch.width[l];
    const size_t widest =
        (size_t)rows * *std::max_element(ch.width.begin(), ch.width.end());
    size_t stride = 0;
    int splits = 0;
    for (int l = 0; l < nlayers; ++l) {
      stride = std::max(stride, ch.poff[l + 1] - ch.poff[l]);
      splits = std::max(splits, xh::layer_gradient_splits(ch.layers[l], rows,
                                                           ch.width[l]));
    }
    stride = (stride + 63) & ~(size_t)63;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    HIPCHK(hipStreamSynchronize(s));
    Scratch sc;
    CHK(sc.alloc(2 * nparams + aoff[nlayers] + 2 * widest + stride * splits));
    float *dp = sc.base, *dg = dp + nparams, *din = dg + nparams;
    float *bp = din + aoff[nlayers], *bq = bp + widest, *slab = bq + widest;
    CHK(upload(dp, params, nparams, s));
    CHK(upload(din, inputs, aoff[nlayers], s));
    CHK(upload(bp, target, (size_t)rows * target_cols, s));
    // nn.h:510-528: gradient then backward from the last layer; layer 0 gets
    // its gradient only
    for (int l = nlayers - 1; l >= 0; --l) {
      const xh::ModelLayer &L = ch.layers[l];
      CHK(launched(xh::layer_gradient(L, din + aoff[l], rows, ch.width[l], bp,
                                      slab, (int)stride, dg + ch.poff[l], s),
                   "model_gradient"));
      if (l == 0) break;
      CHK(launched(xh::layer_backward(L, dp + ch.poff[l], din + aoff[l], rows,
                                      ch.width[l], bp, bq, s),
                   "model_gradient"));
      std::swap(bp, bq);
    }
    CHK(download(grad, dg, nparams, s));
    return XH_OK;
  });
}

// ---------------------------------------------- layer::backward / gradient --
int xh_layer_backward(xh_ctx *ctx, const xh_layer *layer, const float *params,
                      size_t nparams, const float *input, int rows, int cols,
                      const float *backprop, int bp_cols, float *out) {
  return guard([&]() -> int {
    if (!ctx || !layer || !input || !backprop || !out)
      return fail(XH_ERR_INVALID, "layer_backward: null arg");
    if (rows < 1 || cols < 1)
      return fail(XH_ERR_INVALID, "layer_backward: %d x %d input", rows, cols);
    Chain ch;
    CHK(make_chain(layer, 1, cols, nparams, "layer_backward", &ch));
    if (nparams && !params)
      return fail(XH_ERR_INVALID, "layer_backward: null params");
    if (bp_cols != ch.width[1])
      return fail(XH_ERR_INVALID, "layer_backward: backprop has %d columns, "
                  "the layer's output %d", bp_cols, ch.width[1]);
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    HIPCHK(hipStreamSynchronize(s));
    const size_t ni = (size_t)rows * cols, nb = (size_t)rows * bp_cols;
    Scratch sc;
    CHK(sc.alloc(nparams + 2 * ni + nb));
    float *dp = sc.base, *dx = dp + nparams, *db = dx + ni, *dout = db + nb;
    CHK(upload(dp, params, nparams, s));
    CHK(upload(dx, input, ni, s));
    CHK(upload(db, backprop, nb, s));
    CHK(launched(xh::layer_backward(ch.layers[0], dp, dx, rows, cols, db, dout, s),
                 "layer_backward"));
    CHK(download(out, dout, ni, s));
    return XH_OK;
  });
}

int xh_layer_gradient(xh_ctx *ctx, const xh_layer *layer, const float *input,
                      int rows, int cols, const float *backprop, int bp_cols,
                      float *grad, size_t ngrad) {
  return guard([&]() -> int {
    if (!ctx || !layer || !input || !backprop || (ngrad && !grad))
      return fail(XH_ERR_INVALID, "layer_gradient: null arg");
    if (rows < 1 || cols < 1)
      return fail(XH_ERR_INVALID, "layer_gradient: %d x %d input", rows, cols);
    Chain ch;
    CHK(make_chain(layer, 1, cols, ngrad, "layer_gradient", &ch));
    if (bp_cols != ch.width[1])
      return fail(XH_ERR_INVALID, "layer_gradient: backprop has %d columns, "
                  "the layer's output %d", bp_cols, ch.width[1]);
    if (!ngrad) return XH_OK;  // activations have no parameters
    const int splits = xh::layer_gradient_splits(ch.layers[0], rows, cols);
    const size_t stride = (ngrad + 63) & ~(size_t)63;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    HIPCHK(hipStreamSynchronize(s));
    const size_t ni = (size_t)rows * cols, nb = (size_t)rows * bp_cols;
    Scratch sc;
    CHK(sc.alloc(ni + nb + ngrad + stride * splits));
    float *dx = sc.base, *db = dx + ni, *dg = db + nb, *slab = dg + ngrad;
    CHK(upload(dx, input, ni, s));
    CHK(upload(db, backprop, nb, s));
    CHK(launched(xh::layer_gradient(ch.layers[0], dx, rows, cols, db, slab,
                                    (int)stride, dg, s),
                 "layer_gradient"));
    CHK(download(grad, dg, ngrad, s));
    return XH_OK;
  });
}

// --------------------------------------------------- action loss gradients --
int xh_action_loss_grad(xh_ctx *ctx, int kind, int rows, int range,
                        const int32_t *choice, const float *distrib,
                        const float *advantage, const float *probs, float param,
                        float *out) {
  return guard([&]() -> int {
    if (!ctx || !choice || !advantage || !probs || !out)
      return fail(XH_ERR_INVALID, "action_loss_grad: null arg");
    if (kind < XH_LOSS_GRADIENT_LOG || kind > XH_LOSS_KL_REGULATED)
      return fail(XH_ERR_INVALID, "action_loss_grad: kind %d", kind);
    if (kind != XH_LOSS_SOFTMAX_GRADIENT_LOG && !distrib)
      return fail(XH_ERR_INVALID, "action_loss_grad: kind %d needs the sampling "
                  "distributions", kind);
    if (rows < 0 || range < 1)
      return fail(XH_ERR_INVALID, "action_loss_grad: %d rows x %d", rows, range);
    for (int r = 0; r < rows; ++r)  // rl.h throws on a wrong-size input
      if (choice[r] < 0 || choice[r] >= range)
        return fail(XH_ERR_INVALID, "action_loss_grad: row %d choice %d outside "
                    "[0, %d)", r, choice[r], range);
    if (!rows) return XH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    HIPCHK(hipStreamSynchronize(s));
    const size_t n = (size_t)rows * range;
    Scratch sc;
    CHK(sc.alloc(3 * n + 2 * (size_t)rows));
    float *dq = sc.base, *dpb = dq + n, *dout = dpb + n, *dadv = dout + n;
    int32_t *dch = reinterpret_cast<int32_t *>(dadv + rows);
    if (distrib) CHK(upload(dq, distrib, n, s));
    CHK(upload(dpb, probs, n, s));
    CHK(upload(dadv, advantage, (size_t)rows, s));
    CHK(copy_ok(copy_to_device(dch, choice, (size_t)rows * 4, s)));
    CHK(launched(xh::launch_action_loss(kind, rows, range, dch,
                                        distrib ? dq : nullptr, dadv, dpb, param,
                                        dout, s),
                 "action_loss_grad"));
    CHK(download(out, dout, n, s));
    return XH_OK;
  });
}

// --------------------------------------------- optimizer::next_parameters --
int xh_optimizer_apply(xh_ctx *ctx, int kind, float lr, float weight_decay,
                       float beta1, float beta2, float t, float *params,
                       const float *grad, float *m, float *v, size_t n) {
  return guard([&]() -> int {
    if (!ctx || (n && (!params || !grad)))
      return fail(XH_ERR_INVALID, "optimizer_apply: null arg");
    if (kind != XH_OPT_SGD && kind != XH_OPT_MOMENTUM && kind != XH_OPT_ADAM)
      return fail(XH_ERR_INVALID, "optimizer_apply: kind %d", kind);
    if ((kind != XH_OPT_SGD && n && !m) || (kind == XH_OPT_ADAM && n && !v))
      return fail(XH_ERR_INVALID, "optimizer_apply: missing optimizer state");
    if (n > (size_t)0x7fffffff)
      return fail(XH_ERR_INVALID, "optimizer_apply: %zu parameters", n);
    if (!n) return XH_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    HIPCHK(hipStreamSynchronize(s));
    Scratch sc;
    CHK(sc.alloc(4 * n));
    float *dp = sc.base, *dg = dp + n, *dm = dg + n, *dv = dm + n;
    CHK(upload(dp, params, n, s));
    CHK(upload(dg, grad, n, s));
    xh::OptStep o{};
    o.kind = kind;
    o.lr = lr;
    o.wd = weight_decay;
    o.beta1 = beta1;
    o.beta2 = beta2;
    if (kind == XH_OPT_ADAM) {  // host float powf, as the reference (nn.h:684)
      o.c1 = 1 - powf(beta1, t);
      o.c2 = 1 - powf(beta2, t);
    }
    if (kind == XH_OPT_SGD) {
      CHK(launched(xh::launch_sgd(dp, dg, (int)n, lr, weight_decay, s),
                   "optimizer_apply"));
    } else {
      CHK(upload(dm, m, n, s));
      if (kind == XH_OPT_ADAM) CHK(upload(dv, v, n, s));
      CHK(launched(xh::launch_opt(dp, dg, dm, dv, (int)n, o, s),
                   "optimizer_apply"));
      CHK(download(m, dm, n, s));
      if (kind == XH_OPT_ADAM) CHK(download(v, dv, n, s));
    }
    CHK(download(params, dp, n, s));
    return XH_OK;
  });
}
