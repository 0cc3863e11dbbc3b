// xylo_hip.cpp -- host runtime behind the C ABI (include/xylo_hip.h).
//
// One xh_trainer owns every device buffer of the vectorised PPO / AC path and
// drives it on one HIP stream: T rollout-step kernels, then learn() in the
// reference order (policy_gradient.h:159-185): value eval -> TD targets ->
// value SGD step -> value re-eval -> GAE -> k policy epochs.  With world > 1
// each flat gradient is SUM-all-reduced with RCCL on the same stream before
// the identical SGD step on every rank (the reference's loss is a sum over
// rows, nn.h:94-98, so the sharded sum equals the single-process gradient).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <string>
#include <vector>

#include "../../include/xylo_hip.h"
#include "xh_host.h"
#include "xh_kernels.h"

using namespace xh::host;

namespace {

uint32_t mstd_pow(uint64_t k) {  // 16807^k mod (2^31-1)
  uint64_t acc = 1, base = 16807;
  while (k) {
    if (k & 1) acc = acc * base % 2147483647ull;
    base = base * base % 2147483647ull;
    k >>= 1;
  }
  return (uint32_t)acc;
}

}  // namespace

namespace {
void ctx_free(xh_ctx *c) {
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->comm) ncclCommDestroy(c->comm);
  (void)hipStreamDestroy(c->stream);
  delete c;
}
}  // namespace

struct timed_event {
  std::string name;
  hipEvent_t start, stop;
};

struct xh_trainer {
  xh_ctx *ctx = nullptr;
  xh_config cfg{};
  xh::EnvDesc env{};
  xh::PolicyLayout pl{};
  xh::ValueLayout vl{};
  int np = 0, nv = 0;
  // trajectory batch
  int8_t *bins = nullptr, *items = nullptr;
  int32_t *action = nullptr, *forced = nullptr;
  float *pold = nullptr;
  uint8_t *done = nullptr;
  uint32_t *rng = nullptr;
  // parameters and learner buffers
  float *pp = nullptr, *vp = nullptr;
  float *v_state = nullptr, *v_state0 = nullptr, *v_term = nullptr;
  float *targets = nullptr, *adv = nullptr;
  float *row_g = nullptr;               // [T*N] dL/dV of the value step
  float *vact[2] = {nullptr, nullptr};  // value layer 1 / 2 outputs
  float *vgr[2] = {nullptr, nullptr};   // their dL/d(pre-activation)
  float *pslab = nullptr, *vslab = nullptr;
  float *vw0red = nullptr;  // value layer 0 on the reduced observation
  uint8_t *vw0frag = nullptr;  // W0's bf16 fragments (value_net_kernels.hip)
  // vw0frag holds the fragments of the current value parameters (set by a
  // bf16 value forward, cleared by every write of vp): the next iteration's
  // first forward then skips the preparation launch
  bool vfrag_ready = false;
  int pslab_stride = 0, vslab_stride = 0, pslab_n = 0, vslab_n = 0;
  float *pgrads = nullptr, *vgrad = nullptr;
  float *logits = nullptr, *probs = nullptr;
  double *adv_part = nullptr, *adv_stats = nullptr;  // adv_normalize
  // KL-PPO state
  float *qold = nullptr, *beta = nullptr, *kl_log = nullptr;
  int *end_list = nullptr, *n_end = nullptr, *n_open = nullptr;
  int *vrows = nullptr;  // device: (T+1)N + n_end rows of the first V batch
  int *end_scratch = nullptr;  // launch_end_list_par's block totals
  double *kl_part = nullptr, *kl_sum = nullptr;
  // optimizers of the policy [0] and value [1] nets (nn.h:589-698)
  struct opt_state {
    int kind = XH_OPT_SGD;
    float lr = 0, wd = 0, beta1 = 0.9f, beta2 = 0.999f;
    float t = 1.0f;                    // adam_optimizer::t (nn.h:694)
    float *m = nullptr, *v = nullptr;  // velocity / moments (device)
  } opt[2];
  // REINFORCE (XH_PG): full-MLP policy buffers and episode bookkeeping
  struct pg_state {
    int nlayers = 0, w[4] = {0, 0, 0, 0};
    float *act[3] = {nullptr, nullptr, nullptr};
    float *grad[3] = {nullptr, nullptr, nullptr};
    int *ep_done = nullptr, *len = nullptr, *active = nullptr;
    int *row_off = nullptr, *list = nullptr, *nrows = nullptr;
    float *rtg = nullptr;
    double *ep_part = nullptr, *stats = nullptr;
    int *host_active = nullptr;  // pinned
    int slot_end = 0;            // slot holding the envs' current states
  } pg;
  int Tb = 0;  // Batch steps: cfg.steps, or REINFORCE's per-iteration bound
  uint32_t jump_mul = 1;
  int rgrid = 0;
  bool need_shift = false;
  // a rollout window exists that no learn() / forget() has consumed yet
  // (xh_trainer_forget refuses to shift without one)
  bool rolled = false;
  // XH_BUF_LOGITS / XH_BUF_PROBS hold a recorded rollout step
  bool last_step_recorded = false;
  // xh_trainer_set_env_state: states the next rollout starts from, keyed by
  // env (B*D bin bytes then D item bytes), applied after the forget() shift
  std::map<int, std::vector<int8_t>> env_override;
  bool use_forced = false;
  // Slots of `items` whose every env holds an item-table entry.  The train
  // kernels fold the item's layer-1 contribution into per-table-entry biases,
  // so learn() refuses a batch that reads a slot with any other item
  // (xh_trainer_set_buffer accepts them for rollout-only use).
  std::vector<char> items_ok;
  // Slots of `bins` that may hold a bin below -capacity (an overflowed state
  // the reference reaches by applying to a game-over env again, bin_packing.h:
  // 53-63, uploaded by hand).  The f16-pair kernels bound every observation
  // feature by |bins / capacity| <= 1, so a rollout step
  // or learn() that reads such a slot runs the f32-MFMA kernels instead.
  std::vector<char> bins_wide;
  // what the last rollout step / policy epoch launched (xh_trainer_kernel_info)
  xh::KernelInfo last_rollout, last_train;
  int timing = 0;  // 0 off, 1 every launch, XH_TIMING_TRAIN policy_train only
  bool counted = false;  // holds a reference on ctx
  std::vector<timed_event> events;
  std::vector<hipEvent_t> event_pool;  // recycled by reset_timing
  std::vector<void *> allocs;

  xh::Batch batch() const {
    xh::Batch b;
    b.N = cfg.num_envs;
    b.T = Tb;
    b.bins = bins;
    b.items = items;
    b.action = action;
    b.pold = pold;
    b.done = done;
    b.rng = rng;
    return b;
  }
  xh::ValueArgs vargs() const {
    xh::ValueArgs a{};
    a.env = env;
    a.b = batch();
    a.v_state = v_state;
    a.v_term = v_term;
    a.row_g = row_g;
    return a;
  }
  size_t N() const { return (size_t)cfg.num_envs; }
  size_t T() const { return (size_t)Tb; }
  size_t BD() const { return (size_t)cfg.bins * cfg.dims; }
};

// N vectorised envs for a caller's own policy (xh_venv_*, venv_kernels.hip).
struct xh_venv {
  xh_ctx *ctx = nullptr;
  xh::EnvDesc env{};
  int N = 0, Ng = 0, offset = 0, policy_draws = 0;
  uint32_t skip_mul = 1, jump_mul = 1;
  void *buf[XH_VENV_BUF_COUNT] = {};
  size_t bytes[XH_VENV_BUF_COUNT] = {};
  int *err = nullptr;
  bool counted = false;
  // xh_venv_set_timing: HIP events around every step / apply / reset /
  // observe launch on the context's stream
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;  // recorded pairs
  std::vector<hipEvent_t> event_pool;  // recycled by set_timing

  xh::VenvArgs args() const {
    xh::VenvArgs a{};
    a.env = env;
    a.N = N;
    a.bins = (int8_t *)buf[XH_VENV_BINS];
    a.items = (int8_t *)buf[XH_VENV_ITEMS];
    a.rng = (uint32_t *)buf[XH_VENV_RNG];
    a.action = (const int32_t *)buf[XH_VENV_ACTIONS];
    a.reward = (float *)buf[XH_VENV_REWARD];
    a.done = (uint8_t *)buf[XH_VENV_DONE];
    a.err = err;
    a.skip_mul = skip_mul;
    a.jump_mul = jump_mul;
    return a;
  }
};

namespace {

template <class P>
int dalloc(xh_trainer *t, P **p, size_t bytes) {
  void *q = nullptr;
  HIPCHK(hipMalloc(&q, bytes < 16 ? 16 : bytes));
  // zeroed on the trainer's stream: a null-stream hipMemset is not ordered
  // before the non-blocking stream's next copy / kernel (measured: the zero
  // fill landing after the parameter upload, intermittently)
  HIPCHK(hipMemsetAsync(q, 0, bytes < 16 ? 16 : bytes, t->ctx->stream));
  t->allocs.push_back(q);
  *p = reinterpret_cast<P *>(q);
  return XH_OK;
}

// Timing events come from a pool (reset_timing returns them), without the
// system-scope fence: they only time launches, every host read of device
// memory synchronises the stream itself.
hipError_t pooled_event(xh_trainer *t, hipEvent_t *e) {
  if (!t->event_pool.empty()) {
    *e = t->event_pool.back();
    t->event_pool.pop_back();
    return hipSuccess;
  }
  return hipEventCreateWithFlags(e, hipEventDisableSystemFence);
}

// Launch wrapper: optional HIP-event timing on the trainer's stream.
template <class F>
int timed(xh_trainer *t, const char *name, F &&launch) {
  hipStream_t s = t->ctx->stream;
  timed_event ev;
  const bool rec = t->timing == 1 ||
                   (t->timing == XH_TIMING_TRAIN && std::strcmp(name, "policy_train") == 0);
  if (rec) {
    ev.name = name;
    HIPCHK(pooled_event(t, &ev.start));
    HIPCHK(pooled_event(t, &ev.stop));
    HIPCHK(hipEventRecord(ev.start, s));
  }
  hipError_t e = launch();
  if (e != hipSuccess)
    return fail(XH_ERR_HIP, "launch %s: %s", name, hipGetErrorString(e));
  if (rec) {
    HIPCHK(hipEventRecord(ev.stop, s));
    t->events.push_back(ev);
  }
  return XH_OK;
}

// SUM all-reduce of a flat device buffer on the trainer's stream.  An RCCL
// failure is reported as XH_ERR_RCCL with ncclGetErrorString (and the
// communicator's async error, if it holds one), not as a HIP error.
int allreduce_t(xh_trainer *t, void *buf, int n, ncclDataType_t dt) {
  if (!t->ctx->comm) return XH_OK;
  hipStream_t s = t->ctx->stream;
  ncclResult_t r = ncclSuccess;
  if (t->ctx->fault == XH_FAULT_RCCL_ARG) {
    // test hook: the next all-reduce passes RCCL an invalid datatype, so RCCL
    // itself rejects the call
    dt = (ncclDataType_t)ncclNumTypes;
    t->ctx->fault = 0;
  }
  const int st = timed(t, "allreduce", [&]() -> hipError_t {
    r = ncclAllReduce(buf, buf, (size_t)n, dt, ncclSum, t->ctx->comm, s);
    return hipSuccess;
  });
  if (st != XH_OK) return st;
  if (r != ncclSuccess) {
    ncclResult_t ar = ncclSuccess;
    (void)ncclCommGetAsyncError(t->ctx->comm, &ar);
    return fail(XH_ERR_RCCL, "ncclAllReduce(%d x %s, rank %d of %d): %s%s%s", n,
                dt == ncclFloat64 ? "f64" : dt == ncclFloat32 ? "f32" : "?",
                t->ctx->rank, t->ctx->world,
                ncclGetErrorString(r), ar != ncclSuccess ? "; async: " : "",
                ar != ncclSuccess ? ncclGetErrorString(ar) : "");
  }
  return XH_OK;
}
int allreduce(xh_trainer *t, float *buf, int n) {
  return allreduce_t(t, buf, n, ncclFloat32);
}
int allreduce_d(xh_trainer *t, double *buf, int n) {
  return allreduce_t(t, buf, n, ncclFloat64);
}

size_t buffer_bytes(const xh_trainer *t, int which) {
  const size_t N = t->N(), T = t->T();
  switch (which) {
    case XH_BUF_BINS: return (T + 1) * N * t->BD();
    case XH_BUF_ITEMS: return (T + 1) * N * 4;
    case XH_BUF_ACTION: return T * N * 4;
    case XH_BUF_POLD: return T * N * 4;
    case XH_BUF_DONE: return T * N;
    case XH_BUF_RNG: return N * 4;
    case XH_BUF_V_STATE: return (T + 1) * N * 4;
    case XH_BUF_V_STATE0: return (T + 1) * N * 4;
    case XH_BUF_V_TERM: return T * N * 4;
    case XH_BUF_TARGETS: return T * N * 4;
    case XH_BUF_ADV: return T * N * 4;
    case XH_BUF_VALUE_GRAD: return (size_t)t->nv * 4;
    case XH_BUF_POLICY_GRADS: return (size_t)t->cfg.epochs * t->np * 4;
    case XH_BUF_LOGITS: return N * t->cfg.bins * 4;
    case XH_BUF_PROBS: return N * t->cfg.bins * 4;
    case XH_BUF_QOLD: return t->qold ? T * N * t->cfg.bins * 4 : 0;
    case XH_BUF_KL: return t->kl_log ? (size_t)t->cfg.epochs * 12 : 0;
    case XH_BUF_LEN: return t->pg.len ? N * 4 : 0;
  }
  return 0;
}

void *buffer_ptr(const xh_trainer *t, int which) {
  switch (which) {
    case XH_BUF_BINS: return t->bins;
    case XH_BUF_ITEMS: return t->items;
    case XH_BUF_ACTION: return t->action;
    case XH_BUF_POLD: return t->pold;
    case XH_BUF_DONE: return t->done;
    case XH_BUF_RNG: return t->rng;
    case XH_BUF_QOLD: return t->qold;
    case XH_BUF_KL: return t->kl_log;
    case XH_BUF_V_STATE: return t->v_state;
    case XH_BUF_V_STATE0: return t->v_state0;
    case XH_BUF_V_TERM: return t->v_term;
    case XH_BUF_TARGETS: return t->targets;
    case XH_BUF_ADV: return t->adv;
    case XH_BUF_VALUE_GRAD: return t->vgrad;
    case XH_BUF_POLICY_GRADS: return t->pgrads;
    case XH_BUF_LOGITS: return t->logits;
    case XH_BUF_PROBS: return t->probs;
    case XH_BUF_LEN: return t->pg.len;
  }
  return nullptr;
}

constexpr uint64_t kEvalStride = 1ull << 26;  // draws between env streams
// row groups one policy-train workgroup sums into its gradient slab at most
// (= BASELINE configs 3 and 5 per GPU: 131072 groups over 256 workgroups)
constexpr int kMaxTrainDepth = 512;
constexpr int kBinCapacity = 8;             // bin_packing.h:48, every dim

xh::EnvDesc make_env(int bins, int dims) {
  static const int ia[3][3] = {{4, 0, 0}, {4, 2, 0}, {4, 2, 2}};
  static const int ib[3][3] = {{1, 0, 0}, {1, 2, 0}, {1, 2, 1}};
  xh::EnvDesc env{};
  env.B = bins;
  env.D = dims;
  for (int d = 0; d < 3; ++d) {
    env.item_a[d] = ia[dims - 1][d];
    env.item_b[d] = ib[dims - 1][d];
  }
  env.p_a = 0.4;
  return env;
}

struct EvalBuffers {
  uint32_t x0;
  long max_steps;
  const int *init_items;
  double *total;
  long *steps;
  uint32_t *rng_out;
  int *final_items;
  int *trace;
  long trace_cap;
};

// Shared host side of the episode evaluators (xh_trainer_evaluate,
// xh_heuristic_evaluate): one device scratch block for the per-env outputs,
// the launch bracketed by HIP events (e->elapsed_ms), copies back, sync.
template <class Launch>
int eval_common(xh_ctx *ctx, const xh::EnvDesc &env, int G, xh_eval *e,
                Launch launch) {
  const int n = e->n_envs, D = env.D;
  if (n <= 0 || n % G || e->episodes < 0 || e->trace_cap < 0)
    return fail(XH_ERR_INVALID, "evaluate: n_envs %d (multiple of %d), "
                "episodes %d", n, G, e->episodes);
  if (e->init_items)
    for (long i = 0; i < (long)n * D; ++i)
      if (e->init_items[i] != env.item_a[i % D] &&
          e->init_items[i] != env.item_b[i % D])
        return fail(XH_ERR_INVALID, "evaluate: init_items[%ld] = %d is not "
                    "an item of the table", i, e->init_items[i]);
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_steps = up(sizeof(double) * n),
               o_rng = o_steps + up(8 * (size_t)n),
               o_init = o_rng + up(4 * (size_t)n),
               o_fin = o_init + up(4 * (size_t)n * D),
               o_trace = o_fin + up(4 * (size_t)n * D),
               bytes = o_trace + up(4 * (size_t)(e->trace ? e->trace_cap : 0));
  // a plain device allocation, each region on its own 256-byte boundary
  // (the stream-ordered allocator returned trace bytes that read back wrong
  // for some sizes on ROCm 7.2: measured at trace_cap 2049 and 10000)
  char *scratch = nullptr;
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipMalloc((void **)&scratch, bytes));
  EvalBuffers eb{};
  const uint32_t x0 = e->rng_state % 2147483647u;
  eb.x0 = x0 ? x0 : 1u;
  // an episode lasts at most B * capacity * D + 1 steps (every step puts at
  // least one unit into some bin)
  eb.max_steps = (long)(e->episodes + 1) * (env.B * 8 * D + 2);
  eb.total = (double *)scratch;
  eb.steps = (long *)(scratch + o_steps);
  eb.rng_out = (uint32_t *)(scratch + o_rng);
  eb.final_items = (int *)(scratch + o_fin);
  eb.trace = e->trace ? (int *)(scratch + o_trace) : nullptr;
  eb.trace_cap = e->trace ? e->trace_cap : 0;
  int st = XH_OK;
  if (e->init_items) {
    eb.init_items = (const int *)(scratch + o_init);
    st = copy_ok(copy_to_device(scratch + o_init, e->init_items,
                                4 * (size_t)n * D, s));
  }
  // from here on a failure is recorded in `st` and the scratch block, the
  // events and the stream are still released / drained below
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  auto hip_ok = [&](hipError_t e, const char *what) {
    if (st == XH_OK && e != hipSuccess)
      st = fail(XH_ERR_HIP, "evaluate %s: %s", what, hipGetErrorString(e));
    return st == XH_OK;
  };
  if (st == XH_OK && hip_ok(hipEventCreate(&ev0), "event") &&
      hip_ok(hipEventCreate(&ev1), "event") &&
      hip_ok(hipEventRecord(ev0, s), "event record")) {
    if (hip_ok(launch(eb), "launch")) hip_ok(hipEventRecord(ev1, s), "event record");
  }
  auto out = [&](void *host, size_t off, size_t nb) {
    if (st == XH_OK && host)
      st = copy_ok(copy_to_host(host, scratch + off, nb, s));
  };
  out(e->totals, 0, sizeof(double) * n);
  out(e->steps, o_steps, 8 * (size_t)n);
  out(e->rng_out, o_rng, 4 * (size_t)n);
  out(e->final_items, o_fin, 4 * (size_t)n * D);
  out(e->trace, o_trace, 4 * (size_t)eb.trace_cap);
  (void)hipStreamSynchronize(s);
  (void)hipFree(scratch);
  hip_ok(hipStreamSynchronize(s), "synchronize");
  float ms = 0.0f;
  if (st == XH_OK && hipEventElapsedTime(&ms, ev0, ev1) == hipSuccess)
    e->elapsed_ms = ms;
  if (ev0) (void)hipEventDestroy(ev0);
  if (ev1) (void)hipEventDestroy(ev1);
  return st;
}

// optimizer::step's next_parameters for net `which` (nn.h:594-698).
// The optimizer step's scalars (advances adam's step counter).
xh::OptStep opt_step(xh_trainer *t, int which) {
  auto &o = t->opt[which];
  // lr_scale_rows (opt-in): lr / rows of the job instead of the raw lr on
  // the row-summed gradient (nn.h:94-98, 624)
  const float lr = t->cfg.lr_scale_rows
                       ? (float)((double)o.lr /
                                 ((double)t->T() * t->cfg.num_envs_global))
                       : o.lr;
  xh::OptStep st{o.kind, lr, o.beta1, o.beta2, 1.0f, 1.0f, o.wd};
  if (o.kind == XH_OPT_ADAM) {  // host float powf, as the reference
    st.c1 = 1 - powf(o.beta1, o.t);
    st.c2 = 1 - powf(o.beta2, o.t);
    o.t += 1;
  }
  return st;
}

int opt_apply(xh_trainer *t, int which, float *params, const float *grad,
              int n) {
  hipStream_t s = t->ctx->stream;
  auto &o = t->opt[which];
  const xh::OptStep st = opt_step(t, which);
  if (o.kind == XH_OPT_SGD)
    return timed(t, "reduce_sgd", [&]() {
      return xh::launch_sgd(params, grad, n, st.lr, st.wd, s);
    });
  return timed(t, "reduce_sgd", [&]() {
    return xh::launch_opt(params, grad, o.m, o.v, n, st, s);
  });
}

// Slab reduce -> (all-reduce) -> optimizer step.  One rank: one fused launch
// (the same sums and updates); more ranks: the all-reduce sits between.
int reduce_and_step(xh_trainer *t, int which, const float *slab, int nslab,
                    int stride, int n, float *grad, float *params,
                    xh::SlabAlias al = xh::SlabAlias{0, 0, 0, 0}) {
  hipStream_t s = t->ctx->stream;
  if (!t->ctx->comm) {
    auto &o = t->opt[which];
    const xh::OptStep st = opt_step(t, which);
    return timed(t, "reduce_sgd", [&]() {
      return xh::launch_slab_reduce_opt(slab, nslab, stride, n, grad, params,
                                        o.m, o.v, st, s, al);
    });
  }
  CHK(timed(t, "reduce_sgd", [&]() {
    return xh::launch_slab_reduce(slab, nslab, stride, n, grad, s, al);
  }));
  CHK(allreduce(t, grad, n));
  return opt_apply(t, which, params, grad, n);
}

int do_pg_rollout(xh_trainer *t);
int do_pg_learn(xh_trainer *t);

// Pending xh_trainer_set_env_state writes -> slot 0 (the rollout's S_0).  The
// host vectors stay alive until the stream has consumed them (synchronised
// before the map is cleared).
// items_ok[0] / bins_wide[0] from the device's slot 0 (after host writes that
// replaced part of it)
int rescan_slot0(xh_trainer *t) {
  const size_t N = t->N(), BD = t->BD(), D = (size_t)t->cfg.dims;
  std::vector<int8_t> b(N * BD), it(N * 4);
  HIPCHK(copy_to_host(b.data(), t->bins, b.size(), t->ctx->stream));
  HIPCHK(copy_to_host(it.data(), t->items, it.size(), t->ctx->stream));
  HIPCHK(hipStreamSynchronize(t->ctx->stream));
  char ok = 1, wide = 0;
  for (size_t e = 0; e < N; ++e) {
    bool is_a = true, is_b = true;
    for (size_t d = 0; d < D; ++d) {
      is_a &= it[e * 4 + d] == t->env.item_a[d];
      is_b &= it[e * 4 + d] == t->env.item_b[d];
    }
    if (!is_a && !is_b) ok = 0;
  }
  for (int8_t v : b) wide |= v < -kBinCapacity;
  t->items_ok[0] = ok;
  t->bins_wide[0] = wide;
  return XH_OK;
}

int apply_env_overrides(xh_trainer *t) {
  if (t->env_override.empty()) return XH_OK;
  hipStream_t s = t->ctx->stream;
  const size_t BD = t->BD(), D = (size_t)t->cfg.dims;
  // runs of consecutive env ids (the map is ordered): one bins copy and one
  // items copy per run from host staging that lives until the single stream
  // synchronisation at the end (pageable sources)
  std::vector<std::vector<int8_t>> stage;
  auto it = t->env_override.begin();
  while (it != t->env_override.end()) {
    const size_t first = (size_t)it->first;
    std::vector<int8_t> rb, ri;
    size_t next = first;
    for (; it != t->env_override.end() && (size_t)it->first == next; ++it, ++next) {
      rb.insert(rb.end(), it->second.begin(), it->second.begin() + BD);
      int8_t item[4] = {0, 0, 0, 0};
      for (size_t d = 0; d < D; ++d) item[d] = it->second[BD + d];
      ri.insert(ri.end(), item, item + 4);
    }
    stage.push_back(std::move(rb));
    stage.push_back(std::move(ri));
    const std::vector<int8_t> &sb = stage[stage.size() - 2], &si = stage.back();
    hipError_t e = hipMemcpyAsync(t->bins + first * BD, sb.data(), sb.size(),
                                  hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
      e = hipMemcpyAsync(t->items + first * 4, si.data(), si.size(),
                         hipMemcpyHostToDevice, s);
    if (e != hipSuccess) {
      (void)hipStreamSynchronize(s);  // nothing in flight reads `stage` after this
      return fail(XH_ERR_HIP, "env override upload: %s", hipGetErrorString(e));
    }
  }
  HIPCHK(hipStreamSynchronize(s));
  bool wide = false;
  for (const auto &kv : t->env_override)
    for (size_t i = 0; i < BD; ++i) wide |= kv.second[i] < -kBinCapacity;
  t->env_override.clear();
  // slot 0's flags: the overrides are whole item-table entries, but envs they
  // did not touch keep what an earlier set_buffer left -> re-read the slot
  // when either flag was off its default
  if (!t->items_ok[0] || t->bins_wide[0]) return rescan_slot0(t);
  if (wide) t->bins_wide[0] = 1;
  return XH_OK;
}

int do_rollout(xh_trainer *t) {
  if (t->cfg.algo == XH_PG) return do_pg_rollout(t);
  hipStream_t s = t->ctx->stream;
  const size_t N = t->N(), T = t->T();
  if (t->items_ok.size() != T + 1) {  // constructed envs in slot 0 only
    t->items_ok.assign(T + 1, 0);
    t->items_ok[0] = 1;
  }
  if (t->bins_wide.size() != T + 1) t->bins_wide.assign(T + 1, 0);
  // replay_buffer::forget(): open trajectories continue from slot T.  With
  // no host overrides pending the rollout launch moves slot T to slot 0
  // itself (the register-stepping kernels as they fetch; copies otherwise)
  int src_slot = -1;
  if (t->need_shift) {
    if (t->env_override.empty()) {
      src_slot = (int)T;
    } else {
      HIPCHK(hipMemcpyAsync(t->bins, t->bins + T * N * t->BD(), N * t->BD(),
                            hipMemcpyDeviceToDevice, s));
      HIPCHK(hipMemcpyAsync(t->items, t->items + T * N * 4, N * 4,
                            hipMemcpyDeviceToDevice, s));
    }
    t->need_shift = false;
    t->items_ok[0] = t->items_ok[T];
    t->bins_wide[0] = t->bins_wide[T];
  }
  CHK(apply_env_overrides(t));  // whole item-table entries only
  xh::RolloutArgs a{};
  a.src_slot = src_slot;
  a.env = t->env;
  a.b = t->batch();
  a.jump_mul = t->jump_mul;
  a.params = t->pp;
  a.forced = t->use_forced ? t->forced : nullptr;
  a.qold_out = t->qold;  // KL-PPO only (nullptr otherwise)
  // all T slots in one call (one launch where the kernel steps in registers);
  // only slot 0 can hold a wide state
  a.t = 0;
  a.nsteps = (int)T;
  // the f32 kernels for a slot 0 the split rollouts cannot take: a bin below
  // -capacity, or an item outside the item table (set_buffer; the split
  // rollouts fold the item into per-entry biases)
  a.wide = t->bins_wide[0] || !t->items_ok[0];
  // diagnostics only (tests, health checks): off in the product path
  a.logits_out = t->cfg.record_last_step ? t->logits : nullptr;
  a.probs_out = t->cfg.record_last_step ? t->probs : nullptr;
  // cleared as well: a rollout without recording leaves no current logits
  t->last_step_recorded = t->cfg.record_last_step != 0;
  CHK(timed(t, "rollout_step", [&]() {
    return xh::launch_rollout_step(a, t->cfg.policy_h1, t->cfg.policy_h2,
                                   t->rgrid, s, &t->last_rollout);
  }));
  for (size_t step = 0; step < T; ++step) {
    t->items_ok[step + 1] = 1;  // items drawn from the table (get_item)
    t->bins_wide[step + 1] = 0;  // apply + reset on game over: bins >= 0
  }
  t->rolled = true;
  return XH_OK;
}

// The value net (full_layer Fin -> V1 -> V2 -> 1, ppo_training.cc:19-26) as a
// Dense MLP over `rows` rows: S_0..S_T (row = slot * N + env), then the
// terminal views E_t of transition row - N(T+1).  `out` receives V.
// layer 0 of the value net on the reduced observation (dense_kernels.hip)
#ifndef XH_VALUE_REDUCED
#define XH_VALUE_REDUCED 1
#endif
xh::MlpArgs value_mlp(xh_trainer *t, int rows, float *out) {
  xh::MlpArgs m{};
  m.env = t->env;
  m.bins = t->bins;
  m.items = t->items;
  m.N = (int)t->N();
  m.action = t->action;
  m.term_from = (int)((t->T() + 1) * t->N());
  m.max_rows = rows;
  m.nlayers = 3;
  m.w[0] = t->vl.Fin;
  m.w[1] = t->vl.V1;
  m.w[2] = t->vl.V2;
  m.w[3] = 1;
  m.params = t->vp;
  m.act[0] = t->vact[0];
  m.act[1] = t->vact[1];
  m.act[2] = out;
  m.grad[0] = t->vgr[0];
  m.grad[1] = t->vgr[1];
  m.grad[2] = t->row_g;
  // worth its extra launch from a 256-wide input on (config 2's 64-wide
  // layer 0 measured 1% slower with it)
  m.w0red = XH_VALUE_REDUCED && t->vl.Fin >= 256 ? t->vw0red : nullptr;
  m.w0frag = t->vw0frag;
  return m;
}

int do_learn(xh_trainer *t) {
  if (t->cfg.algo == XH_PG) return do_pg_learn(t);
  // the train kernels fold the item into per-table-entry biases: every slot
  // they read must hold item-table entries only
  for (size_t sl = 0; sl < t->T(); ++sl)
    if (sl >= t->items_ok.size() || !t->items_ok[sl])
      return fail(XH_ERR_STATE,
                  "learn: slot %zu of the batch holds an item that is not an "
                  "item-table entry (set by xh_trainer_set_buffer, or no "
                  "rollout yet)", sl);
  hipStream_t s = t->ctx->stream;
  const xh_config &c = t->cfg;
  xh::ValueArgs va = t->vargs();
  const int NS = (int)((t->T() + 1) * t->N()), NT = (int)(t->T() * t->N());
  // the transitions that ended an episode (env-major, t ascending); their
  // terminal views are the only end rows whose V the targets read
  xh::EndListArgs ea{t->done, (int)t->N(), (int)t->T(), t->end_list,
                     t->n_end, t->n_open, t->vrows, NS};
  CHK(timed(t, "value", [&]() {
    return xh::launch_end_list(ea, t->end_scratch, s);
  }));
  // update_value_model (policy_gradient.h:196-218): V over S_0..S_T and the
  // terminal views E_t of the ended transitions in one batch (NS + n_end
  // rows, a device count), TD targets and dL/dV = V - target on the
  // transition rows (end rows have zero gradient), backward, one step
  // (the terminal views' values also land on their transition rows, v_term)
  xh::MlpArgs vm = value_mlp(t, NS + NT, t->v_state0);
  vm.act_rows = NT;  // the backward reads the transition rows' activations
  vm.rows = t->vrows;
  vm.term_list = t->end_list;
  vm.v_term = t->v_term;
  vm.term_n = t->n_end;
  const bool vnet = std::strcmp(xh::value_kernel_name(vm), "vnet_bf16") == 0;
  vm.w0frag_ready = vnet && t->vfrag_ready;
  CHK(timed(t, "value", [&]() { return xh::mlp_forward(vm, s); }));
  t->vfrag_ready = vnet;
  vm.rows = nullptr;
  vm.term_list = nullptr;
  vm.v_term = nullptr;
  va.v_state = t->v_state0;
  vm.max_rows = NT;
  CHK(timed(t, "value", [&]() {
    return xh::value_backward(vm, va, c.gamma, t->targets, t->vslab,
                              t->vslab_stride, t->vslab_n, s);
  }));
  // the reduced layer 0 writes bin 0's item columns only (EpSlabRed)
  const xh::SlabAlias al =
      xh::value_reduced_slab(vm) ? xh::SlabAlias{t->cfg.value_h1, t->vl.Fin, t->cfg.bins,
                               t->cfg.dims}
               : xh::SlabAlias{0, 0, 0, 0};
  t->vfrag_ready = false;  // the step below writes vp
  CHK(reduce_and_step(t, XH_VALUE, t->vslab, t->vslab_n, t->vslab_stride,
                      t->nv, t->vgrad, t->vp, al));
  // calculate_advantage (policy_gradient.h:220-281) on post-update values;
  // GAE zeroes V(terminal), the targets above used V(E_t)
  vm.max_rows = NS;
  vm.act[2] = t->v_state;
  vm.act_rows = -1;  // no backward reads these
  vm.w0frag_ready = 0;  // (new parameters)
  CHK(timed(t, "value", [&]() { return xh::mlp_forward(vm, s); }));
  t->vfrag_ready = vnet;
  va.v_state = t->v_state;
  va.row_g = nullptr;
  CHK(timed(t, "value", [&]() {
    return xh::launch_gae(va, c.gamma, c.lambda, t->adv,
                          c.adv_normalize ? t->adv_part : nullptr, s);
  }));
  if (c.adv_normalize) {  // opt-in: job-wide mean / std of the advantages
    CHK(timed(t, "value", [&]() {
      return xh::launch_adv_stats(t->adv_part, xh::gae_grid((int)t->N()),
                                  t->adv_stats, s);
    }));
    CHK(allreduce_d(t, t->adv_stats, 2));
    CHK(timed(t, "value", [&]() {
      return xh::launch_adv_normalize(t->adv, (long)(t->T() * t->N()),
                                      t->adv_stats,
                                      (double)t->T() * c.num_envs_global, s);
    }));
  }
  // optimize_action: k policy steps (policy_gradient.h:297-307)
  xh::PolicyTrainArgs pa{};
  pa.env = t->env;
  pa.b = t->batch();
  pa.algo = c.algo;
  pa.clip_eps = c.clip_eps;
  pa.params = t->pp;
  pa.adv = t->adv;
  pa.slab = t->pslab;
  pa.slab_stride = t->pslab_stride;
  for (size_t sl = 0; sl < t->T() && sl < t->bins_wide.size(); ++sl)
    pa.wide |= t->bins_wide[sl];
  {
    // XH_ABLATE drops whole phases (wrong results by design): honoured by the
    // diagnostic build only, refused by the product library
    const char *ab = std::getenv("XH_ABLATE");
    pa.ablate = ab ? std::atoi(ab) : 0;
    if (pa.ablate && !xh::diag_build())
      return fail(XH_ERR_INVALID, "XH_ABLATE=%s is set but this is the "
                  "product library (phase ablation exists only in `make "
                  "diag`)", ab);
  }
  // XH_PHASE_TRACE (diagnostic build): phase stamps of the first epoch's
  // train launch, summarised on stderr
  static long long *trace_buf = nullptr;
  const size_t trace_n = (size_t)xh::kTraceBlocks * xh::kTraceGroups * 8 *
                         xh::kTraceSlots;
  if (xh::diag_build() && std::getenv("XH_PHASE_TRACE")) {
    // + the kernel span words: earliest start (init all ones), latest end
    // and per-workgroup start / end words for 1024 workgroups
    if (!trace_buf && hipMalloc(&trace_buf, trace_n * 8 + 16 + 4096 * 8) != hipSuccess)
      return fail(XH_ERR_HIP, "trace buffer");
    if (hipMemsetAsync(trace_buf, 0, trace_n * 8 + 16 + 4096 * 8, s) != hipSuccess ||
        hipMemsetAsync(trace_buf + trace_n, 0xFF, 8, s) != hipSuccess)
      return fail(XH_ERR_HIP, "trace buffer");
    pa.trace = trace_buf;
  }
  const bool kl = c.algo == XH_KLPPO;
  if (kl) {
    pa.qold = t->qold;
    pa.beta = t->beta;
    pa.end_list = t->end_list;
    pa.n_end = t->n_end;
    pa.kl_part = t->kl_part;
    // end_list / n_end / n_open: built before the value step above
  }
  for (int e = 0; e < c.epochs; ++e) {
    float *g = t->pgrads + (size_t)e * t->np;
    CHK(timed(t, "policy_train", [&]() {
      return xh::launch_policy_train(pa, c.policy_h1, c.policy_h2, t->pslab_n,
                                     s, &t->last_train);
    }));
    if (pa.trace) {
      std::vector<long long> tr(trace_n + 2 + 4096);
      if (hipMemcpyAsync(tr.data(), pa.trace, trace_n * 8 + 16 + 4096 * 8,
                         hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return fail(XH_ERR_HIP, "trace read-back");
      // per phase: mean cycles over waves and groups 1.. (group 0 warms up);
      // "group" = stamp 0 of the next group minus stamp 0 of this one
      double sum[xh::kTraceSlots + 1] = {0};
      long n = 0;
      for (int b = 0; b < xh::kTraceBlocks; ++b)
        for (int gi = 1; gi + 1 < xh::kTraceGroups; ++gi)
          for (int w = 0; w < 8; ++w) {
            const long long *p =
                &tr[((b * xh::kTraceGroups + gi) * 8 + w) * xh::kTraceSlots];
            const long long *pn = p + 8 * xh::kTraceSlots;
            if (!p[0] || !pn[0]) continue;
            for (int k = 1; k < xh::kTraceSlots; ++k) sum[k] += p[k] - p[k - 1];
            sum[xh::kTraceSlots] += pn[0] - p[xh::kTraceSlots - 1];
            sum[0] += pn[0] - p[0];
            ++n;
          }
      std::fprintf(stderr, "phase trace (%ld wave-groups, cycles): group %.0f |"
                   " fwd %.0f bar1 %.0f softmax %.0f layer3 %.0f bar2 %.0f"
                   " dH1 %.0f dW2 %.0f end+bar3 %.0f\n", n,
                   sum[0] / n, sum[1] / n, sum[2] / n, sum[3] / n, sum[4] / n,
                   sum[5] / n, sum[6] / n, sum[7] / n, sum[8] / n);
      if (std::getenv("XH_PHASE_TRACE_WAVES")) {  // the same means per wave
        for (int w = 0; w < 8; ++w) {
          double sw[xh::kTraceSlots + 1] = {0};
          long nw = 0;
          for (int b = 0; b < xh::kTraceBlocks; ++b)
            for (int gi = 1; gi + 1 < xh::kTraceGroups; ++gi) {
              const long long *p =
                  &tr[((b * xh::kTraceGroups + gi) * 8 + w) * xh::kTraceSlots];
              const long long *pn = p + 8 * xh::kTraceSlots;
              if (!p[0] || !pn[0]) continue;
              for (int k = 1; k < xh::kTraceSlots; ++k) sw[k] += p[k] - p[k - 1];
              sw[xh::kTraceSlots] += pn[0] - p[xh::kTraceSlots - 1];
              sw[0] += pn[0] - p[0];
              ++nw;
            }
          if (!nw) continue;
          std::fprintf(stderr, "  wave %d:", w);
          for (int k = 0; k <= xh::kTraceSlots; ++k)
            std::fprintf(stderr, " %.0f", sw[k] / nw);
          std::fprintf(stderr, "\n");
        }
      }
      {  // kernel-level stamps (4-wave kernel: the last trace group)
        double k1 = 0, k2 = 0, k3 = 0;
        long kn = 0;
        for (int b = 0; b < xh::kTraceBlocks; ++b)
          for (int w = 0; w < 8; ++w) {
            const long long *p =
                &tr[((b * xh::kTraceGroups + xh::kTraceGroups - 1) * 8 + w) *
                    xh::kTraceSlots];
            if (!p[0] || !p[3]) continue;
            k1 += p[1] - p[0];
            k2 += p[2] - p[1];
            k3 += p[3] - p[2];
            ++kn;
          }
        if (kn)
          std::fprintf(stderr, "kernel stamps (%ld waves, cycles): stage %.0f "
                       "| groups %.0f | epilogue %.0f\n", kn, k1 / kn,
                       k2 / kn, k3 / kn);
        int wc = 0;
        (void)hipDeviceGetAttribute(&wc, hipDeviceAttributeWallClockRate,
                                    t->ctx->device);
        if (tr[trace_n + 1] && wc > 0)
          std::fprintf(stderr, "workgroup span: %.1f us (wall clock %d kHz)\n",
                       (double)(tr[trace_n + 1] - tr[trace_n]) * 1e3 / wc, wc);
        if (tr[trace_n + 1] && wc > 0) {  // per-workgroup phase spread
          // [b][start, staged, loop done, end] on the wall clock
          std::vector<double> ph[4];
          for (int b = 0; b < 512; ++b) {
            const long long *w4 = &tr[trace_n + 2 + 4 * b];
            if (!w4[0] || !w4[3]) continue;
            ph[0].push_back((w4[1] - w4[0]) * 1e3 / wc);
            ph[1].push_back((w4[2] - w4[1]) * 1e3 / wc);
            ph[2].push_back((w4[3] - w4[2]) * 1e3 / wc);
            ph[3].push_back((w4[3] - w4[0]) * 1e3 / wc);
          }
          auto q = [](std::vector<double> v, double f) {
            std::sort(v.begin(), v.end());
            return v.empty() ? 0.0 : v[(size_t)(f * (v.size() - 1))];
          };
          const char *nm[4] = {"stage", "groups", "epilogue", "total"};
          std::fprintf(stderr, "workgroups %zu (us, min/p10/med/p90/max):",
                       ph[3].size());
          for (int k = 0; k < 4; ++k)
            std::fprintf(stderr, " %s %.1f/%.1f/%.1f/%.1f/%.1f", nm[k],
                         q(ph[k], 0), q(ph[k], .1), q(ph[k], .5), q(ph[k], .9),
                         q(ph[k], 1));
          std::fprintf(stderr, "\n");
          // placement: workgroups per CU (xcc, se, sh, cu from HW_ID /
          // XCC_ID) and the duration of each CU's pair
          std::map<long, std::vector<double>> cu;
          std::map<long, std::vector<int>> cub;
          for (int b = 0; b < 512; ++b) {
            const long long *w4 = &tr[trace_n + 2 + 4 * b];
            if (!w4[0] || !w4[3]) continue;
            const unsigned hw = (unsigned)tr[trace_n + 2 + 2048 + 2 * b];
            const unsigned xc = (unsigned)tr[trace_n + 2 + 2048 + 2 * b + 1];
            const long key = ((long)(xc & 15) << 12) | (((hw >> 13) & 7) << 8) |
                             (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
            cu[key].push_back((w4[3] - w4[0]) * 1e3 / wc);
            cub[key].push_back(b);
          }
          std::map<size_t, int> per;
          std::vector<double> pmax, pdiff;
          for (auto &kv : cu) {
            per[kv.second.size()]++;
            if (kv.second.size() == 2) {
              pmax.push_back(std::max(kv.second[0], kv.second[1]));
              pdiff.push_back(std::fabs(kv.second[0] - kv.second[1]));
            }
          }
          std::fprintf(stderr, "placement: %zu CUs;", cu.size());
          for (auto &kv : per) std::fprintf(stderr, " %d CUs with %zu wg;", kv.second, kv.first);
          std::fprintf(stderr, " pair max dur p10/med/p90 %.1f/%.1f/%.1f, pair |diff| med/p90 %.1f/%.1f\n",
                       q(pmax, .1), q(pmax, .5), q(pmax, .9), q(pdiff, .5), q(pdiff, .9));
          int shown = 0;
          for (auto &kv : cub) {
            if (shown++ >= 6) break;
            std::fprintf(stderr, "  cu %05lx: blocks", kv.first);
            for (size_t i = 0; i < kv.second.size(); ++i)
              std::fprintf(stderr, " %d(%.1fus)", kv.second[i], cu[kv.first][i]);
            std::fprintf(stderr, "\n");
          }
        }
      }
      pa.trace = nullptr;  // first epoch only
    }
    // the optimizer step does not read beta: it may precede the KL update
    CHK(reduce_and_step(t, XH_POLICY, t->pslab, t->pslab_n, t->pslab_stride,
                        t->np, g, t->pp));
    if (kl) {  // mean KL over the job's rows -> beta for the next epoch
      CHK(timed(t, "kl", [&]() {
        return xh::launch_kl_reduce(t->kl_part, t->pslab_n, t->n_end,
                                    t->n_open, (double)t->T() * t->N(),
                                    t->kl_sum, s);
      }));
      CHK(allreduce_d(t, t->kl_sum, 2));
      CHK(timed(t, "kl", [&]() {
        return xh::launch_kl_beta_update(t->kl_sum, t->beta, c.kl_target,
                                         t->kl_log + 3 * e, s);
      }));
    }
  }
  t->need_shift = true;
  t->rolled = false;
  return XH_OK;
}

// ------------------------------------------------------------ REINFORCE ----
// policy_gradient_learner (policy_gradient.h:88-147) with a full-MLP
// softmax-xent policy (pg_training.cc:10-20), each env playing cfg.steps
// whole episodes per iteration.

// Upper bound of an episode's length: every non-final step puts an item into
// a bin, and a bin takes at most min_d floor(8 / smallest item extent in d)
// items before some extent would go negative.
int pg_episode_bound(const xh::EnvDesc &E) {
  int per_bin = 8;  // capacity per dim (bin_packing.h:48)
  for (int d = 0; d < E.D; ++d) {
    const int m = std::min(E.item_a[d], E.item_b[d]);
    per_bin = std::min(per_bin, 8 / m);
  }
  return E.B * per_bin + 1;
}

xh::MlpArgs pg_mlp(const xh_trainer *t, bool learn, int slot) {
  xh::MlpArgs m{};
  m.env = t->env;
  m.bins = t->bins;
  m.items = t->items;
  m.N = (int)t->N();
  m.nlayers = t->pg.nlayers;
  for (int i = 0; i < 4; ++i) m.w[i] = t->pg.w[i];
  m.params = t->pp;
  for (int i = 0; i < 3; ++i) {
    m.act[i] = t->pg.act[i];
    m.grad[i] = t->pg.grad[i];
  }
  if (learn) {
    m.list = t->pg.list;
    m.rows = t->pg.nrows;
    m.max_rows = (int)(t->T() * t->N());
  } else {
    m.slot = slot;
    m.max_rows = (int)t->N();
  }
  return m;
}

int create_pg(xh_ctx *ctx, const xh_config &c, xh_trainer **out) {
  if (c.adv_normalize || c.lr_scale_rows)
    return fail(XH_ERR_INVALID, "REINFORCE: adv_normalize / lr_scale_rows are "
                "actor-critic / PPO options (REINFORCE has its own mean-return "
                "baseline, policy_gradient.h:125-147)");
  if (c.bins < 2 || c.bins > 128 || c.dims < 1 || c.dims > 3)
    return fail(XH_ERR_INVALID, "REINFORCE: bins %d (2..128), dims %d (1..3)",
                c.bins, c.dims);
  if (c.policy_h1 < 1 || c.policy_h2 < 0 || c.policy_h1 > 1024 ||
      c.policy_h2 > 1024)
    return fail(XH_ERR_INVALID, "REINFORCE: widths [%d,%d]", c.policy_h1,
                c.policy_h2);
  if (c.steps < 1 || c.steps > 64)
    return fail(XH_ERR_INVALID, "REINFORCE: episodes per env %d not in [1,64]",
                c.steps);
  if (c.num_envs < 1 || c.num_envs_global < c.num_envs || c.env_offset < 0 ||
      c.env_offset + c.num_envs > c.num_envs_global)
    return fail(XH_ERR_INVALID, "env partition offset %d + %d > global %d",
                c.env_offset, c.num_envs, c.num_envs_global);
  HIPCHK(hipSetDevice(ctx->device));
  auto *t = new xh_trainer;
  t->ctx = ctx;
  t->cfg = c;
  t->cfg.epochs = 1;
  t->cfg.rng_state = c.rng_state % 2147483647u;
  if (t->cfg.rng_state == 0) t->cfg.rng_state = 1;
  t->env = make_env(c.bins, c.dims);
  t->Tb = c.steps * pg_episode_bound(t->env);
  auto &pg = t->pg;
  pg.w[0] = c.bins * 2 * c.dims;
  pg.w[1] = c.policy_h1;
  pg.nlayers = 2;
  if (c.policy_h2 > 0) {
    pg.w[2] = c.policy_h2;
    pg.nlayers = 3;
  }
  pg.w[pg.nlayers] = c.bins;
  t->np = 0;
  for (int l = 0; l < pg.nlayers; ++l) t->np += pg.w[l + 1] * pg.w[l] + pg.w[l + 1];
  t->nv = 0;
  const size_t N = t->N(), T = t->T(), R = T * N;
  int st = XH_OK;
  auto A = [&](auto **p, size_t bytes) {
    if (st == XH_OK) st = dalloc(t, p, bytes);
  };
  A(&t->bins, (T + 1) * N * t->BD());
  A(&t->items, (T + 1) * N * 4);
  A(&t->action, T * N * 4);
  A(&t->forced, T * N * 4);
  A(&t->pold, T * N * 4);
  A(&t->done, T * N);
  A(&t->rng, N * 4);
  A(&t->pp, (size_t)t->np * 4);
  A(&t->adv, T * N * 4);
  for (int l = 0; l < pg.nlayers; ++l) {
    A(&pg.act[l], R * pg.w[l + 1] * 4);
    A(&pg.grad[l], R * pg.w[l + 1] * 4);
  }
  A(&pg.ep_done, N * 4);
  A(&pg.len, N * 4);
  A(&pg.active, 4);
  A(&pg.row_off, N * 4);
  A(&pg.list, R * 4);
  A(&pg.nrows, 4);
  A(&pg.rtg, R * 4);
  A(&pg.ep_part, N * 8);
  A(&pg.stats, 2 * 8);
  t->pslab_n = 64;
  t->pslab_stride = (t->np + 63) & ~63;
  A(&t->pslab, (size_t)t->pslab_n * t->pslab_stride * 4);
  A(&t->pgrads, (size_t)t->np * 4);
  A(&t->logits, N * c.bins * 4);
  A(&t->probs, N * c.bins * 4);
  if (st == XH_OK && hipHostMalloc((void **)&pg.host_active, 4) != hipSuccess)
    st = fail(XH_ERR_HIP, "hipHostMalloc");
  t->opt[XH_POLICY].lr = c.lr_policy;
  t->opt[XH_POLICY].wd = c.wd_policy;
  hipError_t e = hipSuccess;
  if (st == XH_OK) {
    e = xh::launch_pg_env_init(t->env, t->batch(), t->cfg.rng_state,
                               c.env_offset, kEvalStride, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) st = fail(XH_ERR_HIP, "env init: %s", hipGetErrorString(e));
  }
  t->counted = true;
  ++ctx->trainers;
  if (st != XH_OK) {
    std::string keep = g_err;
    xh_trainer_destroy(t);
    g_err = keep;
    return st;
  }
  *out = t;
  return XH_OK;
}

// agent::play_one_episode x cfg.steps for every env (rl.h:325-354): one
// forward + one step kernel per env step, until every env has finished its
// episodes (checked every 8 steps through a pinned flag).
int do_pg_rollout(xh_trainer *t) {
  hipStream_t s = t->ctx->stream;
  const size_t N = t->N();
  auto &pg = t->pg;
  if (t->need_shift) {  // the envs' current states -> slot 0
    HIPCHK(hipMemcpyAsync(t->bins, t->bins + (size_t)pg.slot_end * N * t->BD(),
                          N * t->BD(), hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(t->items, t->items + (size_t)pg.slot_end * N * 4,
                          N * 4, hipMemcpyDeviceToDevice, s));
    t->need_shift = false;
  }
  CHK(timed(t, "rollout_step", [&]() {
    return xh::launch_pg_begin((int)N, pg.active, pg.ep_done, pg.len, s);
  }));
  xh::PgStepArgs a{};
  a.env = t->env;
  a.b = t->batch();
  a.episodes = t->cfg.steps;
  a.logits = pg.act[pg.nlayers - 1];
  a.forced = t->use_forced ? t->forced : nullptr;
  a.ep_done = pg.ep_done;
  a.len = pg.len;
  a.active = pg.active;
  int steps = 0;
  for (int step = 0; step < t->Tb; ++step) {
    xh::MlpArgs m = pg_mlp(t, false, step);
    CHK(timed(t, "rollout_step", [&]() { return xh::mlp_forward(m, s); }));
    a.t = step;
    CHK(timed(t, "rollout_step", [&]() { return xh::launch_pg_step(a, s); }));
    steps = step + 1;
    if (steps % 8 == 0 || steps == t->Tb) {
      HIPCHK(hipMemcpyAsync(pg.host_active, pg.active, 4,
                            hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      if (*pg.host_active == 0) break;
    }
  }
  if (*pg.host_active != 0)
    return fail(XH_ERR_STATE, "REINFORCE rollout: %d envs still playing after "
                "the step bound %d", *pg.host_active, t->Tb);
  pg.slot_end = steps;
  t->rolled = true;
  return XH_OK;
}

// policy_gradient_learner::learn (policy_gradient.h:95-123): rows = every
// transition in replay-buffer order, advantages = reversed rewards-to-go minus
// the mean trajectory return, one optimizer step on policy_loss.
int do_pg_learn(xh_trainer *t) {
  hipStream_t s = t->ctx->stream;
  auto &pg = t->pg;
  xh::PgLearnArgs L{};
  L.N = (int)t->N();
  L.B = t->cfg.bins;
  L.episodes = t->cfg.steps;
  L.gamma = t->cfg.gamma;
  L.len = pg.len;
  L.row_off = pg.row_off;
  L.list = pg.list;
  L.nrows = pg.nrows;
  L.done = t->done;
  L.action = t->action;
  L.rtg = pg.rtg;
  L.ep_part = pg.ep_part;
  L.stats = pg.stats;
  L.logits = pg.act[pg.nlayers - 1];
  L.dlogits = pg.grad[pg.nlayers - 1];
  L.adv_grid = t->adv;
  CHK(timed(t, "policy_train", [&]() { return xh::launch_pg_rows(L, s); }));
  CHK(timed(t, "policy_train", [&]() { return xh::launch_pg_adv(L, s); }));
  CHK(allreduce_d(t, pg.stats, 2));  // baseline over the job's trajectories
  const xh::MlpArgs m = pg_mlp(t, true, 0);
  CHK(timed(t, "policy_train", [&]() { return xh::mlp_forward(m, s); }));
  CHK(timed(t, "policy_train", [&]() {
    return xh::launch_pg_loss(L, m.max_rows, s);
  }));
  CHK(timed(t, "policy_train", [&]() {
    return xh::mlp_backward(m, t->pslab, t->pslab_stride, t->pslab_n, s);
  }));
  CHK(reduce_and_step(t, XH_POLICY, t->pslab, t->pslab_n, t->pslab_stride,
                      t->np, t->pgrads, t->pp));
  t->need_shift = true;
  t->rolled = false;
  return XH_OK;
}

}  // namespace

// ================================================================= C ABI ==
namespace {
constexpr double kBf16DensePeakTflops = 2500.0;  // MI355X_MICROARCH.md
constexpr double kF32MfmaPeakTflops = 157.3;

std::string kernel_json(const xh::KernelInfo &k) {
  char buf[320];
  if (!k.name) return "{\"kernel\": null}";
  // MFMA products per f32 product of the kernel's arithmetic (equal FLOPs
  // per GEMM): bf16 / f16 run at the same dense rate (MI355X_MICROARCH.md)
  const double prod = k.math == xh::kMathSplitTrain      ? 4.0
                      : k.math == xh::kMathSplitRollout  ? 3.0
                      : k.math == xh::kMathSplitTrainF16 ? 8.0 / 3.0
                                                         : 0.0;
  if (k.math == xh::kMathSplitTrainF16 || k.math == xh::kMathSplitRollout)
    std::snprintf(buf, sizeof buf,
                  "{\"kernel\": \"%s\", \"math\": \"%s\", "
                  "\"bf16_products_per_f32_product\": null, "
                  "\"products_per_f32_product\": %.6g, \"peak_tflops\": %.6g}",
                  k.name,
                  k.math == xh::kMathSplitRollout ? "f16_pair" : "f16_pair_bf16_split",
                  prod, kBf16DensePeakTflops / prod);
  else if (prod > 0)
    std::snprintf(buf, sizeof buf,
                  "{\"kernel\": \"%s\", \"math\": \"bf16_split\", "
                  "\"bf16_products_per_f32_product\": %d, "
                  "\"products_per_f32_product\": %d, \"peak_tflops\": %.6g}",
                  k.name, (int)prod, (int)prod, kBf16DensePeakTflops / prod);
  else
    std::snprintf(buf, sizeof buf,
                  "{\"kernel\": \"%s\", \"math\": \"f32_mfma\", "
                  "\"bf16_products_per_f32_product\": null, "
                  "\"products_per_f32_product\": null, \"peak_tflops\": %.6g}",
                  k.name, kF32MfmaPeakTflops);
  return buf;
}

std::string env_json(const char *name) {
  const char *v = std::getenv(name);
  if (!v) return std::string("\"") + name + "\": null";
  std::string out = std::string("\"") + name + "\": \"";
  for (const char *p = v; *p; ++p)
    if (*p != '"' && *p != '\\' && (unsigned char)*p >= 32) out += *p;
  return out + "\"";
}
}  // namespace

extern "C" {

const char *xh_last_error(void) { return g_err.c_str(); }
const char *xh_version(void) { return "xylo-hip 0.2 (gfx950)"; }

int xh_device_count(int *out) {
  return guard([&]() -> int {
    if (!out) return fail(XH_ERR_INVALID, "null out");
    *out = 0;
    HIPCHK(hipGetDeviceCount(out));
    return XH_OK;
  });
}

// Which HIP / RCCL shared objects this process actually bound (a process that
// loaded another copy under the same soname first, e.g. a framework's bundled
// runtime, makes the library bind that one).
int xh_runtime_info(char *buf, size_t cap) {
  return guard([&]() -> int {
    if (!buf || cap == 0) return fail(XH_ERR_INVALID, "null buffer");
    Dl_info hi{}, ri{};
    const char *hp = dladdr(reinterpret_cast<void *>(&hipRuntimeGetVersion), &hi) &&
                             hi.dli_fname ? hi.dli_fname : "?";
    const char *rp = dladdr(reinterpret_cast<void *>(&ncclAllReduce), &ri) &&
                             ri.dli_fname ? ri.dli_fname : "?";
    int hv = 0, rv = 0;
    (void)hipRuntimeGetVersion(&hv);
    (void)ncclGetVersion(&rv);
    const int n = std::snprintf(buf, cap,
                                "{\"libamdhip64\": \"%s\", \"hip_runtime\": %d, "
                                "\"librccl\": \"%s\", \"rccl_version\": %d}",
                                hp, hv, rp, rv);
    if (n < 0 || (size_t)n >= cap)
      return fail(XH_ERR_INVALID, "runtime info needs %d bytes", n + 1);
    return XH_OK;
  });
}

size_t xh_struct_size(const char *name) {
  if (!name) return 0;
  if (!std::strcmp(name, "xh_config")) return sizeof(xh_config);
  if (!std::strcmp(name, "xh_eval")) return sizeof(xh_eval);
  if (!std::strcmp(name, "xh_layer")) return sizeof(xh_layer);
  return 0;
}

int xh_comm_unique_id(void *out128) {
  return guard([&]() -> int {
    if (!out128) return fail(XH_ERR_INVALID, "null out");
    ncclUniqueId id;
    RCCLCHK(ncclGetUniqueId(&id));
    static_assert(sizeof(id) == 128, "nccl unique id size");
    std::memcpy(out128, &id, sizeof id);
    return XH_OK;
  });
}

int xh_ctx_create(int device, int rank, int world, const void *uid128,
                  xh_ctx **out) {
  return guard([&]() -> int {
    if (!out) return fail(XH_ERR_INVALID, "null out");
    if (world < 1 || rank < 0 || rank >= world)
      return fail(XH_ERR_INVALID, "bad rank %d / world %d", rank, world);
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev)
      return fail(XH_ERR_INVALID, "device %d of %d", device, ndev);
    HIPCHK(hipSetDevice(device));
    auto *c = new xh_ctx;
    c->device = device;
    c->rank = rank;
    c->world = world;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete c;
      return fail(XH_ERR_HIP, "stream: %s", hipGetErrorString(e));
    }
    // a communicator for world > 1, and for world == 1 when a unique id is
    // given (a one-rank RCCL comm: the multi-GPU code path on one device)
    if (world > 1 || uid128) {
      if (!uid128) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return fail(XH_ERR_INVALID, "world > 1 needs the RCCL unique id");
      }
      ncclUniqueId id;
      std::memcpy(&id, uid128, sizeof id);
      ncclResult_t r = ncclCommInitRank(&c->comm, world, id, rank);
      if (r != ncclSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return fail(XH_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
      }
    }
    *out = c;
    return XH_OK;
  });
}

// A context outlives its trainers: destroying it with live trainers defers
// the release to the last xh_trainer_destroy.
int xh_ctx_destroy(xh_ctx *c) {
  return guard([&]() -> int {
    if (!c) return XH_OK;
    if (c->trainers > 0) {
      c->closing = true;
      return XH_OK;
    }
    ctx_free(c);
    return XH_OK;
  });
}

int xh_ctx_synchronize(xh_ctx *c) {
  return guard([&]() -> int {
    if (!c) return fail(XH_ERR_INVALID, "null ctx");
    HIPCHK(hipStreamSynchronize(c->stream));
    return XH_OK;
  });
}

int xh_ctx_allreduce_host(xh_ctx *c, float *data, size_t n) {
  return guard([&]() -> int {
    if (!c || (!data && n)) return fail(XH_ERR_INVALID, "null arg");
    if (!c->comm || n == 0) return XH_OK;
    float *d = nullptr;
    HIPCHK(hipMalloc(&d, n * sizeof(float)));
    // the device buffer is freed on every path (the stream drained first)
    int st = copy_ok(copy_to_device(d, data, n * sizeof(float), c->stream));
    if (st == XH_OK) {
      const ncclResult_t r =
          ncclAllReduce(d, d, n, ncclFloat32, ncclSum, c->comm, c->stream);
      if (r != ncclSuccess)
        st = fail(XH_ERR_RCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
    }
    if (st == XH_OK)
      st = copy_ok(copy_to_host(data, d, n * sizeof(float), c->stream));
    const hipError_t se = hipStreamSynchronize(c->stream);
    if (st == XH_OK && se != hipSuccess)
      st = fail(XH_ERR_HIP, "synchronize: %s", hipGetErrorString(se));
    (void)hipFree(d);
    return st;
  });
}

void xh_config_default(xh_config *c, int algo, int bins, int dims, int num_envs,
                       int steps) {
  std::memset(c, 0, sizeof *c);
  c->algo = algo;
  c->num_envs = c->num_envs_global = num_envs;
  c->env_offset = 0;
  c->bins = bins;
  c->dims = dims;
  c->steps = steps;
  c->epochs = algo == XH_AC ? 1 : 4;
  c->policy_h1 = 128;
  c->policy_h2 = algo == XH_AC ? 32 : 64;
  if (algo == XH_AC) c->policy_h1 = 64;
  c->value_h1 = 64;
  c->value_h2 = 32;
  // ppo_training.cc:17,26 / ac_training.cc:17,26
  c->lr_policy = algo == XH_AC ? 1e-5f : 1e-4f;
  c->lr_value = algo == XH_AC ? 1e-4f : 1e-5f;
  if (algo == XH_KLPPO) c->wd_policy = 1e-5f;  // ppo2_training.cc:20
  if (algo == XH_PG) {  // pg_training.cc:10-20: full 4B->256->128->B, 1e-4
    c->policy_h1 = 256;
    c->policy_h2 = 128;
    c->epochs = 1;
    c->lr_policy = 1e-4f;
    c->lr_value = 0.0f;
  }
  c->gamma = 0.99f;
  c->lambda = 0.95f;
  c->clip_eps = 0.2f;
  c->rng_state = 1;
  c->kl_beta = 1.0f;
  c->kl_target = 1e-9f;
}

int xh_trainer_create(xh_ctx *ctx, const xh_config *cfg, xh_trainer **out) {
  return guard([&]() -> int {
    if (!ctx || !cfg || !out) return fail(XH_ERR_INVALID, "null arg");
    const xh_config &c = *cfg;
    if (c.algo == XH_PG) return create_pg(ctx, c, out);
    if (c.algo != XH_PPO && c.algo != XH_AC && c.algo != XH_KLPPO)
      return fail(XH_ERR_INVALID, "algo %d", c.algo);
    // KL-PPO beyond 64 bins: the 128-bin 3-D [128,128] shape's split train
    // kernel only (the f32 KL kernel is written for <= 64 bins)
    if (c.algo == XH_KLPPO && c.bins > 64 &&
        !(c.bins == 128 && c.dims == 3 && c.policy_h1 == 128 && c.policy_h2 == 128))
      return fail(XH_ERR_INVALID,
                  "KL-PPO: bins %d > 64 supported at 128 bins, 3-D, [128,128] only",
                  c.bins);
    if (!xh::policy_shape_supported(c.bins, c.dims, c.policy_h1, c.policy_h2))
      return fail(XH_ERR_INVALID,
                  "unsupported policy shape B=%d D=%d widths=[%d,%d]", c.bins,
                  c.dims, c.policy_h1, c.policy_h2);
    if (!xh::value_shape_supported(c.value_h1, c.value_h2))
      return fail(XH_ERR_INVALID, "unsupported value widths [%d,%d]",
                  c.value_h1, c.value_h2);
    const int G = c.bins <= 64 ? 64 / c.bins : 1;  // envs per 64-row group
    if (c.num_envs <= 0 || c.num_envs % G)
      return fail(XH_ERR_INVALID, "num_envs %d must be a positive multiple of %d",
                  c.num_envs, G);
    if (c.steps < 1 || c.steps > 1024)
      return fail(XH_ERR_INVALID, "steps %d not in [1,1024]", c.steps);
    if (c.epochs < 1 || c.epochs > 64)
      return fail(XH_ERR_INVALID, "epochs %d", c.epochs);
    if (c.num_envs_global < c.num_envs || c.env_offset < 0 ||
        c.env_offset + c.num_envs > c.num_envs_global)
      return fail(XH_ERR_INVALID, "env partition offset %d + %d > global %d",
                  c.env_offset, c.num_envs, c.num_envs_global);
    if (c.bins * 2 * c.dims > 768)
      return fail(XH_ERR_INVALID, "value input %d > 768", c.bins * 2 * c.dims);
    if (c.train_grid_cap < 0)
      return fail(XH_ERR_INVALID, "train_grid_cap %d < 0", c.train_grid_cap);
    HIPCHK(hipSetDevice(ctx->device));

    auto *t = new xh_trainer;
    t->ctx = ctx;
    t->cfg = c;
    t->Tb = c.steps;
    // minstd_rand0 seeding rule: s mod m, 0 -> 1
    t->cfg.rng_state = c.rng_state % 2147483647u;
    if (t->cfg.rng_state == 0) t->cfg.rng_state = 1;
    t->env = make_env(c.bins, c.dims);
    t->pl = xh::PolicyLayout{2 * c.dims, c.policy_h1, c.policy_h2};
    t->vl = xh::ValueLayout{c.bins * 2 * c.dims, c.value_h1, c.value_h2};
    t->np = t->pl.size();
    t->nv = t->vl.size();
    const size_t N = t->N(), T = t->T();
    int st = XH_OK;
    auto A = [&](auto **p, size_t bytes) {
      if (st == XH_OK) st = dalloc(t, p, bytes);
    };
    // + 64 B: the value forward's 8-byte loads may read past a row's last
    // byte (vnet_forward_kernel; the bytes meet zero weights)
    A(&t->bins, (T + 1) * N * t->BD() + 64);
    A(&t->items, (T + 1) * N * 4 + 64);
    A(&t->action, T * N * 4);
    A(&t->forced, T * N * 4);
    A(&t->pold, T * N * 4);
    A(&t->done, T * N);
    A(&t->rng, N * 4);
    A(&t->pp, (size_t)t->np * 4);
    A(&t->vp, (size_t)t->nv * 4);
    A(&t->v_state, (T + 1) * N * 4);
    // V(S_0..S_T) then V(E_t) of the terminal transitions only (end_list
    // order, n_end rows): one forward batch; v_term receives them by row
    A(&t->v_state0, (2 * T + 1) * N * 4);
    A(&t->v_term, T * N * 4);
    A(&t->end_list, T * N * 4);
    A(&t->n_end, 4);
    A(&t->n_open, 4);
    A(&t->vrows, 4);
    A(&t->end_scratch, (size_t)xh::end_list_scratch_ints((int)N) * 4);
    A(&t->targets, T * N * 4);
    A(&t->adv, T * N * 4);
    A(&t->row_g, T * N * 4);
    A(&t->vact[0], (2 * T + 1) * N * c.value_h1 * 4);
    A(&t->vact[1], (2 * T + 1) * N * c.value_h2 * 4);
    A(&t->vgr[0], T * N * c.value_h1 * 4);
    A(&t->vgr[1], T * N * c.value_h2 * 4);
    t->rgrid = xh::rollout_grid(c.bins, c.dims, c.policy_h1, c.policy_h2);
    t->pslab_n = xh::policy_train_grid(c.bins, c.dims, c.policy_h1, c.policy_h2,
                                       c.algo == XH_KLPPO);
    const int groups = (int)(T * N / (size_t)G);
    if (c.train_grid_cap > 0) {
      if (t->pslab_n > c.train_grid_cap)
        t->pslab_n = c.train_grid_cap;  // test-only depth control (xylo_hip.h)
    } else if (groups > t->pslab_n * kMaxTrainDepth) {
      // a batch beyond one GPU's BASELINE share (the 8-GPU jobs' whole
      // batches on one device): more workgroups than the one-per-CU grid, so
      // that no f32 gradient slab accumulates more than kMaxTrainDepth row
      // groups -- the depth the bench configurations run at, where the
      // tests hold the gradient error flat (tests/test_gpu_depth.py).  A
      // multiple of 8 keeps the kernels' XCD-aware work order.
      const int want = (groups + kMaxTrainDepth - 1) / kMaxTrainDepth;
      t->pslab_n = (want + 7) & ~7;
    }
    if (t->pslab_n > groups) t->pslab_n = groups;
    t->pslab_stride = (t->np + 63) & ~63;
    t->vslab_n = 256;
    const long vrows = (long)T * N;
    if (t->vslab_n > vrows) t->vslab_n = (int)vrows;
    t->vslab_stride = (t->nv + 63) & ~63;
    A(&t->pslab, (size_t)t->pslab_n * t->pslab_stride * 4);
    A(&t->vslab, (size_t)t->vslab_n * t->vslab_stride * 4);
    A(&t->vw0red, (size_t)c.value_h1 * (c.bins * c.dims + c.dims) * 4);
    A(&t->vw0frag, xh::vnet_frag_bytes(t->env));
    A(&t->pgrads, (size_t)c.epochs * t->np * 4);
    A(&t->vgrad, (size_t)t->nv * 4);
    A(&t->logits, N * c.bins * 4);
    A(&t->probs, N * c.bins * 4);
    if (c.adv_normalize) {
      A(&t->adv_part, (size_t)xh::gae_grid((int)N) * 2 * 8);
      A(&t->adv_stats, 2 * 8);
    }
    if (c.algo == XH_KLPPO || c.record_distrib)
      A(&t->qold, T * N * c.bins * 4);
    if (c.algo == XH_KLPPO) {
      A(&t->beta, 4);
      A(&t->kl_log, (size_t)c.epochs * 3 * 4);
      A(&t->kl_part, (size_t)t->pslab_n * 8);
      A(&t->kl_sum, 2 * 8);
    }
    if (st != XH_OK) {
      std::string keep = g_err;
      xh_trainer_destroy(t);
      g_err = keep;
      return st;
    }
    if (st == XH_OK && t->beta)
      st = copy_ok(copy_to_device(t->beta, &c.kl_beta, 4, ctx->stream));
    t->opt[XH_POLICY].lr = c.lr_policy;
    t->opt[XH_POLICY].wd = c.wd_policy;
    t->opt[XH_VALUE].lr = c.lr_value;
    t->opt[XH_VALUE].wd = c.wd_value;
    if (st != XH_OK) {
      std::string keep = g_err;
      xh_trainer_destroy(t);
      g_err = keep;
      return st;
    }
    // a^(4T(Ng-1)): from this env's last draw of an iteration to its next.
    t->jump_mul = mstd_pow(4ull * T * (uint64_t)(c.num_envs_global - 1));
    hipError_t e = xh::launch_env_init(t->env, t->batch(), t->cfg.rng_state,
                                       c.env_offset, c.num_envs_global,
                                       ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
      xh_trainer_destroy(t);
      return fail(XH_ERR_HIP, "env init: %s", hipGetErrorString(e));
    }
    t->counted = true;
    ++ctx->trainers;
    *out = t;
    return XH_OK;
  });
}

int xh_trainer_destroy(xh_trainer *t) {
  return guard([&]() -> int {
    if (!t) return XH_OK;
    (void)hipSetDevice(t->ctx->device);
    (void)hipStreamSynchronize(t->ctx->stream);
    for (auto &ev : t->events) {
      (void)hipEventDestroy(ev.start);
      (void)hipEventDestroy(ev.stop);
    }
    for (hipEvent_t e : t->event_pool) (void)hipEventDestroy(e);
    for (void *p : t->allocs) (void)hipFree(p);
    if (t->pg.host_active) (void)hipHostFree(t->pg.host_active);
    xh_ctx *c = t->ctx;
    const bool counted = t->counted;
    delete t;
    if (counted && --c->trainers == 0 && c->closing) ctx_free(c);
    return XH_OK;
  });
}

size_t xh_trainer_num_params(const xh_trainer *t, int which) {
  if (!t) return 0;
  return which == XH_POLICY ? (size_t)t->np : (size_t)t->nv;
}

int xh_trainer_set_params(xh_trainer *t, int which, const float *host,
                          size_t n) {
  return guard([&]() -> int {
    if (!t || !host) return fail(XH_ERR_INVALID, "null arg");
    const size_t want = xh_trainer_num_params(t, which);
    if (n != want)
      return fail(XH_ERR_INVALID, "params: got %zu floats, model has %zu", n,
                  want);
    HIPCHK(hipSetDevice(t->ctx->device));
    if (which != XH_POLICY) t->vfrag_ready = false;
    float *dst = which == XH_POLICY ? t->pp : t->vp;
    HIPCHK(copy_to_device(dst, host, n * 4, t->ctx->stream));
    HIPCHK(hipStreamSynchronize(t->ctx->stream));
    return XH_OK;
  });
}

int xh_trainer_get_params(xh_trainer *t, int which, float *host, size_t n) {
  return guard([&]() -> int {
    if (!t || !host) return fail(XH_ERR_INVALID, "null arg");
    const size_t want = xh_trainer_num_params(t, which);
    if (n != want)
      return fail(XH_ERR_INVALID, "params: got %zu floats, model has %zu", n,
                  want);
    HIPCHK(hipSetDevice(t->ctx->device));
    HIPCHK(copy_to_host(host, which == XH_POLICY ? t->pp : t->vp, n * 4,
                        t->ctx->stream));
    HIPCHK(hipStreamSynchronize(t->ctx->stream));
    return XH_OK;
  });
}

int xh_trainer_set_optimizer(xh_trainer *t, int which, int kind, float lr,
                             float weight_decay, float beta1, float beta2) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    if (which != XH_POLICY && which != XH_VALUE)
      return fail(XH_ERR_INVALID, "optimizer: which %d", which);
    if (kind != XH_OPT_SGD && kind != XH_OPT_MOMENTUM && kind != XH_OPT_ADAM)
      return fail(XH_ERR_INVALID, "optimizer: kind %d", kind);
    if (kind != XH_OPT_SGD && weight_decay != 0.0f)
      return fail(XH_ERR_INVALID, "optimizer: weight decay is an "
                  "sgd_optimizer parameter only (nn.h:616-628)");
    HIPCHK(hipSetDevice(t->ctx->device));
    auto &o = t->opt[which];
    const int n = which == XH_POLICY ? t->np : t->nv;
    if (kind != XH_OPT_SGD && !o.m) {
      CHK(dalloc(t, &o.m, (size_t)n * 4));
      CHK(dalloc(t, &o.v, (size_t)n * 4));
    }
    if (o.m) {  // fresh state: the reference emplaces zeros on the first step
      HIPCHK(hipMemsetAsync(o.m, 0, (size_t)n * 4, t->ctx->stream));
      HIPCHK(hipMemsetAsync(o.v, 0, (size_t)n * 4, t->ctx->stream));
    }
    o.kind = kind;
    o.lr = lr;
    o.wd = weight_decay;
    o.beta1 = beta1;
    o.beta2 = beta2;
    o.t = 1.0f;
    (which == XH_POLICY ? t->cfg.lr_policy : t->cfg.lr_value) = lr;
    (which == XH_POLICY ? t->cfg.wd_policy : t->cfg.wd_value) = weight_decay;
    HIPCHK(hipStreamSynchronize(t->ctx->stream));
    return XH_OK;
  });
}

int xh_trainer_set_learning_rate(xh_trainer *t, int which, float lr) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    if (which != XH_POLICY && which != XH_VALUE)
      return fail(XH_ERR_INVALID, "learning rate: which %d", which);
    if (which == XH_VALUE && t->cfg.algo == XH_PG)
      return fail(XH_ERR_INVALID, "learning rate: REINFORCE has no value net");
    t->opt[which].lr = lr;
    (which == XH_POLICY ? t->cfg.lr_policy : t->cfg.lr_value) = lr;
    return XH_OK;
  });
}

int xh_trainer_set_record_last_step(xh_trainer *t, int on) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    t->cfg.record_last_step = on ? 1 : 0;
    return XH_OK;
  });
}

int xh_trainer_rollout(xh_trainer *t) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    HIPCHK(hipSetDevice(t->ctx->device));
    return do_rollout(t);
  });
}

int xh_trainer_learn(xh_trainer *t) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    HIPCHK(hipSetDevice(t->ctx->device));
    return do_learn(t);
  });
}

int xh_trainer_forget(xh_trainer *t) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    // replay_buffer::forget() keeps the last state of the open trajectories
    // of a window that exists: without a rollout since the last learn() /
    // forget() there is none, and slot T holds no start states to shift
    if (!t->rolled)
      return fail(XH_ERR_STATE, "forget: no rollout since the last learn() / "
                  "forget()");
    t->need_shift = true;  // as at the end of do_learn / do_pg_learn
    t->rolled = false;
    return XH_OK;
  });
}

int xh_trainer_iterate(xh_trainer *t, int iterations) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    HIPCHK(hipSetDevice(t->ctx->device));
    for (int i = 0; i < iterations; ++i) {
      CHK(do_rollout(t));
      CHK(do_learn(t));
    }
    return XH_OK;
  });
}

int xh_trainer_set_forced_actions(xh_trainer *t, const int32_t *host) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    if (!host) {
      t->use_forced = false;
      return XH_OK;
    }
    const size_t n = t->T() * t->N();
    for (size_t i = 0; i < n; ++i)
      if (host[i] < 0 || host[i] >= t->cfg.bins)
        return fail(XH_ERR_INVALID, "forced action %d out of range", host[i]);
    HIPCHK(hipSetDevice(t->ctx->device));
    HIPCHK(copy_to_device(t->forced, host, n * 4, t->ctx->stream));
    HIPCHK(hipStreamSynchronize(t->ctx->stream));
    t->use_forced = true;
    return XH_OK;
  });
}

size_t xh_trainer_buffer_bytes(const xh_trainer *t, int which) {
  return t && buffer_ptr(t, which) ? buffer_bytes(t, which) : 0;
}

int xh_trainer_get_buffer(xh_trainer *t, int which, void *host, size_t bytes) {
  return guard([&]() -> int {
    if (!t || !host) return fail(XH_ERR_INVALID, "null arg");
    const size_t want = xh_trainer_buffer_bytes(t, which);
    if (!want || bytes != want)
      return fail(XH_ERR_INVALID, "buffer %d: %zu bytes, expected %zu", which,
                  bytes, want);
    if ((which == XH_BUF_LOGITS || which == XH_BUF_PROBS) &&
        t->cfg.algo != XH_PG && !t->last_step_recorded)
      return fail(XH_ERR_STATE, "buffer %d: no rollout recorded its last step "
                  "(xh_config.record_last_step is off)", which);
    HIPCHK(hipSetDevice(t->ctx->device));
    HIPCHK(copy_to_host(host, buffer_ptr(t, which), bytes, t->ctx->stream));
    HIPCHK(hipStreamSynchronize(t->ctx->stream));
    return XH_OK;
  });
}

int xh_trainer_set_buffer(xh_trainer *t, int which, const void *host,
                          size_t bytes) {
  return guard([&]() -> int {
    if (!t || !host) return fail(XH_ERR_INVALID, "null arg");
    const size_t want = xh_trainer_buffer_bytes(t, which);
    if (!want || bytes != want)
      return fail(XH_ERR_INVALID, "buffer %d: %zu bytes, expected %zu", which,
                  bytes, want);
    if (which == XH_BUF_ACTION) {
      const int32_t *a = static_cast<const int32_t *>(host);
      for (size_t i = 0; i < bytes / 4; ++i)
        if (a[i] < 0 || a[i] >= t->cfg.bins)
          return fail(XH_ERR_INVALID, "action %d out of range", a[i]);
    }
    const bool states = t->cfg.algo != XH_PG &&
                        (which == XH_BUF_BINS || which == XH_BUF_ITEMS);
    std::vector<char> wide;
    if (states && which == XH_BUF_BINS) {  // as xh_trainer_set_env_state
      const int8_t *b = static_cast<const int8_t *>(host);
      const size_t per_slot = t->N() * t->BD();
      wide.assign(t->T() + 1, 0);
      for (size_t i = 0; i < bytes; ++i) {
        if (b[i] > kBinCapacity)
          return fail(XH_ERR_INVALID, "bin value %d above the capacity %d",
                      b[i], kBinCapacity);
        if (b[i] < -kBinCapacity) wide[i / per_slot] = 1;
      }
    }
    std::vector<char> ok;
    if (states && which == XH_BUF_ITEMS) {
      const int8_t *v = static_cast<const int8_t *>(host);
      const size_t N = t->N(), D = (size_t)t->cfg.dims;
      ok.assign(t->T() + 1, 1);
      for (size_t sl = 0; sl <= t->T(); ++sl)
        for (size_t e = 0; e < N; ++e) {
          const int8_t *it = v + (sl * N + e) * 4;
          bool is_a = true, is_b = true;
          for (size_t d = 0; d < D; ++d) {
            if (it[d] < 0 || it[d] > kBinCapacity)
              return fail(XH_ERR_INVALID, "item value %d outside [0, %d]", it[d],
                          kBinCapacity);
            is_a &= it[d] == t->env.item_a[d];
            is_b &= it[d] == t->env.item_b[d];
          }
          if (!is_a && !is_b) ok[sl] = 0;
        }
    }
    HIPCHK(hipSetDevice(t->ctx->device));
    HIPCHK(copy_to_device(buffer_ptr(t, which), host, bytes, t->ctx->stream));
    HIPCHK(hipStreamSynchronize(t->ctx->stream));
    if (which == XH_BUF_BINS || which == XH_BUF_ITEMS) t->need_shift = false;
    if (!ok.empty()) t->items_ok = std::move(ok);
    if (!wide.empty()) t->bins_wide = std::move(wide);
    return XH_OK;
  });
}

int xh_trainer_evaluate(xh_trainer *t, xh_eval *e) {
  return guard([&]() -> int {
    if (!t || !e) return fail(XH_ERR_INVALID, "null trainer / eval");
    const int G = t->cfg.bins <= 64 ? 64 / t->cfg.bins : 0;
    if (G == 0)
      return fail(XH_ERR_INVALID, "evaluate: bins %d > 64 not supported",
                  t->cfg.bins);
    return eval_common(t->ctx, t->env, G, e, [&](const EvalBuffers &eb) {
      xh::EvalArgs a{};
      a.env = t->env;
      a.params = t->pp;
      a.n_envs = e->n_envs;
      a.episodes = e->episodes;
      a.argmax_probs = e->argmax_probs ? 1 : 0;
      a.x0 = eb.x0;
      a.stream_stride = kEvalStride;
      a.max_steps = eb.max_steps;
      a.init_items = eb.init_items;
      a.total = eb.total;
      a.steps = eb.steps;
      a.rng_out = eb.rng_out;
      a.final_items = eb.final_items;
      a.trace = eb.trace;
      a.trace_cap = eb.trace_cap;
      return xh::launch_eval_argmax(a, t->cfg.policy_h1, t->cfg.policy_h2,
                                    t->ctx->stream);
    });
  });
}

int xh_heuristic_evaluate(xh_ctx *ctx, int policy, int bins, int dims,
                          xh_eval *e) {
  return guard([&]() -> int {
    if (!ctx || !e) return fail(XH_ERR_INVALID, "null ctx / eval");
    if (policy < XH_HEUR_RANDOM || policy > XH_HEUR_MINWASTE)
      return fail(XH_ERR_INVALID, "heuristic policy %d", policy);
    if (!xh::heuristic_shape_supported(bins, dims))
      return fail(XH_ERR_INVALID, "heuristic: bins %d dims %d not supported",
                  bins, dims);
    const xh::EnvDesc env = make_env(bins, dims);
    return eval_common(ctx, env, 64 / bins, e, [&](const EvalBuffers &eb) {
      xh::HeuristicArgs a{};
      a.env = env;
      a.n_envs = e->n_envs;
      a.episodes = e->episodes;
      a.x0 = eb.x0;
      a.stream_stride = kEvalStride;
      a.max_steps = eb.max_steps;
      a.init_items = eb.init_items;
      a.total = eb.total;
      a.steps = eb.steps;
      a.rng_out = eb.rng_out;
      a.final_items = eb.final_items;
      a.trace = eb.trace;
      a.trace_cap = eb.trace_cap;
      return xh::launch_heuristic(a, policy, ctx->stream);
    });
  });
}

int xh_trainer_seed_streams(xh_trainer *t, uint32_t x) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    x %= 2147483647u;
    HIPCHK(hipSetDevice(t->ctx->device));
    if (t->cfg.algo == XH_PG) {
      HIPCHK(xh::launch_pg_seed(t->batch(), x ? x : 1u, t->cfg.env_offset,
                                kEvalStride, t->ctx->stream));
      return XH_OK;
    }
    HIPCHK(xh::launch_env_seed(t->batch(), x ? x : 1u, t->cfg.env_offset,
                               t->ctx->stream));
    return XH_OK;
  });
}

int xh_trainer_set_timing(xh_trainer *t, int on) {
  if (!t) return fail(XH_ERR_INVALID, "null trainer");
  if (on < 0 || on > XH_TIMING_TRAIN)
    return fail(XH_ERR_INVALID, "set_timing: mode %d (0, 1 or XH_TIMING_TRAIN)", on);
  t->timing = on;
  return XH_OK;
}

int xh_trainer_reset_timing(xh_trainer *t) {
  return guard([&]() -> int {
    if (!t) return fail(XH_ERR_INVALID, "null trainer");
    HIPCHK(hipStreamSynchronize(t->ctx->stream));
    for (auto &ev : t->events) {
      t->event_pool.push_back(ev.start);
      t->event_pool.push_back(ev.stop);
    }
    t->events.clear();
    return XH_OK;
  });
}


int xh_trainer_kernel_info(xh_trainer *t, char *buf, size_t cap) {
  return guard([&]() -> int {
    if (!t || !buf || cap == 0) return fail(XH_ERR_INVALID, "null arg");
    const std::string js = "{\"rollout_step\": " + kernel_json(t->last_rollout) +
                           ", \"policy_train\": " + kernel_json(t->last_train) +
                           ", \"value\": \"" +
                           std::string(t->cfg.algo != XH_PG
                                           ? xh::value_kernel_name(value_mlp(t, 0, nullptr))
                                           : "gemm") +
                           "\", \"train_grid\": " + std::to_string(t->pslab_n) +
                           ", \"train_grid_cap\": " +
                           std::to_string(t->cfg.train_grid_cap) +
                           ", \"overrides\": {" + env_json("XH_TRAIN_KERNEL") +
                           ", " + env_json("XH_ROLLOUT_KERNEL") + ", " +
                           env_json("XH_VALUE_KERNEL") + "}}";
    if (js.size() + 1 > cap)
      return fail(XH_ERR_INVALID, "kernel_info: %zu bytes needed", js.size() + 1);
    std::memcpy(buf, js.c_str(), js.size() + 1);
    return XH_OK;
  });
}

int xh_ctx_inject_fault(xh_ctx *c, int kind) {
  return guard([&]() -> int {
    if (!c) return fail(XH_ERR_INVALID, "null ctx");
    if (kind != XH_FAULT_NONE && kind != XH_FAULT_RCCL_ARG)
      return fail(XH_ERR_INVALID, "unknown fault %d", kind);
    if (kind == XH_FAULT_RCCL_ARG && !c->comm)
      return fail(XH_ERR_STATE, "inject_fault: the context has no communicator");
    c->fault = kind;
    return XH_OK;
  });
}

int xh_trainer_kernel_time(xh_trainer *t, const char *name, double *ms,
                           long *launches) {
  return guard([&]() -> int {
    if (!t || !name || !ms || !launches) return fail(XH_ERR_INVALID, "null arg");
    HIPCHK(hipStreamSynchronize(t->ctx->stream));
    double total = 0;
    long n = 0;
    for (auto &ev : t->events) {
      if (ev.name != name) continue;
      float e = 0;
      HIPCHK(hipEventElapsedTime(&e, ev.start, ev.stop));
      total += e;
      ++n;
    }
    *ms = total;
    *launches = n;
    return XH_OK;
  });
}

int xh_trainer_get_env_state(xh_trainer *t, int first, int count, int8_t *bins,
                             int8_t *items) {
  return guard([&]() -> int {
    if (!t || (count && (!bins || !items)))
      return fail(XH_ERR_INVALID, "null arg");
    if (t->cfg.algo == XH_PG)
      return fail(XH_ERR_INVALID, "env state access: not for XH_PG trainers");
    if (first < 0 || count < 0 || first + count > t->cfg.num_envs)
      return fail(XH_ERR_INVALID, "envs [%d, %d) of %d", first, first + count,
                  t->cfg.num_envs);
    HIPCHK(hipSetDevice(t->ctx->device));
    hipStream_t s = t->ctx->stream;
    const size_t BD = t->BD(), D = (size_t)t->cfg.dims, N = t->N();
    const size_t slot = t->need_shift ? t->T() : 0;
    std::vector<int8_t> it((size_t)count * 4);
    HIPCHK(copy_to_host(bins, t->bins + (slot * N + first) * BD,
                        (size_t)count * BD, s));
    HIPCHK(copy_to_host(it.data(), t->items + (slot * N + first) * 4,
                        (size_t)count * 4, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int e = 0; e < count; ++e) {
      auto o = t->env_override.find(first + e);
      if (o != t->env_override.end()) {
        std::memcpy(bins + (size_t)e * BD, o->second.data(), BD);
        std::memcpy(items + (size_t)e * D, o->second.data() + BD, D);
      } else {
        std::memcpy(items + (size_t)e * D, it.data() + (size_t)e * 4, D);
      }
    }
    return XH_OK;
  });
}

int xh_trainer_set_env_state(xh_trainer *t, int first, int count,
                             const int8_t *bins, const int8_t *items) {
  return guard([&]() -> int {
    if (!t || (count && (!bins || !items)))
      return fail(XH_ERR_INVALID, "null arg");
    if (t->cfg.algo == XH_PG)
      return fail(XH_ERR_INVALID, "env state access: not for XH_PG trainers");
    if (first < 0 || count < 0 || first + count > t->cfg.num_envs)
      return fail(XH_ERR_INVALID, "envs [%d, %d) of %d", first, first + count,
                  t->cfg.num_envs);
    const size_t BD = t->BD(), D = (size_t)t->cfg.dims;
    // negative values are the overflowed (game-over) states an apply by hand
    // leaves (bin_packing.h:53-63); applying to a game-over env again keeps
    // subtracting, so any int8 value up to the capacity is a reachable state
    // (below -capacity the next rollout step / learn() run the f32 kernels,
    // bins_wide)
    for (size_t i = 0; i < (size_t)count * BD; ++i)
      if (bins[i] > kBinCapacity)
        return fail(XH_ERR_INVALID, "bin value %d above the capacity %d",
                    bins[i], kBinCapacity);
    // a whole item-table entry (the train kernels carry the item columns of
    // dW1 as per-entry sums)
    for (int e = 0; e < count; ++e) {
      bool is_a = true, is_b = true;
      for (size_t d = 0; d < D; ++d) {
        is_a &= items[e * D + d] == t->env.item_a[d];
        is_b &= items[e * D + d] == t->env.item_b[d];
      }
      if (!is_a && !is_b)
        return fail(XH_ERR_INVALID, "env %d: item is not an item-table entry",
                    first + e);
    }
    for (int e = 0; e < count; ++e) {
      std::vector<int8_t> v(BD + D);
      std::memcpy(v.data(), bins + (size_t)e * BD, BD);
      std::memcpy(v.data() + BD, items + (size_t)e * D, D);
      t->env_override[first + e] = std::move(v);
    }
    return XH_OK;
  });
}

// ------------------------------------------------------------------ venv --
}  // extern "C"
namespace {
void venv_drop_events(xh_venv *v, bool destroy = false);
}  // namespace
extern "C" {

int xh_venv_create(xh_ctx *ctx, int num_envs, int bins, int dims,
                   uint32_t rng_state, int env_offset, int num_envs_global,
                   int policy_draws, xh_venv **out) {
  return guard([&]() -> int {
    if (!ctx || !out) return fail(XH_ERR_INVALID, "null arg");
    if (!xh::venv_shape_supported(bins, dims))
      return fail(XH_ERR_INVALID, "venv: bins %d (8/16/32/64/128), dims %d "
                  "(1..3)", bins, dims);
    if (num_envs < 1 || env_offset < 0 || num_envs_global < num_envs ||
        env_offset + num_envs > num_envs_global)
      return fail(XH_ERR_INVALID, "venv: envs %d at offset %d of %d", num_envs,
                  env_offset, num_envs_global);
    if (policy_draws < 0 || policy_draws > 64)
      return fail(XH_ERR_INVALID, "venv: policy_draws %d", policy_draws);
    HIPCHK(hipSetDevice(ctx->device));
    auto *v = new xh_venv;
    v->ctx = ctx;
    v->env = make_env(bins, dims);
    v->N = num_envs;
    v->Ng = num_envs_global;
    v->offset = env_offset;
    v->policy_draws = policy_draws;
    const uint64_t k = (uint64_t)policy_draws + 2;
    v->skip_mul = mstd_pow((uint64_t)policy_draws);
    v->jump_mul = mstd_pow(k * (uint64_t)(num_envs_global - 1));
    const size_t N = (size_t)num_envs, BD = (size_t)bins * dims;
    const size_t sz[XH_VENV_BUF_COUNT] = {N * 4, N * 4, N, N * BD, N * 4, N * 4,
                                          N * BD * 2 * 4, N};
    int st = XH_OK;
    for (int b = 0; b < XH_VENV_BUF_COUNT && st == XH_OK; ++b) {
      v->bytes[b] = sz[b];
      if (hipMalloc(&v->buf[b], sz[b]) != hipSuccess ||
          hipMemsetAsync(v->buf[b], 0, sz[b], ctx->stream) != hipSuccess)
        st = fail(XH_ERR_HIP, "venv: allocating %zu bytes", sz[b]);
    }
    if (st == XH_OK && (hipMalloc((void **)&v->err, 4) != hipSuccess ||
                        hipMemsetAsync(v->err, 0, 4, ctx->stream) != hipSuccess))
      st = fail(XH_ERR_HIP, "venv: error flag");
    if (st == XH_OK) {
      uint32_t x0 = rng_state % 2147483647u;
      const hipError_t e = xh::launch_venv_init(v->args(), x0 ? x0 : 1u,
                                                env_offset, num_envs_global,
                                                (int)k, ctx->stream);
      if (e != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess)
        st = fail(XH_ERR_HIP, "venv init: %s", hipGetErrorString(e));
    }
    v->counted = true;
    ++ctx->trainers;
    if (st != XH_OK) {
      std::string keep = g_err;
      xh_venv_destroy(v);
      g_err = keep;
      return st;
    }
    *out = v;
    return XH_OK;
  });
}

int xh_venv_destroy(xh_venv *v) {
  return guard([&]() -> int {
    if (!v) return XH_OK;
    (void)hipSetDevice(v->ctx->device);
    (void)hipStreamSynchronize(v->ctx->stream);
    venv_drop_events(v, true);
    for (void *p : v->buf)
      if (p) (void)hipFree(p);
    if (v->err) (void)hipFree(v->err);
    xh_ctx *c = v->ctx;
    const bool counted = v->counted;
    delete v;
    if (counted && --c->trainers == 0 && c->closing) ctx_free(c);
    return XH_OK;
  });
}

size_t xh_venv_bytes(const xh_venv *v, int which) {
  return v && which >= 0 && which < XH_VENV_BUF_COUNT ? v->bytes[which] : 0;
}

void *xh_venv_device_ptr(xh_venv *v, int which) {
  return v && which >= 0 && which < XH_VENV_BUF_COUNT ? v->buf[which] : nullptr;
}

namespace {
int venv_check_err(xh_venv *v) {
  int err = 0;
  HIPCHK(copy_to_host(&err, v->err, 4, v->ctx->stream));
  HIPCHK(hipStreamSynchronize(v->ctx->stream));
  if (err) {
    HIPCHK(hipMemsetAsync(v->err, 0, 4, v->ctx->stream));
    HIPCHK(hipStreamSynchronize(v->ctx->stream));
    return fail(XH_ERR_INVALID, "venv: an action was outside [0, %d); those "
                "envs were left untouched", v->env.B);
  }
  return XH_OK;
}
int venv_launch(xh_venv *v, int op, int mode, bool use_mask, bool obs) {
  HIPCHK(hipSetDevice(v->ctx->device));
  xh::VenvArgs a = v->args();
  a.mode = mode;
  a.mask = use_mask ? (const uint8_t *)v->buf[XH_VENV_MASK] : nullptr;
  a.obs = obs ? (float *)v->buf[XH_VENV_OBS] : nullptr;
  if (op == xh::kVenvObserve) a.obs = (float *)v->buf[XH_VENV_OBS];
  if (mode == 0) a.reward = nullptr;
  // events from a pool (no creation per launch); a pair is kept only once
  // both of its records are on the stream, so a failed launch leaves no
  // half-recorded pair behind
  std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
  auto pooled = [&](hipEvent_t *e) -> hipError_t {
    if (!v->event_pool.empty()) {
      *e = v->event_pool.back();
      v->event_pool.pop_back();
      return hipSuccess;
    }
    return hipEventCreateWithFlags(e, hipEventDisableSystemFence);
  };
  if (v->timing) {
    HIPCHK(pooled(&ev.first));
    HIPCHK(pooled(&ev.second));
    HIPCHK(hipEventRecord(ev.first, v->ctx->stream));
  }
  const hipError_t e = xh::launch_venv(a, op, v->ctx->stream);
  if (e != hipSuccess) {
    if (v->timing) {
      v->event_pool.push_back(ev.first);
      v->event_pool.push_back(ev.second);
    }
    return fail(XH_ERR_HIP, "venv launch: %s", hipGetErrorString(e));
  }
  if (v->timing) {
    HIPCHK(hipEventRecord(ev.second, v->ctx->stream));
    v->events.push_back(ev);
  }
  return XH_OK;
}
// the recorded pairs back into the pool (the stream is synchronised first);
// destroy = true at xh_venv_destroy
void venv_drop_events(xh_venv *v, bool destroy) {
  for (auto &ev : v->events) {
    v->event_pool.push_back(ev.first);
    v->event_pool.push_back(ev.second);
  }
  v->events.clear();
  if (destroy) {
    for (hipEvent_t e : v->event_pool) (void)hipEventDestroy(e);
    v->event_pool.clear();
  }
}
}  // namespace

int xh_venv_get(xh_venv *v, int which, void *host, size_t bytes) {
  return guard([&]() -> int {
    if (!v || !host) return fail(XH_ERR_INVALID, "null arg");
    if (which < 0 || which >= XH_VENV_BUF_COUNT || bytes != v->bytes[which])
      return fail(XH_ERR_INVALID, "venv buffer %d: %zu bytes, expected %zu",
                  which, bytes, xh_venv_bytes(v, which));
    HIPCHK(hipSetDevice(v->ctx->device));
    HIPCHK(copy_to_host(host, v->buf[which], bytes, v->ctx->stream));
    return venv_check_err(v);
  });
}

int xh_venv_set(xh_venv *v, int which, const void *host, size_t bytes) {
  return guard([&]() -> int {
    if (!v || !host) return fail(XH_ERR_INVALID, "null arg");
    if (which < 0 || which >= XH_VENV_BUF_COUNT || bytes != v->bytes[which])
      return fail(XH_ERR_INVALID, "venv buffer %d: %zu bytes, expected %zu",
                  which, bytes, xh_venv_bytes(v, which));
    if (which == XH_VENV_ACTIONS) {
      const int32_t *a = static_cast<const int32_t *>(host);
      for (int i = 0; i < v->N; ++i)
        if (a[i] < 0 || a[i] >= v->env.B)
          return fail(XH_ERR_INVALID, "venv: action %d of env %d outside "
                      "[0, %d)", a[i], i, v->env.B);
    }
    if (which == XH_VENV_BINS) {
      const int8_t *b = static_cast<const int8_t *>(host);
      // any int8 value up to the capacity: the venv computes in int / f32
      // (an apply to a game-over env keeps subtracting, bin_packing.h:53-63)
      for (size_t i = 0; i < bytes; ++i)
        if (b[i] > kBinCapacity)
          return fail(XH_ERR_INVALID, "venv: bin value %d above the capacity %d",
                      b[i], kBinCapacity);
    }
    HIPCHK(hipSetDevice(v->ctx->device));
    HIPCHK(copy_to_device(v->buf[which], host, bytes, v->ctx->stream));
    HIPCHK(hipStreamSynchronize(v->ctx->stream));
    return XH_OK;
  });
}

int xh_venv_step(xh_venv *v, int write_obs) {
  return guard([&]() -> int {
    if (!v) return fail(XH_ERR_INVALID, "null venv");
    return venv_launch(v, xh::kVenvStep, 1, false, write_obs != 0);
  });
}

int xh_venv_apply(xh_venv *v, int use_mask) {
  return guard([&]() -> int {
    if (!v) return fail(XH_ERR_INVALID, "null venv");
    return venv_launch(v, xh::kVenvStep, 0, use_mask != 0, false);
  });
}

int xh_venv_reset(xh_venv *v, int use_mask) {
  return guard([&]() -> int {
    if (!v) return fail(XH_ERR_INVALID, "null venv");
    return venv_launch(v, xh::kVenvReset, 0, use_mask != 0, false);
  });
}

int xh_venv_observe(xh_venv *v) {
  return guard([&]() -> int {
    if (!v) return fail(XH_ERR_INVALID, "null venv");
    return venv_launch(v, xh::kVenvObserve, 0, false, true);
  });
}

int xh_venv_set_timing(xh_venv *v, int on) {
  return guard([&]() -> int {
    if (!v) return fail(XH_ERR_INVALID, "null venv");
    HIPCHK(hipSetDevice(v->ctx->device));
    HIPCHK(hipStreamSynchronize(v->ctx->stream));
    venv_drop_events(v);
    v->timing = on != 0;
    return XH_OK;
  });
}

int xh_venv_kernel_time(xh_venv *v, double *ms, long *launches) {
  return guard([&]() -> int {
    if (!v || !ms || !launches) return fail(XH_ERR_INVALID, "null arg");
    HIPCHK(hipSetDevice(v->ctx->device));
    HIPCHK(hipStreamSynchronize(v->ctx->stream));
    double total = 0;
    for (auto &ev : v->events) {
      float e = 0;
      HIPCHK(hipEventElapsedTime(&e, ev.first, ev.second));
      total += e;
    }
    *ms = total;
    *launches = (long)v->events.size();
    return XH_OK;
  });
}

int xh_venv_synchronize(xh_venv *v) {
  return guard([&]() -> int {
    if (!v) return fail(XH_ERR_INVALID, "null venv");
    HIPCHK(hipSetDevice(v->ctx->device));
    return venv_check_err(v);
  });
}

}  // extern "C"
