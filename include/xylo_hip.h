/* xylo_hip.h -- C ABI of the MI355X-native PPO / actor-critic hot path.
 *
 * The drop-in boundary for the rollout-and-update path of
 * beehover/dependence_free_rl (reference @ 2024_10_08; citations are
 * file:line under that tree).  Plain pointers, sizes and int status codes;
 * no C++ or torch types cross this boundary; no exception escapes it.
 * Host wrappers (include/xylo_hip/ headers, dependence_free_rl_amd/_lib.py)
 * rethrow / raise on a non-zero status with xh_last_error().
 *
 * Reference interfaces replaced (one xh_trainer = many envs + the learner):
 *   xylo::environment<A,S>::apply/view/reset   xylo/rl.h:163-170
 *   bp::environment, bp::agent                 apps/bin_packing/bin_packing.h:46-107
 *   xylo::agent::step / play_steps             xylo/rl.h:325-360
 *   xylo::replay_buffer (sample_td, forget)    xylo/rl.h:213-296
 *   xylo::policy_gradient_policy::react        xylo/policy_gradient.h:337-354
 *   xylo::discrete_action::from_vector         xylo/rl.h:27-30
 *   xylo::actor_critic_learner::learn          xylo/policy_gradient.h:159-281
 *   xylo::ppo_learner::optimize_action         xylo/policy_gradient.h:297-307
 *   xylo::model::parameters / set_parameters   xylo/nn.h:490-508
 *   xylo::sgd_optimizer                        xylo/nn.h:616-628
 *   (and the tensor.{h,cc} / nn.h Dense, relu, softmax loops underneath)
 */
#ifndef XYLO_HIP_H_
#define XYLO_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------ status ---- */
enum {
  XH_OK = 0,
  XH_ERR_INVALID = 1,     /* bad argument / unsupported shape   */
  XH_ERR_HIP = 2,         /* HIP runtime error                   */
  XH_ERR_RCCL = 3,        /* RCCL error                          */
  XH_ERR_STATE = 4        /* call out of order                   */
};
/* Message of the last failing call on this thread ("" if none). */
const char *xh_last_error(void);
/* Library version string. */
const char *xh_version(void);
/* Number of visible HIP devices (initialises the HIP runtime). */
int xh_device_count(int *out);
/* JSON object naming the HIP and RCCL shared objects this process bound and
 * their versions: {"libamdhip64": path, "hip_runtime": n, "librccl": path,
 * "rccl_version": n}.  Written NUL-terminated into buf[cap]. */
int xh_runtime_info(char *buf, size_t cap);

/* ------------------------------------------------------------ context --- */
typedef struct xh_ctx xh_ctx;
/* 128-byte RCCL unique id (ncclGetUniqueId) for a world > 1 job. */
int xh_comm_unique_id(void *out128);
/* device: HIP device ordinal; rank/world: this process in a one-process-per-
 * GPU job; uid128 (required when world > 1): the id from rank 0, broadcast
 * by the caller.  With world == 1 a non-null uid128 creates a one-rank RCCL
 * communicator, so the all-reduce path runs on a single device too. */
int xh_ctx_create(int device, int rank, int world, const void *uid128,
                  xh_ctx **out);
int xh_ctx_destroy(xh_ctx *ctx);
int xh_ctx_synchronize(xh_ctx *ctx);
/* Sum-all-reduce of n floats of host memory over the job (tests/tools). */
int xh_ctx_allreduce_host(xh_ctx *ctx, float *data, size_t n);
/* Test hook: make the next gradient all-reduce of a trainer on this context
 * pass RCCL an invalid argument (XH_FAULT_RCCL_ARG), so that the error path
 * (XH_ERR_RCCL with ncclGetErrorString) runs against the real library.
 * XH_FAULT_NONE clears it.  XH_ERR_STATE without a communicator. */
enum { XH_FAULT_NONE = 0, XH_FAULT_RCCL_ARG = 1 };
int xh_ctx_inject_fault(xh_ctx *ctx, int kind);

/* ------------------------------------------------------------ trainer --- */
/* XH_KLPPO: kl_ppo_learner (policy_gradient.h:310-335, ppo2_training.cc):
 * PPO's k = 4 full-batch epochs with kl_regulated_loss and an adaptive beta
 * that carries over from one learn() to the next.  Per-bin shapes with
 * bins <= 64, and 128 bins 3-D [128,128] (the split train kernel only: a
 * batch holding an overflowed bin fails its learn() there). */
/* XH_PG: policy_gradient_learner = REINFORCE (policy_gradient.h:88-147,
 * bp::pg_learner, pg_training.cc) with a FULL-layer policy
 * full(4B, policy_h1) - relu [- full(policy_h1, policy_h2) - relu] -
 * full(., B) - softmax_cross_entropy (policy_h2 = 0: one hidden layer), no
 * value net.  `steps` is the number of whole episodes each env plays per
 * iteration (play_one_episode, rl.h:351-354); env g plays on its own engine
 * stream, rng_state advanced by g * 2^26 draws (env 0 = the single-env
 * reference run).  The batch buffers hold `xh_trainer_buffer_bytes`-sized
 * [Tmax][N] grids, Tmax = steps * (longest possible episode); XH_BUF_LEN
 * gives each env's step count of the last rollout. */
enum { XH_PPO = 0, XH_AC = 1, XH_KLPPO = 2, XH_PG = 3 };

typedef struct {
  int algo;            /* XH_PPO | XH_AC (actor_critic_learner) | XH_KLPPO
                          | XH_PG */
  int num_envs;        /* envs on this rank (multiple of 64/bins)            */
  int num_envs_global; /* envs in the whole job (reference-order RNG streams) */
  int env_offset;      /* global index of this rank's first env              */
  int bins, dims;      /* B (bin_packing.h:12 num_bins), D (2 in the ref)    */
  int steps;           /* T: env steps per env per iteration (play_steps(T));
                          1..1024 (REINFORCE: episodes per env, 1..64)     */
  int epochs;          /* PPO / KL-PPO k (policy_gradient.h:300), 1 for AC  */
  int policy_h1, policy_h2; /* per-bin conv1d_1 widths                       */
  int value_h1, value_h2;   /* value full_layer widths (64, 32)              */
  float lr_policy, lr_value, wd_policy, wd_value;
  float gamma;         /* 0.99 */
  float lambda;        /* 0.95 (policy_gradient.h:286) */
  float clip_eps;      /* 0.2  (rl.h:56) */
  uint32_t rng_state;  /* minstd_rand0 state before the envs are constructed */
  float kl_beta;       /* KL-PPO initial beta (1, policy_gradient.h:332)     */
  float kl_target;     /* KL-PPO d_targ (1e-9, policy_gradient.h:333)        */
  /* Opt-in options, both 0 (off) in the reference-parity configuration:   */
  int adv_normalize;   /* 1: after GAE, A <- (A - mean) / (std + 1e-8) over
                          the job's T * num_envs_global transitions (the
                          reference normalises nothing, policy_gradient.h:
                          220-281); statistics by wave reductions, summed
                          across ranks */
  int lr_scale_rows;   /* 1: both optimizers apply lr / rows, rows = T *
                          num_envs_global, i.e. SGD on the mean instead of the
                          reference's sum over rows (nn.h:94-98, 624) */
  /* Test-only: 0 (default) = the policy train kernels' own grid (one or two
     workgroups per CU); > 0 caps the number of train workgroups, so that a
     batch the oracle can check in seconds runs each workgroup over as many
     row groups as the benchmark's full batch does (the f32 accumulation
     depth of the per-workgroup gradient slabs).  Reported by
     xh_trainer_kernel_info ("train_grid", "train_grid_cap"); bench.py
     refuses a trainer with a cap. */
  int train_grid_cap;
  /* 1: rollouts also record every step's whole sampling distribution into
     XH_BUF_QOLD (always on for XH_KLPPO), for a learner assembled on the
     host from the layer / loss pieces below whose loss reads it
     (discrete_action::distrib, rl.h:27-30).  0 (default): only p_old. */
  int record_distrib;
  /* 1: the rollout also writes the last slot's logits and probabilities
     (XH_BUF_LOGITS / XH_BUF_PROBS: [N][B] f32 each, 16.8 MB per iteration at
     config 3) for tests and health checks.  0 (default): the product path
     writes neither, and reading those buffers fails with XH_ERR_STATE.
     xh_trainer_set_record_last_step changes it between iterations. */
  int record_last_step;
} xh_config;

/* Fill `c` with the reference defaults (ppo_training.cc) for B bins, D dims. */
void xh_config_default(xh_config *c, int algo, int bins, int dims, int num_envs,
                       int steps);

typedef struct xh_trainer xh_trainer;
/* Allocates all device buffers, constructs the envs (2 engine draws each,
 * bin_packing.h:50-52) and zero-initialises both nets (set params next). */
int xh_trainer_create(xh_ctx *ctx, const xh_config *cfg, xh_trainer **out);
int xh_trainer_destroy(xh_trainer *t);

enum { XH_POLICY = 0, XH_VALUE = 1 };
/* Flat parameters in the reference model::parameters() layout (nn.h:499-508):
 * per dense layer [A(out x in) row-major, b(out)]; weights.20 loads as-is. */
size_t xh_trainer_num_params(const xh_trainer *t, int which);
int xh_trainer_set_params(xh_trainer *t, int which, const float *host,
                          size_t n);
int xh_trainer_get_params(xh_trainer *t, int which, float *host, size_t n);

/* Optimizer of the policy (XH_POLICY) or value (XH_VALUE) net, replacing
 * xylo::sgd_optimizer / momentum_optimizer / adam_optimizer (nn.h:616-698)
 * passed to the learner constructor.  Default: sgd with the xh_config lr /
 * wd.  momentum: v = 0.9 v + g, p - lr v.  adam: moments with beta1, beta2,
 * bias-corrected with the step counter t = 1, 2, ... of this optimizer,
 * p - lr m^ / (sqrt(v^) + 1e-7).  weight_decay must be 0 unless sgd.  The
 * state (velocity, moments, t) restarts from zero at this call and then
 * persists across learn() calls, as the reference optimizer object's does. */
enum { XH_OPT_SGD = 0, XH_OPT_MOMENTUM = 1, XH_OPT_ADAM = 2 };
int xh_trainer_set_optimizer(xh_trainer *t, int which, int kind, float lr,
                             float weight_decay, float beta1, float beta2);

/* optimizer::set_rate (nn.h:591): new learning rate for the policy / value
 * optimizer from the next learn() on; its state (velocity, moments, adam's
 * step counter) is kept. */
int xh_trainer_set_learning_rate(xh_trainer *t, int which, float lr);

/* Turn the last-step logits / probabilities record (xh_config.
 * record_last_step) on or off from the next rollout on. */
int xh_trainer_set_record_last_step(xh_trainer *t, int on);

/* One iteration's rollout: T steps of every env (one kernel per step). */
int xh_trainer_rollout(xh_trainer *t);
/* learn(): value step, advantages, `epochs` policy steps; then the batch's
 * final states become the next iteration's starting states (forget()). */
int xh_trainer_learn(xh_trainer *t);
/* `iterations` x (rollout + learn), asynchronous on the trainer's stream. */
int xh_trainer_iterate(xh_trainer *t, int iterations);
/* Teacher forcing: actions [T][N] used instead of sampling (the sampler's two
 * engine draws are still consumed).  NULL disables. */
int xh_trainer_set_forced_actions(xh_trainer *t, const int32_t *host);

/* Batch / diagnostics buffers (host copies; sizes in bytes must match). */
enum {
  XH_BUF_BINS = 0,     /* int8  [T+1][N][B][D]  states S_t (slot T = next S_0) */
  XH_BUF_ITEMS = 1,    /* int8  [T+1][N][4]                                  */
  XH_BUF_ACTION = 2,   /* int32 [T][N]                                       */
  XH_BUF_POLD = 3,     /* f32   [T][N]  distrib[choice] at sampling          */
  XH_BUF_DONE = 4,     /* uint8 [T][N]                                       */
  XH_BUF_RNG = 5,      /* uint32 [N]   per-env engine state                  */
  XH_BUF_V_STATE = 6,  /* f32   [T+1][N] V(S_t) of the last value eval       */
  XH_BUF_V_TERM = 7,   /* f32   [T][N]  V(terminal view of step t); entries  */
                       /*   of transitions that did not end are unspecified */
  XH_BUF_TARGETS = 8,  /* f32   [T][N]  TD targets                           */
  XH_BUF_ADV = 9,      /* f32   [T][N]  advantages                           */
  XH_BUF_VALUE_GRAD = 10,  /* f32 [value params]  last value gradient        */
  XH_BUF_POLICY_GRADS = 11,/* f32 [epochs][policy params]                    */
  XH_BUF_LOGITS = 12,  /* f32   [N][B]  logits of the last rollout step
                                  (xh_config.record_last_step)              */
  XH_BUF_PROBS = 13,   /* f32   [N][B]  probabilities of the last step (idem) */
  XH_BUF_V_STATE0 = 14,/* f32   [T+1][N] V(S_t) before the value step        */
  XH_BUF_QOLD = 15,    /* f32   [T][N][B] sampled distributions (KL-PPO, or
                                  xh_config.record_distrib)                  */
  XH_BUF_KL = 16,      /* f32   [epochs][3] KL-PPO: beta used, mean KL, new
                                  beta of the last learn()                   */
  XH_BUF_LEN = 17,     /* int32 [N]  REINFORCE: env steps of the last rollout */
  XH_BUF_COUNT
};
size_t xh_trainer_buffer_bytes(const xh_trainer *t, int which);
int xh_trainer_get_buffer(xh_trainer *t, int which, void *host, size_t bytes);
int xh_trainer_set_buffer(xh_trainer *t, int which, const void *host,
                          size_t bytes);

/* Deterministic evaluation (policy_gradient_deterministic_policy,
 * policy_gradient.h:356-373; agent::play_one_episode, rl.h:351-354; the
 * drivers' 100-episode eval, ppo_training.cc:67-81; deep_agent.cc:25-41)
 * with the trainer's current policy.  n_envs independent envs (a multiple of
 * 64/bins) each play `episodes` whole episodes taking the argmax action (over
 * the softmax output if argmax_probs, else over the raw logits).
 *
 * Env e's minstd_rand0 stream starts at rng_state advanced by e * 2^26 draws,
 * so env 0 reproduces a single-env reference run whose global engine is at
 * rng_state.  With init_items == NULL every env is first constructed
 * (bins at capacity + get_item = 2 draws, bin_packing.h:50-52); otherwise env
 * e starts with bins at capacity and item init_items[e*dims ...] (an env that
 * was constructed or reset earlier) and draws nothing before its first step.
 * Outputs (host arrays, each may be NULL): totals/steps per env (summed
 * rewards, env steps), final_items (item after the last reset), rng_out (the
 * stream state after the last draw), trace (env 0's actions, the first
 * trace_cap of them). */
typedef struct xh_eval {
  int n_envs;
  int episodes;
  int argmax_probs;
  uint32_t rng_state;
  const int32_t *init_items; /* [n_envs][dims] or NULL */
  int32_t *final_items;      /* [n_envs][dims] or NULL */
  uint32_t *rng_out;         /* [n_envs] or NULL */
  double *totals;            /* [n_envs] or NULL */
  long *steps;               /* [n_envs] or NULL */
  int32_t *trace;            /* [trace_cap] or NULL */
  long trace_cap;
  double elapsed_ms;         /* out: device time of the evaluation kernel */
} xh_eval;
int xh_trainer_evaluate(xh_trainer *t, xh_eval *e);

/* The reference's heuristic agents as device policies, on independent envs
 * with the stream convention of xh_trainer_evaluate (env 0 reproduces a
 * single-env reference run): XH_HEUR_RANDOM = xylo::random_policy (rl.h:
 * 305-316, random_agent.cc), XH_HEUR_FIRSTFIT (firstfit_agent.cc:10-28),
 * XH_HEUR_BESTFIT (bestfit_agent.cc:10-30), XH_HEUR_MINWASTE
 * (minwaste_agent.cc:10-39).  bins in {8,16,32,64}, dims 1..3. */
enum { XH_HEUR_RANDOM = 0, XH_HEUR_FIRSTFIT = 1, XH_HEUR_BESTFIT = 2,
       XH_HEUR_MINWASTE = 3 };
int xh_heuristic_evaluate(xh_ctx *ctx, int policy, int bins, int dims,
                          xh_eval *e);

/* Re-base the per-env engine streams on a global minstd_rand0 state x: the
 * next rollout steps env g (global index) from x advanced by 4*T*g draws, i.e.
 * the reference order in which worker 0 plays its T steps, then worker 1, ...
 * (ppo_training.cc:53-62 run sequentially, 4 draws per step).  After that
 * rollout the global engine is at x advanced by 4*T*num_envs_global.
 * XH_PG: env g's stream <- x advanced by g * 2^26 draws (env 0 continues the
 * engine as a single reference worker does). */
int xh_trainer_seed_streams(xh_trainer *t, uint32_t x);

/* The state each env of the trainer starts its NEXT rollout step from (after
 * learn() that is the batch's final state, which forget() keeps,
 * rl.h:274-291): envs [first, first + count), bins int8 [count][B][D] and
 * items int8 [count][D] (bp::environment::view, bin_packing.h:65).  set
 * replaces it (a host-side apply / reset of that env between iterations);
 * it never alters the current batch the learner reads. */
int xh_trainer_get_env_state(xh_trainer *t, int first, int count, int8_t *bins,
                             int8_t *items);
int xh_trainer_set_env_state(xh_trainer *t, int first, int count,
                             const int8_t *bins, const int8_t *items);

/* ------------------------------------------------- vectorised envs ---- */
/* N bp::environment instances (bin_packing.h:46-85, generalised to B bins /
 * D dims as the trainer's) whose state stays in HBM, for a caller that brings
 * its own policy: xylo::environment<A,S>::apply / view / reset
 * (rl.h:163-170) with the id parameter ranging over the whole batch, and
 * xylo::agent::step minus the policy's react (rl.h:325-349) as ONE kernel for
 * every env.
 *
 * Buffers (device memory owned by the venv; xh_venv_device_ptr gives the
 * address for the caller's own kernels on the same device, xh_venv_get /
 * xh_venv_set copy to / from host memory):
 *   XH_VENV_ACTIONS int32 [N]        the chosen bin of every env (input)
 *   XH_VENV_REWARD  f32   [N]        agent::get_reward of the last step
 *   XH_VENV_DONE    uint8 [N]        agent::game_over after the last apply
 *   XH_VENV_BINS    int8  [N][B][D]  bins (observation::bins)
 *   XH_VENV_ITEMS   int8  [N][4]     item, D used (observation::item)
 *   XH_VENV_RNG     uint32 [N]       per-env minstd_rand0 state
 *   XH_VENV_OBS     f32   [N][B][2D] observation::to_vector (bin_packing.h:
 *                                    31-40), written by xh_venv_observe and
 *                                    by xh_venv_step(write_obs = 1)
 *   XH_VENV_MASK    uint8 [N]        env selection for apply / reset
 *
 * Engine draws: construction 2 per env, get_item 2, reset 2.
 * Env g of the job (env_offset + local index) starts on the global engine
 * stream at x0, constructed in env order, and xh_venv_step reproduces the
 * reference's draw order of a driver that steps every agent once per step in
 * env order, its policy taking `policy_draws` draws per step (2 for the
 * reference's discrete_action sampling and random_policy, 0 for a policy that
 * draws nothing): step s of env g draws at 2 Ng + k (s Ng + g), k =
 * policy_draws + 2.  xh_venv_apply / xh_venv_reset draw from the env's own
 * stream where it stands (with Ng = 1 every call sequence is exactly the
 * single-env reference engine).
 *
 * Calls are asynchronous on the context's stream; an out-of-range action
 * leaves its env untouched and is reported by the next xh_venv_synchronize
 * (or get) as XH_ERR_INVALID. */
typedef struct xh_venv xh_venv;
enum {
  XH_VENV_ACTIONS = 0, XH_VENV_REWARD = 1, XH_VENV_DONE = 2,
  XH_VENV_BINS = 3, XH_VENV_ITEMS = 4, XH_VENV_RNG = 5, XH_VENV_OBS = 6,
  XH_VENV_MASK = 7, XH_VENV_BUF_COUNT
};
int xh_venv_create(xh_ctx *ctx, int num_envs, int bins, int dims,
                   uint32_t rng_state, int env_offset, int num_envs_global,
                   int policy_draws, xh_venv **out);
int xh_venv_destroy(xh_venv *v);
size_t xh_venv_bytes(const xh_venv *v, int which);
void *xh_venv_device_ptr(xh_venv *v, int which);
int xh_venv_get(xh_venv *v, int which, void *host, size_t bytes);
int xh_venv_set(xh_venv *v, int which, const void *host, size_t bytes);
/* agent::step minus react for every env: skip the policy's draws,
 * environment::apply(ACTIONS[e]), REWARD / DONE, reset on game over;
 * write_obs != 0 also writes OBS of the resulting states. */
int xh_venv_step(xh_venv *v, int write_obs);
/* environment::apply(ACTIONS[e], e) for the envs selected by MASK (all if
 * use_mask == 0), no reset; DONE[e] = game_over after the apply, 0 for the
 * envs this call did not apply (masked out, or an out-of-range action). */
int xh_venv_apply(xh_venv *v, int use_mask);
/* environment::reset(e) for the envs selected by MASK (all if use_mask == 0). */
int xh_venv_reset(xh_venv *v, int use_mask);
/* observation::to_vector of every env into OBS. */
int xh_venv_observe(xh_venv *v);
/* Waits for the venv's work; XH_ERR_INVALID if an action was out of range. */
int xh_venv_synchronize(xh_venv *v);
/* Kernel timing: on != 0 brackets every later step / apply / reset /
 * observe launch with HIP events on the context's stream (and drops the
 * events recorded so far); xh_venv_kernel_time returns their accumulated
 * milliseconds and the launch count. */
int xh_venv_set_timing(xh_venv *v, int on);
int xh_venv_kernel_time(xh_venv *v, double *ms, long *launches);

/* ------------------------------------------------------ model::eval -- */
/* xylo::model::eval (nn.h:473-479) of a layer chain on the device: rows x
 * cols host floats in, rows x out_cols host floats out.  Layers (nn.h):
 * full_layer (60-110) and convolution1d_1_layer (113-194, the same Dense
 * over each of the cols / in points of a row), relu (350-377), softmax
 * (379-422, no max shift) and softmax_cross_entropy (424-431, forward =
 * softmax).  params: the flat model::parameters() layout (nn.h:499-508).
 * Synchronous; for host-side callers of model::eval (the drop-in layer's
 * policies on host states, evaluation tools). */
enum { XH_LAYER_FULL = 0, XH_LAYER_CONV1D_1 = 1, XH_LAYER_RELU = 2,
       XH_LAYER_SOFTMAX = 3, XH_LAYER_SOFTMAX_XENT = 4 };
typedef struct {
  int kind;
  int in, out; /* dense layers: input / output features (per point) */
} xh_layer;
int xh_model_eval(xh_ctx *ctx, const xh_layer *layers, int nlayers,
                  const float *params, size_t nparams, const float *x,
                  int rows, int cols, float *out, size_t out_cap,
                  int *out_cols);

/* ------------------------------------- layer / model / optimizer / loss -- */
/* The reference's generic training API on the device, for callers that
 * assemble their own learner from its pieces (the drop-in layer's
 * xylo::layer / model / optimizer / loss functions, include/xylo_compat).
 * Synchronous; host arrays in and out; layers and the flat parameter layout
 * as xh_model_eval.
 *
 * xh_model_forward: model::forward (nn.h:481-488) -- the input and every
 * layer's output, each rows x widths[l], concatenated into acts (widths[0] =
 * cols, widths[nlayers] = the output's).  acts_cap floats; widths has
 * nlayers + 1 entries. */
int xh_model_forward(xh_ctx *ctx, const xh_layer *layers, int nlayers,
                     const float *params, size_t nparams, const float *x,
                     int rows, int cols, float *acts, size_t acts_cap,
                     int *widths);
/* model::gradient (nn.h:510-528): `inputs` = the first nlayers matrices of
 * model::forward, concatenated as xh_model_forward writes them; target =
 * dL/d(output), rows x target_cols.  Backpropagates from the last layer
 * (layer::gradient then layer::backward per layer, layer 0 gradient only)
 * into grad[nparams] (model::parameters() layout). */
int xh_model_gradient(xh_ctx *ctx, const xh_layer *layers, int nlayers,
                      const float *params, size_t nparams, const float *inputs,
                      int rows, int cols, const float *target, int target_cols,
                      float *grad);
/* layer::backward / layer::gradient (nn.h:20-33) of one layer: input rows x
 * cols, backprop rows x bp_cols (the layer's output width).  backward ->
 * out rows x cols (full / conv1d_1: backprop . A; relu: gated by input > 0;
 * softmax: the Jacobian product; softmax_cross_entropy: backprop itself);
 * gradient -> grad[ngrad], the layer's [dA (out x in), db (out)] (ngrad = 0
 * for activations). */
int xh_layer_backward(xh_ctx *ctx, const xh_layer *layer, const float *params,
                      size_t nparams, const float *input, int rows, int cols,
                      const float *backprop, int bp_cols, float *out);
int xh_layer_gradient(xh_ctx *ctx, const xh_layer *layer, const float *input,
                      int rows, int cols, const float *backprop, int bp_cols,
                      float *grad, size_t ngrad);
/* The discrete-action loss gradients of a batch of `rows` actions over
 * `range` choices, out[rows][range] (rl.h:33-74 per row):
 *   XH_LOSS_GRADIENT_LOG          discrete_action::gradient_log
 *   XH_LOSS_SOFTMAX_GRADIENT_LOG  softmax_gradient_log = policy_loss
 *                                 (policy_gradient.h:24-34)
 *   XH_LOSS_CLIPPED               clipped_gradient = surrogate_loss
 *                                 (:36-46), param = epsilon (0.2)
 *   XH_LOSS_KL_REGULATED          the gradient of kl_regulated_loss (:55-74):
 *                                 softmax_gradient_log + param (beta) times
 *                                 (probs - distrib); the beta adaptation is
 *                                 the caller's
 * choice[rows], advantage[rows], probs = the model's output rows (the
 * reference's orig_action_matrix), distrib = each action's sampling
 * distribution [rows][range] (unused by SOFTMAX_GRADIENT_LOG, may be NULL
 * there). */
enum { XH_LOSS_GRADIENT_LOG = 0, XH_LOSS_SOFTMAX_GRADIENT_LOG = 1,
       XH_LOSS_CLIPPED = 2, XH_LOSS_KL_REGULATED = 3 };
int xh_action_loss_grad(xh_ctx *ctx, int kind, int rows, int range,
                        const int32_t *choice, const float *distrib,
                        const float *advantage, const float *probs, float param,
                        float *out);
/* optimizer::next_parameters (nn.h:616-698) of n parameters in place:
 * XH_OPT_SGD p (1 - wd) - g lr; XH_OPT_MOMENTUM v = 0.9 v + g, p - v lr (m =
 * v); XH_OPT_ADAM moments m, v, bias-corrected with step t (1, 2, ...),
 * p - m^ lr / (sqrt(v^) + 1e-7).  m / v: the caller's state arrays (NULL for
 * sgd). */
int xh_optimizer_apply(xh_ctx *ctx, int kind, float lr, float weight_decay,
                       float beta1, float beta2, float t, float *params,
                       const float *grad, float *m, float *v, size_t n);
/* replay_buffer::forget() (rl.h:274-291) after a learn() that did not run on
 * this trainer (a learner assembled from the pieces above consumed the
 * batch): the batch's final states become the next rollout's start states. */
int xh_trainer_forget(xh_trainer *t);

/* ---------------------------------------------------------- tensor ---- */
/* xylo/tensor.{h,cc} on the device, for the drop-in tensor type
 * (include/xylo_compat/xylo/tensor.h): tensors created with on_device = true
 * live in HBM (the reference's memory_blob on_device bit with its gpu_alloc /
 * gpu_dealloc stubs, tensor.cc:38-39, 78-102, made real), and their
 * arithmetic runs here; large operations on host tensors (GEMMs, long
 * reductions) stage through the device.  Every call is synchronous on the
 * context's stream.
 *
 * xh_tensor_alloc / free: n floats of device memory, zero-filled (NULL for
 * n = 0).
 * xh_tensor_copy: n floats, kind XH_COPY_H2D | XH_COPY_D2H | XH_COPY_D2D. */
enum { XH_COPY_H2D = 0, XH_COPY_D2H = 1, XH_COPY_D2D = 2 };
int xh_tensor_alloc(xh_ctx *ctx, size_t n, float **out);
int xh_tensor_free(xh_ctx *ctx, float *p);
int xh_tensor_copy(xh_ctx *ctx, float *dst, const float *src, size_t n,
                   int kind);
/* Elementwise, device arrays (tensor.cc:256-317 and the compound operators
 * :338-398): out[i] = a[i] + b[i] | a - b | a * b | a / b (XH_T_ADD ..
 * XH_T_DIVIDE); a[i] + s | a - s | a * s | a / s (XH_T_*_S); fabsf / sinf /
 * expf / logf / sqrtf of a[i]; XH_T_FILL: out[i] = s (vector::operator=(float),
 * tensor.cc:128); XH_T_RMINUS_S s - a[i] and XH_T_RDIVIDE_S s / a[i] (the
 * reference's compound v -= s and v /= s, whose bind_front puts the scalar
 * first: tensor.cc:378-380, 392-394).  out may alias a or b. */
enum { XH_T_ADD = 0, XH_T_MINUS = 1, XH_T_MULTIPLY = 2, XH_T_DIVIDE = 3,
       XH_T_ADD_S = 4, XH_T_MINUS_S = 5, XH_T_MULTIPLY_S = 6,
       XH_T_DIVIDE_S = 7, XH_T_ABS = 8, XH_T_SIN = 9, XH_T_EXP = 10,
       XH_T_LOG = 11, XH_T_SQRT = 12, XH_T_FILL = 13, XH_T_RMINUS_S = 14,
       XH_T_RDIVIDE_S = 15 };
int xh_tensor_map(xh_ctx *ctx, int op, const float *a, const float *b,
                  float scalar, float *out, size_t n);
/* Reductions over n floats (device arrays if on_device, else host arrays
 * staged for the call), accumulated in double and returned unrounded:
 * XH_R_SUM sum a (tensor.cc:434-438), XH_R_DOT sum a*b (:427-432), XH_R_SQDEV
 * sum (a - s)^2 (variance's sum about the mean s, :442-451), XH_R_MAX max a
 * (:462), XH_R_ARGMAX its first index (:464-466) in *index (may be NULL
 * otherwise).  max / argmax of n = 0 is XH_ERR_INVALID. */
enum { XH_R_SUM = 0, XH_R_DOT = 1, XH_R_SQDEV = 2, XH_R_MAX = 3,
       XH_R_ARGMAX = 4 };
int xh_tensor_reduce(xh_ctx *ctx, int op, const float *a, const float *b,
                     float scalar, size_t n, int on_device, double *value,
                     int64_t *index);
/* out[m][n] = sum_k a[m][k] b(n, k), f32 MFMA: XH_GEMM_NT b is [n][k]
 * (matmul_transposed, tensor.cc:218-227), XH_GEMM_NN b is [k][n] (matmul,
 * :228-230).  Row-major, no aliasing of out with a or b. */
enum { XH_GEMM_NT = 0, XH_GEMM_NN = 1 };
int xh_tensor_gemm(xh_ctx *ctx, int layout, const float *a, const float *b,
                   float *out, int m, int n, int k, int on_device);
/* out[cols][rows] = in[rows][cols]^T (transpose, tensor.cc:209-216). */
int xh_tensor_transpose(xh_ctx *ctx, const float *in, float *out, int rows,
                        int cols, int on_device);

/* sizeof of the ABI structs ("xh_config", "xh_eval", "xh_layer"; 0 if
 * unknown), so a
 * foreign-language binding can check its mirror of them. */
size_t xh_struct_size(const char *name);

/* Kernel timing with HIP events on the trainer's stream (off by default).
 * on = 1: every launch (the phase breakdown; the events themselves cost
 * about 2 us per launch of wall time); on = XH_TIMING_TRAIN (2): the policy
 * train launches only (the dominant kernel's average duration, nearly free). */
#define XH_TIMING_TRAIN 2
int xh_trainer_set_timing(xh_trainer *t, int on);
/* name: "rollout_step" | "policy_train" | "value" | "reduce_sgd" | "allreduce"
 * Returns accumulated milliseconds and launch count since the last reset. */
int xh_trainer_kernel_time(xh_trainer *t, const char *name, double *ms,
                           long *launches);
int xh_trainer_reset_timing(xh_trainer *t);
/* Which kernels the trainer's last rollout step and last policy epoch
 * launched, and their arithmetic, as a JSON object written NUL-terminated
 * into buf[cap]:
 *   {"rollout_step": K, "policy_train": K, "value": V, "train_grid": G,
 *    "train_grid_cap": C, "overrides": {...}}
 *   K = {"kernel": name | null (not launched yet),
 *        "math": one of
 *          "f32_mfma"             f32-input MFMA / f32 VALU: peak 157.3
 *          "bf16_split"           bf16 MFMA on exact three-part splits: 4
 *                                 products per f32 product in the train epoch
 *                                 (variant library only): peak 2500 / 4
 *          "f16_pair"             the split rollouts' layer 2 on scaled f16
 *                                 pairs, 3 products per f32 product: 2500 / 3
 *          "f16_pair_bf16_split"  the train epochs: layer 2 three f16
 *                                 products, dH1 two, dW2 three bf16 (8 per 3
 *                                 f32 products, equal FLOPs): 2500 / (8/3),
 *        "products_per_f32_product": p (null for f32_mfma),
 *        "bf16_products_per_f32_product": p for "bf16_split", else null,
 *        "peak_tflops": the dense MFMA peak of that arithmetic on MI355X
 *        (2500 / p, or 157.3)}
 *   V = "vnet_bf16" (the Fin -> 64 -> 32 -> 1 value net on exact bf16
 *   splits: two forwards and one fused backward per update, B*D % 16 == 0,
 *   B*D + D < 416), "mlp3_fused" (the same net on the f32 fused kernels:
 *   XH_VALUE_KERNEL=mlp3, or shapes the bf16 kernels do not take) or "gemm"
 *   (layer by layer: other widths, XH_VALUE_KERNEL=gemm),
 *   G = the train grid (workgroups, = gradient slabs), C = xh_config
 *   train_grid_cap.
 * "overrides" lists the diagnostic environment variables that steer kernel
 * selection (XH_TRAIN_KERNEL, XH_ROLLOUT_KERNEL, XH_VALUE_KERNEL) with their
 * values, or null when unset. */
int xh_trainer_kernel_info(xh_trainer *t, char *buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* XYLO_HIP_H_ */
