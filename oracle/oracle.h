/* oracle/oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference (beehover/dependence_free_rl @
 * 2024_10_08) PPO / actor-critic / REINFORCE rollout-and-update path, used as
 * the CHECKER for the HIP implementation.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load liboracle.so.  The product path
 * (dependence_free_rl_amd/) never links or calls it.
 *
 * Parity pinning: tests/test_oracle_golden.py checks this restatement against
 * golden vectors produced by the real reference (oracle/_ref, built from
 * /root/reference by oracle/Makefile; generator tests/golden/make_golden.py):
 * RNG streams and env trajectories bit-exact, Dense/learner outputs within
 * 1e-4 * max(1, |y|).
 *
 * Third-party arithmetic restated here: libstdc++ 11 (GCC 11.4 headers)
 *   std::minstd_rand0                bits/random.h:1555
 *   std::generate_canonical<double>  bits/random.tcc:3348-3380
 *   std::bernoulli_distribution      bits/random.h:3633-3643
 *   std::discrete_distribution       bits/random.tcc:2654-2713
 */
#ifndef XH_ORACLE_H_
#define XH_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ RNG -- */
uint32_t or_minstd_seed(uint64_t s);
uint32_t or_minstd_next(uint32_t *x);
uint32_t or_minstd_jump(uint32_t x, uint64_t k);
double or_canonical(uint32_t *x);
int or_bernoulli(uint32_t *x, double p);
int or_discrete(uint32_t *x, const float *p, int n);
int or_argmax(const float *v, int n);

/* ------------------------------------------------------------------ env -- */
typedef struct {
  int B, D, cap;
  int item_a[3], item_b[3];
  double p_a;
} or_env_cfg;

void or_env_default(or_env_cfg *c, int B, int D);
void or_env_construct(const or_env_cfg *c, int32_t *bins, int32_t *item,
                      uint32_t *x);
int or_env_apply(const or_env_cfg *c, int32_t *bins, int32_t *item, int choice,
                 uint32_t *x);
void or_env_reset(const or_env_cfg *c, int32_t *bins, int32_t *item,
                  uint32_t *x);
int or_env_game_over(const or_env_cfg *c, const int32_t *bins);
void or_obs(const or_env_cfg *c, const int32_t *bins, const int32_t *item,
            float *out);

/* Sequential reference-order driver of Ng agents stepped once per step in
 * env order (see oracle.c); the checker of the vectorised env (xh_venv). */
uint32_t or_venv_run(const or_env_cfg *c, int N, int Ng, int off, int pd,
                     uint32_t x0, int S, const int32_t *actions, int32_t *bins,
                     int32_t *item, float *reward, uint8_t *done);

/* ---------------------------------------------------------------- model -- */
enum { OR_FULL = 0, OR_POINT = 1, OR_RELU = 2, OR_SOFTMAX = 3,
       OR_SOFTMAX_XENT = 4 };
#define OR_MAX_LAYERS 16
typedef struct {
  int nl;
  int type[OR_MAX_LAYERS];
  int in[OR_MAX_LAYERS];  /* dense: input features / channels */
  int out[OR_MAX_LAYERS]; /* dense: output features / channels */
} or_model;

size_t or_model_nparams(const or_model *m);
/* x: rows x xcols; out: rows x (output cols). Returns output cols. */
int or_model_eval(const or_model *m, const float *params, const float *x,
                  int rows, int xcols, float *out);
/* forward + reference gradient (nn.h:510-528) with the given loss gradient
 * function applied to the model output. */
typedef void (*or_loss_fn)(void *ctx, const float *out, int rows, int cols,
                           float *target);
void or_model_grad(const or_model *m, const float *params, const float *x,
                   int rows, int xcols, or_loss_fn loss, void *ctx,
                   float *grad);
void or_model_grad_mag(const or_model *m, const float *params, const float *x,
                       int rows, int xcols, or_loss_fn loss, void *ctx,
                       float *grad, float *grad_mag);
void or_sgd(float *params, const float *grad, size_t n, float lr, float wd);
/* sgd / momentum / adam optimizers (nn.h:616-698) with their state. */
enum { OR_OPT_SGD = 0, OR_OPT_MOMENTUM = 1, OR_OPT_ADAM = 2 };
typedef struct {
  int kind;
  float lr, wd, b1, b2, t;
  float *m, *v; /* velocity / first, second moment (NULL until first step) */
} or_opt;
void or_opt_step(or_opt *o, float *params, const float *grad, size_t n);
void or_opt_free(or_opt *o);

/* --------------------------------------------------------------- learner -- */
enum { OR_PPO = 0, OR_AC = 1, OR_PG = 2, OR_KLPPO = 3 };

typedef struct or_trainer or_trainer;

or_trainer *or_trainer_create(int algo, const or_env_cfg *env, int N, int T,
                              int episodes, const or_model *pol,
                              const float *pol_params, const or_model *val,
                              const float *val_params, float lr_pi, float lr_v,
                              float wd_pi, float wd_v, float gamma,
                              uint32_t x0);
void or_trainer_destroy(or_trainer *t);
/* Replace the policy (which = 0) or value (1) optimizer; its state restarts. */
void or_trainer_set_optimizer(or_trainer *t, int which, int kind, float lr,
                              float wd, float beta1, float beta2);
/* Rollout of one iteration: workers stepped one after another. If `forced`
 * is non-NULL it supplies the actions (env-major, T per env; the sampler's 2
 * engine draws are still consumed). */
void or_trainer_rollout(or_trainer *t, const int32_t *forced);
void or_trainer_learn(or_trainer *t); /* learn() + replay_buffer.forget() */
/* Opt-in options of the device trainer (xh_config.adv_normalize /
 * lr_scale_rows; not in the reference): advantage normalisation over the
 * transition rows, and lr / (T * N) for both optimizers.  AC / PPO only. */
void or_trainer_set_options(or_trainer *t, int adv_normalize,
                            int lr_scale_rows);
uint32_t or_trainer_rng(const or_trainer *t);
/* Per-env streams: env i draws from x0 advanced by i * stride (env 0 = the
 * single-env reference run), re-constructing the envs on those streams; or,
 * with reconstruct = 0, keeps the envs (constructed in worker order on the
 * shared engine) and starts env i's stream at the engine state advanced by
 * i * stride (the drop-in layer's REINFORCE windows). */
void or_trainer_set_env_streams(or_trainer *t, uint64_t stride,
                                int reconstruct);
const uint32_t *or_trainer_env_streams(const or_trainer *t);
/* Explicit per-env stream states xs[N] (envs kept), from the next rollout. */
void or_trainer_set_stream_states(or_trainer *t, const uint32_t *xs);
void or_trainer_get_params(const or_trainer *t, int which, float *out);
void or_trainer_set_params(or_trainer *t, int which, const float *in);
/* Introspection of the last rollout / learn (valid until the next call). */
enum {
  OR_BUF_STEP_BINS = 0, /* int32  [steps][B][D]   state before each apply  */
  OR_BUF_STEP_ITEM,     /* int32  [steps][D]                               */
  OR_BUF_STEP_CHOICE,   /* int32  [steps]                                  */
  OR_BUF_STEP_DONE,     /* int32  [steps]                                  */
  OR_BUF_STEP_PCHOICE,  /* float  [steps]  distrib[choice] (old prob)      */
  OR_BUF_ROWS,          /* float  [rows][S::length()]                      */
  OR_BUF_ROW_ENV,       /* int32  [rows]                                   */
  OR_BUF_ROW_STEP,      /* int32  [rows]  env apply-count at view time     */
  OR_BUF_ROW_IS_END,    /* int32  [rows]                                   */
  OR_BUF_VALUES,        /* float  [rows]  V before the value step          */
  OR_BUF_TARGETS,       /* float  [rows]                                   */
  OR_BUF_VALUE_GRAD,    /* float  [value params]                           */
  OR_BUF_ADVANTAGES,    /* float  [rows]                                   */
  OR_BUF_POLICY_GRADS,  /* float  [epochs][policy params]                  */
  OR_BUF_FINAL_BINS,    /* int32  [N][B][D]  env states after the rollout   */
  OR_BUF_FINAL_ITEM,    /* int32  [N][D]                                   */
  OR_BUF_ROW_CHOICE,    /* int32  [rows]  action of the row                */
  OR_BUF_ROW_POLD,      /* float  [rows]  distrib[choice] of the row       */
  OR_BUF_KL,            /* float  [epochs][3] KL-PPO: beta used, mean KL,
                                              beta after                   */
  OR_BUF_POLICY_GRADS_MAG, /* float [epochs][policy params]: per entry, the
                              sum of |terms| of its row sums (rounding
                              scale, or_model_grad_mag) -- AC / PPO / KL   */
  OR_BUF_VALUE_GRAD_MAG,   /* float [value params]: the same              */
  OR_BUF_COUNT
};
/* Returns a pointer to the buffer and its element count. */
const void *or_trainer_buf(const or_trainer *t, int which, size_t *count);

/* Gradient of one loss over an explicit set of rows (any subset of a learn()
 * batch): the building block of the sharded (multi-rank) check.  algo selects
 * the loss as in or_trainer_learn (PPO surrogate / AC and PG softmax-log). */
void or_policy_grad_rows(const or_model *m, const float *params, const float *x,
                         int rows, int xcols, const int32_t *choice,
                         const float *pold, const float *adv, int algo,
                         float *grad);
void or_value_grad_rows(const or_model *m, const float *params, const float *x,
                        int rows, int xcols, const float *targets, float *grad);
/* The same two with, per gradient entry, the sum of |terms| of its row sums
 * (the rounding scale of or_model_grad_mag). */
void or_policy_grad_rows_mag(const or_model *m, const float *params,
                             const float *x, int rows, int xcols,
                             const int32_t *choice, const float *pold,
                             const float *adv, int algo, float *grad,
                             float *mag);
void or_value_grad_rows_mag(const or_model *m, const float *params,
                            const float *x, int rows, int xcols,
                            const float *targets, float *grad, float *mag);

/* Deterministic (argmax) evaluation, deep_agent.cc:25-41: `episodes` episodes
 * on one env seeded at x0; returns total reward, engine state via *x. */
double or_eval_argmax(const or_env_cfg *env, const or_model *pol,
                      const float *params, long episodes, uint32_t *x);

/* Heuristic agents (firstfit / bestfit / minwaste / random), one env seeded
 * at *x: total reward; per-episode lengths into lens (may be NULL). */
enum { OR_HEUR_RANDOM = 0, OR_HEUR_FIRSTFIT = 1, OR_HEUR_BESTFIT = 2,
       OR_HEUR_MINWASTE = 3 };
double or_heuristic_eval(const or_env_cfg *env, int kind, long episodes,
                         uint32_t *x, int32_t *lens);

#ifdef __cplusplus
}
#endif
#endif
