/* oracle/asan_driver.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Drives every entry point of the C restatement (oracle.c) at small sizes so
 * that an AddressSanitizer + UndefinedBehaviorSanitizer build of it
 * (`make -C oracle asan`, SURVEY §5 "race / memory checking") runs its
 * pointer-heavy parts: the replay-buffer trajectory lists and their
 * forget() re-linking, the end-row state matrix, the per-env streams, the
 * model gradient buffers and the optimizer state.  Exit status 0 and a final
 * "asan driver ok" line; any sanitizer report aborts (halt_on_error). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static float *randn(size_t n, uint32_t *x, float scale) {
  float *p = (float *)malloc(sizeof(float) * (n ? n : 1));
  for (size_t i = 0; i < n; ++i)
    p[i] = (float)((or_canonical(x) - 0.5) * 2.0 * scale);
  return p;
}

static void perbin(or_model *m, int f0, int h1, int h2, int head) {
  int k = 0;
  m->type[k] = OR_POINT, m->in[k] = f0, m->out[k++] = h1;
  m->type[k] = OR_RELU, m->in[k] = 0, m->out[k++] = 0;
  m->type[k] = OR_POINT, m->in[k] = h1, m->out[k++] = h2;
  m->type[k] = OR_RELU, m->in[k] = 0, m->out[k++] = 0;
  m->type[k] = OR_POINT, m->in[k] = h2, m->out[k++] = 1;
  m->type[k] = head, m->in[k] = 0, m->out[k++] = 0;
  m->nl = k;
}

static void full(or_model *m, int in, int h1, int h2, int out, int head) {
  int k = 0;
  m->type[k] = OR_FULL, m->in[k] = in, m->out[k++] = h1;
  m->type[k] = OR_RELU, m->in[k] = 0, m->out[k++] = 0;
  if (h2) {
    m->type[k] = OR_FULL, m->in[k] = h1, m->out[k++] = h2;
    m->type[k] = OR_RELU, m->in[k] = 0, m->out[k++] = 0;
  }
  m->type[k] = OR_FULL, m->in[k] = h2 ? h2 : h1, m->out[k++] = out;
  if (head >= 0) m->type[k] = head, m->in[k] = 0, m->out[k++] = 0;
  m->nl = k;
}

static double checksum(const or_trainer *t, int which) {
  size_t n = 0;
  const void *p = or_trainer_buf(t, which, &n);
  double s = 0;
  for (size_t i = 0; i < n; ++i) s += ((const float *)p)[i];
  return s;
}

/* PPO / AC / KL-PPO: rollout + learn iterations, the optimizers, options */
static void run_actor_critic(int algo, int B, int D, int N, int T, int iters,
                             int opt) {
  uint32_t x = 777u + (uint32_t)algo;
  or_env_cfg env;
  or_env_default(&env, B, D);
  or_model pol, val;
  memset(&pol, 0, sizeof pol);
  memset(&val, 0, sizeof val);
  perbin(&pol, 2 * D, 16, 8, algo == OR_AC ? OR_SOFTMAX_XENT : OR_SOFTMAX);
  full(&val, B * 2 * D, 16, 8, 1, -1);
  float *pp = randn(or_model_nparams(&pol), &x, 0.3f);
  float *vp = randn(or_model_nparams(&val), &x, 0.05f);
  or_trainer *t = or_trainer_create(algo, &env, N, T, 1, &pol, pp, &val, vp,
                                    1e-3f, 1e-3f, 0.0f, 0.0f, 0.99f, 4242u);
  if (opt) {
    or_trainer_set_optimizer(t, 0, opt, 1e-3f, 0.0f, 0.9f, 0.999f);
    or_trainer_set_optimizer(t, 1, opt, 1e-3f, 0.0f, 0.9f, 0.999f);
  }
  if (algo != OR_KLPPO) or_trainer_set_options(t, opt == OR_OPT_SGD, 0);
  int32_t *forced = (int32_t *)malloc(sizeof(int32_t) * N * T);
  for (int i = 0; i < N * T; ++i) forced[i] = (i * 7) % B;
  for (int it = 0; it < iters; ++it) {
    or_trainer_rollout(t, it == 1 ? forced : NULL);
    or_trainer_learn(t);
  }
  if (algo == OR_PPO) { /* explicit streams, as the full-size sample check */
    uint32_t *xs = (uint32_t *)malloc(sizeof(uint32_t) * N);
    for (int i = 0; i < N; ++i) xs[i] = or_minstd_jump(4242u, 1000u + 16u * i);
    or_trainer_set_stream_states(t, xs);
    free(xs);
    or_trainer_rollout(t, NULL);
    or_trainer_learn(t);
  }
  printf("algo %d B%d D%d N%d T%d: policy grads %.6g, adv %.6g\n", algo, B, D,
         N, T, checksum(t, OR_BUF_POLICY_GRADS), checksum(t, OR_BUF_ADVANTAGES));
  or_trainer_destroy(t);
  free(forced);
  free(pp);
  free(vp);
}

static void run_reinforce(void) {
  uint32_t x = 99u;
  or_env_cfg env;
  or_env_default(&env, 8, 1);
  or_model pol;
  memset(&pol, 0, sizeof pol);
  full(&pol, 8 * 2, 32, 0, 8, OR_SOFTMAX_XENT);
  float *pp = randn(or_model_nparams(&pol), &x, 0.01f);
  or_trainer *t = or_trainer_create(OR_PG, &env, 4, 1, 2, &pol, pp, NULL, NULL,
                                    1e-3f, 0.0f, 0.0f, 0.0f, 0.99f, 5u);
  or_trainer_set_env_streams(t, 1ull << 26, 1);
  for (int it = 0; it < 3; ++it) {
    or_trainer_rollout(t, NULL);
    or_trainer_learn(t);
  }
  or_trainer_set_env_streams(t, 1ull << 26, 0);
  or_trainer_rollout(t, NULL);
  or_trainer_learn(t);
  printf("reinforce: policy grads %.6g\n", checksum(t, OR_BUF_POLICY_GRADS));
  or_trainer_destroy(t);
  free(pp);
}

int main(void) {
  /* RNG and the libstdc++ distributions */
  uint32_t x = or_minstd_seed(0);
  float p[5] = {0.1f, 0.2f, 0.3f, 0.15f, 0.25f};
  int hist[5] = {0};
  for (int i = 0; i < 1000; ++i) hist[or_discrete(&x, p, 5)]++;
  (void)or_bernoulli(&x, 0.4);
  if (or_minstd_jump(1u, 3u) != (uint32_t)(16807ull * 16807ull % 2147483647ull * 16807ull % 2147483647ull))
    return 2;
  /* env + the vectorised driver */
  or_env_cfg env;
  or_env_default(&env, 16, 3);
  int32_t bins[16 * 3], item[3];
  or_env_construct(&env, bins, item, &x);
  for (int s = 0; s < 40; ++s) {
    if (or_env_apply(&env, bins, item, s % 16, &x) || or_env_game_over(&env, bins))
      or_env_reset(&env, bins, item, &x);
  }
  float obs[16 * 6];
  or_obs(&env, bins, item, obs);
  {
    const int N = 6, S = 9;
    int32_t *acts = (int32_t *)malloc(sizeof(int32_t) * N * S);
    for (int i = 0; i < N * S; ++i) acts[i] = (i * 5) % 16;
    int32_t *vb = (int32_t *)malloc(sizeof(int32_t) * (S + 1) * N * 16 * 3);
    int32_t *vi = (int32_t *)malloc(sizeof(int32_t) * (S + 1) * N * 3);
    float *rw = (float *)malloc(sizeof(float) * S * N);
    uint8_t *dn = (uint8_t *)malloc(S * N);
    (void)or_venv_run(&env, N, 3 * N, N, 2, 11u, S, acts, vb, vi, rw, dn);
    free(acts), free(vb), free(vi), free(rw), free(dn);
  }
  /* model eval / gradient with magnitudes, optimizers */
  {
    or_model m;
    memset(&m, 0, sizeof m);
    perbin(&m, 6, 12, 10, OR_SOFTMAX);
    const size_t np = or_model_nparams(&m);
    float *w = randn(np, &x, 0.3f);
    float *in = randn(5 * 16 * 6, &x, 1.0f);
    float *out = (float *)malloc(sizeof(float) * 5 * 16);
    (void)or_model_eval(&m, w, in, 5, 16 * 6, out);
    int32_t ch[5] = {1, 2, 3, 4, 5};
    float po[5] = {0.1f, 0.2f, 0.05f, 0.3f, 0.07f};
    float adv[5] = {1.0f, -0.5f, 0.25f, 2.0f, -1.0f};
    float *g = (float *)calloc(np, sizeof(float));
    float *mg = (float *)calloc(np, sizeof(float));
    or_policy_grad_rows_mag(&m, w, in, 5, 16 * 6, ch, po, adv, OR_PPO, g, mg);
    or_policy_grad_rows(&m, w, in, 5, 16 * 6, ch, po, adv, OR_AC, g);
    for (int k = OR_OPT_SGD; k <= OR_OPT_ADAM; ++k) {
      or_opt o = {k, 1e-3f, 0.0f, 0.9f, 0.999f, 1.0f, NULL, NULL};
      or_opt_step(&o, w, g, np);
      or_opt_step(&o, w, g, np);
      or_opt_free(&o);
    }
    or_model vm;
    memset(&vm, 0, sizeof vm);
    full(&vm, 16 * 6, 8, 4, 1, -1);
    float *vw = randn(or_model_nparams(&vm), &x, 0.05f);
    float tg[5] = {1, 2, 3, 4, 5};
    float *vg = (float *)calloc(or_model_nparams(&vm), sizeof(float));
    float *vmg = (float *)calloc(or_model_nparams(&vm), sizeof(float));
    or_value_grad_rows_mag(&vm, vw, in, 5, 16 * 6, tg, vg, vmg);
    or_value_grad_rows(&vm, vw, in, 5, 16 * 6, tg, vg);
    uint32_t ex = 3u;
    (void)or_eval_argmax(&env, &m, w, 3, &ex);
    free(w), free(in), free(out), free(g), free(mg), free(vw), free(vg),
        free(vmg);
  }
  /* heuristic agents */
  for (int k = OR_HEUR_RANDOM; k <= OR_HEUR_MINWASTE; ++k) {
    or_env_cfg e8;
    or_env_default(&e8, 8, 2);
    uint32_t hx = 17u;
    int32_t lens[5];
    (void)or_heuristic_eval(&e8, k, 5, &hx, lens);
  }
  /* the learners, pointer-heavy replay buffers */
  run_actor_critic(OR_PPO, 8, 2, 5, 6, 4, OR_OPT_SGD);
  run_actor_critic(OR_AC, 16, 3, 4, 5, 3, OR_OPT_MOMENTUM);
  run_actor_critic(OR_KLPPO, 8, 1, 6, 4, 4, OR_OPT_ADAM);
  run_reinforce();
  printf("asan driver ok\n");
  return 0;
}
