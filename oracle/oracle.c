/* oracle/oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the
 * reference rollout-and-update path (see oracle.h for scope and pinning).
 *
 * Each function cites the reference (file:line under /root/reference) or the
 * libstdc++ 11 algorithm it restates.  The loop structure deliberately follows
 * the reference (row-by-row dot products, full-Jacobian softmax backward,
 * O(T^2) GAE) so that its timing stays representative of the reference CPU
 * path; it is built without -ffast-math so its results are reproducible.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define OR_M 2147483647u  /* minstd modulus */
#define OR_A 16807u       /* minstd_rand0 multiplier */

/* ------------------------------------------------------------------ RNG -- */
/* linear_congruential_engine<uint_fast32_t,16807,0,2147483647>::seed:
 * s mod m, 0 -> 1 (libstdc++ bits/random.tcc) */
uint32_t or_minstd_seed(uint64_t s) {
  uint32_t x = (uint32_t)(s % OR_M);
  return x == 0 ? 1u : x;
}

uint32_t or_minstd_next(uint32_t *x) {
  *x = (uint32_t)(((uint64_t)*x * OR_A) % OR_M);
  return *x;
}

/* x * a^k mod m (jump-ahead by k draws). */
uint32_t or_minstd_jump(uint32_t x, uint64_t k) {
  uint64_t acc = 1, base = OR_A;
  while (k) {
    if (k & 1) acc = acc * base % OR_M;
    base = base * base % OR_M;
    k >>= 1;
  }
  return (uint32_t)((uint64_t)x * acc % OR_M);
}

/* std::generate_canonical<double,53>(minstd_rand0): R = max-min+1 =
 * 2147483646, log2r = 30 -> m = 2 engine calls (random.tcc:3348-3380). */
double or_canonical(uint32_t *x) {
  const long double r = 2147483646.0L;
  double sum = 0.0, tmp = 1.0;
  for (int k = 2; k != 0; --k) {
    sum += (double)(or_minstd_next(x) - 1u) * tmp;
    tmp = (double)(tmp * r);
  }
  double ret = sum / tmp;
  if (ret >= 1.0) ret = nextafter(1.0, 0.0);
  return ret;
}

/* bernoulli_distribution::operator() (random.h:3633-3643): u < p */
int or_bernoulli(uint32_t *x, double p) { return or_canonical(x) < p; }

/* ::discrete_distribution (xylo/tensor.cc:467-470) ->
 * std::discrete_distribution<size_t>{p.begin(), p.end()}(g):
 * param init random.tcc:2654-2677, sample random.tcc:2697-2713. */
int or_discrete(uint32_t *x, const float *p, int n) {
  if (n < 2) return 0; /* _M_prob cleared; operator() returns 0, no draw */
  double sum = 0.0;
  for (int i = 0; i < n; ++i) sum += (double)p[i];
  double *cp = (double *)malloc(sizeof(double) * (size_t)n);
  double acc = 0.0;
  for (int i = 0; i < n; ++i) {
    double q = (double)p[i] / sum;
    acc = i == 0 ? q : acc + q;
    cp[i] = acc;
  }
  cp[n - 1] = 1.0;
  double u = or_canonical(x);
  int lo = 0, hi = n; /* lower_bound: first i with !(cp[i] < u) */
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (cp[mid] < u)
      lo = mid + 1;
    else
      hi = mid;
  }
  free(cp);
  return lo;
}

/* std::ranges::max_element: first maximum (tensor.cc:464-466) */
int or_argmax(const float *v, int n) {
  int best = 0;
  for (int i = 1; i < n; ++i)
    if (v[best] < v[i]) best = i;
  return best;
}

/* ------------------------------------------------------------------ env -- */
/* Reference (D=2): capacity (8,8) bin_packing.h:48, items (4,2)/(1,2)
 * :73-74, P((4,2)) = 0.4 :50.  Generalised to D dims (build-defined tables:
 * D=1 (4)/(1), D=3 (4,2,2)/(1,2,1)); reduces exactly to the reference at D=2. */
void or_env_default(or_env_cfg *c, int B, int D) {
  static const int a[3][3] = {{4, 0, 0}, {4, 2, 0}, {4, 2, 2}};
  static const int b[3][3] = {{1, 0, 0}, {1, 2, 0}, {1, 2, 1}};
  memset(c, 0, sizeof(*c));
  c->B = B;
  c->D = D;
  c->cap = 8;
  for (int d = 0; d < 3; ++d) {
    c->item_a[d] = a[D - 1][d];
    c->item_b[d] = b[D - 1][d];
  }
  c->p_a = 0.4;
}

/* get_item, bin_packing.h:76-81 */
static void env_get_item(const or_env_cfg *c, int32_t *item, uint32_t *x) {
  int first = or_bernoulli(x, c->p_a);
  for (int d = 0; d < c->D; ++d) item[d] = first ? c->item_a[d] : c->item_b[d];
}

/* environment(): bins at capacity, draw an item (bin_packing.h:50-52) */
void or_env_construct(const or_env_cfg *c, int32_t *bins, int32_t *item,
                      uint32_t *x) {
  for (int i = 0; i < c->B * c->D; ++i) bins[i] = c->cap;
  env_get_item(c, item, x);
}

/* apply, bin_packing.h:53-64: subtract; overflow -> no new item */
int or_env_apply(const or_env_cfg *c, int32_t *bins, int32_t *item, int choice,
                 uint32_t *x) {
  int32_t *bin = bins + choice * c->D;
  int neg = 0;
  for (int d = 0; d < c->D; ++d) {
    bin[d] -= item[d];
    neg |= bin[d] < 0;
  }
  if (neg) return 1;
  env_get_item(c, item, x);
  return 0;
}

/* reset, bin_packing.h:67-70 */
void or_env_reset(const or_env_cfg *c, int32_t *bins, int32_t *item,
                  uint32_t *x) {
  or_env_construct(c, bins, item, x);
}

/* agent::game_over, bin_packing.h:94-101 */
int or_env_game_over(const or_env_cfg *c, const int32_t *bins) {
  for (int i = 0; i < c->B * c->D; ++i)
    if (bins[i] < 0) return 1;
  return 0;
}

/* observation::to_vector, bin_packing.h:31-40 (per bin [bin/cap, item/cap]) */
void or_obs(const or_env_cfg *c, const int32_t *bins, const int32_t *item,
            float *out) {
  const int D = c->D;
  for (int i = 0; i < c->B; ++i)
    for (int d = 0; d < D; ++d) {
      out[i * 2 * D + d] = (float)bins[i * D + d] / (float)c->cap;
      out[i * 2 * D + D + d] = (float)item[d] / (float)c->cap;
    }
}

/* A driver that steps Ng agents once per step in env order on ONE global
 * engine (the sequential form of xylo::agent::step, rl.h:325-349, with a
 * policy that draws `pd` engine values per react, e.g. 2 for
 * discrete_action::from_vector, rl.h:27-30): construct env 0..Ng-1
 * (bin_packing.h:50-52), then for each of S steps and each env: pd draws,
 * apply(actions[s][g]), reward = game_over ? 0 : 1, reset on game over.
 * Only envs [off, off + N) are recorded (actions given for those; the
 * others' draws are consumed as a step of theirs would: pd + 2).
 * Outputs: bins [S+1][N][B][D] and item [S+1][N][D] (state before step s,
 * slot S = after the last), reward / done [S][N]; returns the engine state. */
uint32_t or_venv_run(const or_env_cfg *c, int N, int Ng, int off, int pd,
                     uint32_t x0, int S, const int32_t *actions, int32_t *bins,
                     int32_t *item, float *reward, uint8_t *done) {
  const int BD = c->B * c->D, D = c->D;
  uint32_t x = x0;
  int32_t *b = (int32_t *)malloc(sizeof(int32_t) * (size_t)N * BD);
  int32_t *it = (int32_t *)calloc((size_t)N * 3, sizeof(int32_t));
  int32_t *scratch_b = (int32_t *)malloc(sizeof(int32_t) * BD);
  int32_t scratch_i[3];
  for (int g = 0; g < Ng; ++g) {
    const int local = g >= off && g < off + N;
    or_env_construct(c, local ? b + (size_t)(g - off) * BD : scratch_b,
                     local ? it + (size_t)(g - off) * 3 : scratch_i, &x);
  }
  for (int s = 0; s <= S; ++s) {
    for (int e = 0; e < N; ++e) {
      memcpy(bins + ((size_t)s * N + e) * BD, b + (size_t)e * BD,
             sizeof(int32_t) * BD);
      memcpy(item + ((size_t)s * N + e) * D, it + (size_t)e * 3,
             sizeof(int32_t) * D);
    }
    if (s == S) break;
    for (int g = 0; g < Ng; ++g) {
      const int local = g >= off && g < off + N;
      for (int k = 0; k < pd; ++k) (void)or_minstd_next(&x);
      if (!local) {
        (void)or_minstd_next(&x);
        (void)or_minstd_next(&x);
        continue;
      }
      const int e = g - off;
      int32_t *eb = b + (size_t)e * BD, *ei = it + (size_t)e * 3;
      or_env_apply(c, eb, ei, actions[(size_t)s * N + e], &x);
      const int over = or_env_game_over(c, eb);
      reward[(size_t)s * N + e] = over ? 0.0f : 1.0f;
      done[(size_t)s * N + e] = (uint8_t)over;
      if (over) or_env_reset(c, eb, ei, &x);
    }
  }
  free(b);
  free(it);
  free(scratch_b);
  return x;
}

/* ---------------------------------------------------------------- model -- */
static int is_dense(int type) { return type == OR_FULL || type == OR_POINT; }

static size_t layer_nparams(const or_model *m, int l) {
  return is_dense(m->type[l]) ? (size_t)m->in[l] * m->out[l] + m->out[l] : 0;
}

/* model::parameters layout (nn.h:499-508, 56-67): per dense layer
 * [A(out x in) row-major, b(out)], activations contribute nothing. */
size_t or_model_nparams(const or_model *m) {
  size_t n = 0;
  for (int l = 0; l < m->nl; ++l) n += layer_nparams(m, l);
  return n;
}

static int layer_out_cols(const or_model *m, int l, int in_cols) {
  switch (m->type[l]) {
    case OR_FULL:
      return m->out[l];
    case OR_POINT:
      return in_cols / m->in[l] * m->out[l];
    default:
      return in_cols;
  }
}

/* Dot products and row sums are accumulated in double and rounded once: the
 * checker is (almost) correctly rounded per reduction, so the reference's and
 * the GPU's fp32 summation orders are both compared against the same accurate
 * value (their own orders differ from each other anyway). */
static float dotf(const float *a, const float *b, int n) {
  double s = 0.0;
  for (int k = 0; k < n; ++k) s += (double)a[k] * (double)b[k];
  return (float)s;
}

/* Dense forward: matmul_transposed(X, A) + b (nn.h:72-79; conv1d_1 nn.h:127-147
 * reshapes to one point per row). X: M x in; Y: M x out. */
static void dense_fwd(const float *A, const float *b, int in, int out,
                      const float *X, size_t M, float *Y) {
  for (size_t r = 0; r < M; ++r)
    for (int o = 0; o < out; ++o) {
      float v = dotf(X + r * in, A + (size_t)o * in, in);
      Y[r * out + o] = v + b[o];
    }
}

/* softmax_layer::forward (nn.h:382-392): exp / sum, no max subtraction */
static void softmax_row(const float *z, int n, float *y) {
  double s = 0.0;
  for (int j = 0; j < n; ++j) {
    y[j] = expf(z[j]);
  }
  for (int j = 0; j < n; ++j) s += y[j];
  const float sf = (float)s;
  for (int j = 0; j < n; ++j) y[j] = y[j] / sf;
}

static void layer_forward(const or_model *m, int l, const float *p,
                          const float *X, int rows, int in_cols, float *Y) {
  const int oc = layer_out_cols(m, l, in_cols);
  switch (m->type[l]) {
    case OR_FULL:
      dense_fwd(p, p + (size_t)m->in[l] * m->out[l], m->in[l], m->out[l], X,
                (size_t)rows, Y);
      break;
    case OR_POINT:
      dense_fwd(p, p + (size_t)m->in[l] * m->out[l], m->in[l], m->out[l], X,
                (size_t)rows * (in_cols / m->in[l]), Y);
      break;
    case OR_RELU: /* nn.h:354-363 */
      for (size_t i = 0; i < (size_t)rows * in_cols; ++i)
        Y[i] = X[i] > 0 ? X[i] : 0;
      break;
    default: /* softmax / softmax-xent */
      for (int r = 0; r < rows; ++r)
        softmax_row(X + (size_t)r * in_cols, in_cols, Y + (size_t)r * oc);
  }
}

/* model::eval (nn.h:473-479) */
int or_model_eval(const or_model *m, const float *params, const float *x,
                  int rows, int xcols, float *out) {
  const float *cur = x;
  float *buf = NULL;
  int cols = xcols;
  const float *p = params;
  for (int l = 0; l < m->nl; ++l) {
    int oc = layer_out_cols(m, l, cols);
    float *y = (float *)malloc(sizeof(float) * (size_t)rows * oc);
    layer_forward(m, l, p, cur, rows, cols, y);
    p += layer_nparams(m, l);
    free(buf);
    buf = y;
    cur = y;
    cols = oc;
  }
  memcpy(out, cur, sizeof(float) * (size_t)rows * cols);
  free(buf);
  return cols;
}

/* matmul_layer::gradient (nn.h:85-100): dA = bp^T X, db = sum_r bp[r].
 * matmul_layer::backward (nn.h:81-83): dX = bp A. */
static void dense_grad(const float *A, int in, int out, const float *X,
                       const float *bp, size_t M, float *g, float *dX) {
  /* row-major sweeps with double accumulators (the sums of nn.h:94-98 in
   * row order; each entry rounded to float once) */
  float *dA = g, *db = g + (size_t)in * out;
  double *acc = (double *)calloc((size_t)in * out + out, sizeof(double));
  double *accb = acc + (size_t)in * out;
  for (size_t r = 0; r < M; ++r) {
    const float *br = bp + r * out, *xr = X + r * in;
    for (int o = 0; o < out; ++o) {
      const double b = br[o];
      double *ao = acc + (size_t)o * in;
      for (int k = 0; k < in; ++k) ao[k] += b * (double)xr[k];
      accb[o] += b;
    }
  }
  for (size_t i = 0; i < (size_t)in * out; ++i) dA[i] = (float)acc[i];
  for (int o = 0; o < out; ++o) db[o] = (float)accb[o];
  free(acc);
  if (dX) {
    double *row = (double *)malloc(sizeof(double) * in);
    for (size_t r = 0; r < M; ++r) {
      for (int k = 0; k < in; ++k) row[k] = 0.0;
      const float *br = bp + r * out;
      for (int o = 0; o < out; ++o) {
        const double b = br[o];
        const float *ao = A + (size_t)o * in;
        for (int k = 0; k < in; ++k) row[k] += b * (double)ao[k];
      }
      for (int k = 0; k < in; ++k) dX[r * in + k] = (float)row[k];
    }
    free(row);
  }
}

/* softmax_layer::backward (nn.h:393-417): recompute s, J = diag(s) - s s^T,
 * out = J g (full Jacobian, as the reference does). */
static void softmax_bwd_row(const float *z, const float *g, int n, float *out,
                            float *s, float *pd) {
  softmax_row(z, n, s);
  for (int j = 0; j < n; ++j)
    for (int k = 0; k < n; ++k) {
      float lin = (j == k) ? s[j] : 0.0f;
      pd[j * n + k] = lin - s[j] * s[k];
    }
  for (int j = 0; j < n; ++j) out[j] = dotf(pd + (size_t)j * n, g, n);
}

/* Magnitude pass of one dense layer: the same sums over |terms| (the
 * fp32-rounding scale of each gradient entry and of dX). */
static void dense_grad_mag(const float *A, int in, int out, const float *X,
                           const float *bpm, size_t M, float *gm, float *dXm) {
  float *dA = gm, *db = gm + (size_t)in * out;
  double *acc = (double *)calloc((size_t)in * out + out, sizeof(double));
  double *accb = acc + (size_t)in * out;
  for (size_t r = 0; r < M; ++r) {
    const float *br = bpm + r * out, *xr = X + r * in;
    for (int o = 0; o < out; ++o) {
      const double b = br[o];
      double *ao = acc + (size_t)o * in;
      for (int k = 0; k < in; ++k) ao[k] += b * fabs((double)xr[k]);
      accb[o] += b;
    }
  }
  for (size_t i = 0; i < (size_t)in * out; ++i) dA[i] = (float)acc[i];
  for (int o = 0; o < out; ++o) db[o] = (float)accb[o];
  free(acc);
  if (dXm) {
    double *row = (double *)malloc(sizeof(double) * in);
    for (size_t r = 0; r < M; ++r) {
      for (int k = 0; k < in; ++k) row[k] = 0.0;
      const float *br = bpm + r * out;
      for (int o = 0; o < out; ++o) {
        const double b = br[o];
        const float *ao = A + (size_t)o * in;
        for (int k = 0; k < in; ++k) row[k] += b * fabs((double)ao[k]);
      }
      for (int k = 0; k < in; ++k) dXm[r * in + k] = (float)row[k];
    }
    free(row);
  }
}

static void or_model_grad_impl(const or_model *m, const float *params,
                               const float *x, int rows, int xcols,
                               or_loss_fn loss, void *ctx, float *grad,
                               float *grad_mag);

/* optimizer::step's forward + loss_grad + model::gradient (nn.h:594-605,
 * 481-488, 510-528).  Layer 0 only gets `gradient`, never `backward`. */
void or_model_grad(const or_model *m, const float *params, const float *x,
                   int rows, int xcols, or_loss_fn loss, void *ctx,
                   float *grad) {
  or_model_grad_impl(m, params, x, rows, xcols, loss, ctx, grad, NULL);
}

/* The same, plus grad_mag: for every gradient entry the sum over the
 * magnitudes of the terms the reference's sums add up (|delta| propagated
 * with |A|, |J| = diag(s) + s s^T for the softmax Jacobian), the scale of
 * its fp32 rounding error under cancellation. */
void or_model_grad_mag(const or_model *m, const float *params, const float *x,
                       int rows, int xcols, or_loss_fn loss, void *ctx,
                       float *grad, float *grad_mag) {
  or_model_grad_impl(m, params, x, rows, xcols, loss, ctx, grad, grad_mag);
}

static void or_model_grad_impl(const or_model *m, const float *params,
                               const float *x, int rows, int xcols,
                               or_loss_fn loss, void *ctx, float *grad,
                               float *grad_mag) {
  const int L = m->nl;
  float *acts[OR_MAX_LAYERS + 1];
  int cols[OR_MAX_LAYERS + 1];
  size_t poff[OR_MAX_LAYERS + 1];
  acts[0] = (float *)x;
  cols[0] = xcols;
  poff[0] = 0;
  for (int l = 0; l < L; ++l) {
    cols[l + 1] = layer_out_cols(m, l, cols[l]);
    acts[l + 1] = (float *)malloc(sizeof(float) * (size_t)rows * cols[l + 1]);
    layer_forward(m, l, params + poff[l], acts[l], rows, cols[l], acts[l + 1]);
    poff[l + 1] = poff[l] + layer_nparams(m, l);
  }
  float *bp = (float *)malloc(sizeof(float) * (size_t)rows * cols[L]);
  loss(ctx, acts[L], rows, cols[L], bp);
  float *bpm = NULL; /* magnitudes of the incoming gradient terms */
  if (grad_mag) {
    bpm = (float *)malloc(sizeof(float) * (size_t)rows * cols[L]);
    for (size_t i = 0; i < (size_t)rows * cols[L]; ++i) bpm[i] = fabsf(bp[i]);
  }
  for (int l = L - 1; l >= 0; --l) {
    const int ic = cols[l], oc = cols[l + 1];
    const float *in = acts[l];
    float *nbp = l > 0 ? (float *)malloc(sizeof(float) * (size_t)rows * ic)
                       : NULL;
    float *nbpm = (l > 0 && bpm)
                      ? (float *)malloc(sizeof(float) * (size_t)rows * ic)
                      : NULL;
    switch (m->type[l]) {
      case OR_FULL:
        dense_grad(params + poff[l], m->in[l], m->out[l], in, bp,
                   (size_t)rows, grad + poff[l], nbp);
        if (bpm)
          dense_grad_mag(params + poff[l], m->in[l], m->out[l], in, bpm,
                         (size_t)rows, grad_mag + poff[l], nbpm);
        break;
      case OR_POINT: /* nn.h:149-186 reshaped to points */
        dense_grad(params + poff[l], m->in[l], m->out[l], in, bp,
                   (size_t)rows * (ic / m->in[l]), grad + poff[l], nbp);
        if (bpm)
          dense_grad_mag(params + poff[l], m->in[l], m->out[l], in, bpm,
                         (size_t)rows * (ic / m->in[l]), grad_mag + poff[l],
                         nbpm);
        break;
      case OR_RELU: /* nn.h:364-376: uses the layer input */
        if (nbp)
          for (size_t i = 0; i < (size_t)rows * ic; ++i)
            nbp[i] = in[i] > 0 ? bp[i] : 0;
        if (nbpm)
          for (size_t i = 0; i < (size_t)rows * ic; ++i)
            nbpm[i] = in[i] > 0 ? bpm[i] : 0;
        break;
      case OR_SOFTMAX:
        if (nbp) {
          float *s = (float *)malloc(sizeof(float) * ic);
          float *pd = (float *)malloc(sizeof(float) * (size_t)ic * ic);
          for (int r = 0; r < rows; ++r) {
            softmax_bwd_row(in + (size_t)r * ic, bp + (size_t)r * oc, ic,
                            nbp + (size_t)r * ic, s, pd);
            if (nbpm) { /* |J| g_m = s * g_m + s (s . g_m) */
              const float *gm = bpm + (size_t)r * oc;
              double sg = 0.0;
              for (int k = 0; k < ic; ++k) sg += (double)s[k] * gm[k];
              for (int j = 0; j < ic; ++j)
                nbpm[(size_t)r * ic + j] =
                    (float)((double)s[j] * gm[j] + (double)s[j] * sg);
            }
          }
          free(s);
          free(pd);
        }
        break;
      case OR_SOFTMAX_XENT: /* nn.h:428-430: identity */
        if (nbp) memcpy(nbp, bp, sizeof(float) * (size_t)rows * ic);
        if (nbpm) memcpy(nbpm, bpm, sizeof(float) * (size_t)rows * ic);
        break;
    }
    free(bp);
    bp = nbp;
    free(bpm);
    bpm = nbpm;
  }
  free(bpm);
  for (int l = 1; l <= L; ++l) free(acts[l]);
}

/* sgd_optimizer::next_parameters (nn.h:622-625): p*(1-wd) - g*lr */
void or_sgd(float *params, const float *grad, size_t n, float lr, float wd) {
  const float keep = 1.0f - wd;
  for (size_t i = 0; i < n; ++i) params[i] = params[i] * keep - grad[i] * lr;
}

/* momentum_optimizer / adam_optimizer::next_parameters (nn.h:630-698).
 * State is created zeroed on the first step (velocity_ / first_moment_ /
 * second_moment_ emplace); adam's step counter t starts at 1 (nn.h:694) and
 * is a float, as in the reference. */
void or_opt_step(or_opt *o, float *params, const float *grad, size_t n) {
  if (o->kind == OR_OPT_SGD) {
    or_sgd(params, grad, n, o->lr, o->wd);
    return;
  }
  if (!o->m) {
    o->m = (float *)calloc(n, sizeof(float));
    o->v = (float *)calloc(n, sizeof(float));
    o->t = 1.0f;
  }
  if (o->kind == OR_OPT_MOMENTUM) { /* v = 0.9 v + g; p - v*lr (nn.h:644-650) */
    const float rho = 0.9f;
    for (size_t i = 0; i < n; ++i) {
      o->m[i] = rho * o->m[i];
      o->m[i] = o->m[i] + grad[i];
      params[i] = params[i] - o->m[i] * o->lr;
    }
    return;
  }
  /* adam (nn.h:677-690) */
  const float b1 = o->b1, b2 = o->b2;
  const float c1 = 1 - powf(b1, o->t), c2 = 1 - powf(b2, o->t);
  for (size_t i = 0; i < n; ++i) {
    const float g = grad[i];
    o->m[i] = o->m[i] * b1 + g * (1 - b1);
    o->v[i] = o->v[i] * b2 + g * g * (1 - b2);
    const float m1 = o->m[i] / c1, m2 = o->v[i] / c2;
    params[i] = params[i] - m1 * o->lr / (sqrtf(m2) + 1e-7f);
  }
  o->t += 1;
}

void or_opt_free(or_opt *o) {
  free(o->m);
  free(o->v);
  o->m = o->v = NULL;
}

/* --------------------------------------------------------------- trainer -- */
typedef struct {
  int32_t *bins; /* B*D */
  int32_t item[3];
  int env, step; /* tags: worker index, apply count at view time */
} st_t;

typedef struct {
  st_t start, end;
  int choice;
  float *distrib; /* B */
  float reward;
} tr_t;

typedef struct {
  st_t opening;
  tr_t *tr;
  int n, cap;
  int frozen;
  int env;
} traj_t;

typedef struct {
  void *data;
  size_t count, bytes;
} buf_t;

struct or_trainer {
  int algo, N, T, episodes;
  or_env_cfg env;
  or_model pol, val;
  float *pp, *vp; /* params */
  size_t np, nv;
  float gamma, lambda;
  float beta, d_targ; /* kl_ppo_learner (policy_gradient.h:332-333) */
  or_opt opt[2];      /* policy, value optimizers */
  uint32_t x, x0;
  uint32_t *xs;       /* per-env streams (or_trainer_set_env_streams) */
  int adv_normalize;  /* opt-in options (or_trainer_set_options) */
  int lr_scale_rows;
  /* workers */
  int32_t *bins, *item; /* N*B*D, N*D */
  int *steps;
  int *cur; /* current trajectory index into list, -1 none */
  /* replay buffer: list of trajectories in creation order */
  traj_t **list;
  int nlist, caplist;
  buf_t buf[OR_BUF_COUNT];
};

static st_t st_copy(const or_trainer *t, const int32_t *bins,
                    const int32_t *item, int env, int step) {
  st_t s;
  const int n = t->env.B * t->env.D;
  s.bins = (int32_t *)malloc(sizeof(int32_t) * n);
  memcpy(s.bins, bins, sizeof(int32_t) * n);
  memset(s.item, 0, sizeof(s.item));
  for (int d = 0; d < t->env.D; ++d) s.item[d] = item[d];
  s.env = env;
  s.step = step;
  return s;
}

static void buf_set(buf_t *b, const void *src, size_t count, size_t el) {
  free(b->data);
  b->data = malloc(count * el + 1);
  if (count) memcpy(b->data, src, count * el);
  b->count = count;
  b->bytes = count * el;
}

static void buf_append(buf_t *b, const void *src, size_t count, size_t el) {
  b->data = realloc(b->data, b->bytes + count * el + 1);
  memcpy((char *)b->data + b->bytes, src, count * el);
  b->bytes += count * el;
  b->count += count;
}

static void buf_clear(buf_t *b) {
  free(b->data);
  b->data = NULL;
  b->count = b->bytes = 0;
}

or_trainer *or_trainer_create(int algo, const or_env_cfg *env, int N, int T,
                              int episodes, const or_model *pol,
                              const float *pol_params, const or_model *val,
                              const float *val_params, float lr_pi, float lr_v,
                              float wd_pi, float wd_v, float gamma,
                              uint32_t x0) {
  or_trainer *t = (or_trainer *)calloc(1, sizeof(or_trainer));
  t->algo = algo;
  t->N = N;
  t->T = T;
  t->episodes = episodes;
  t->env = *env;
  t->pol = *pol;
  t->np = or_model_nparams(pol);
  t->pp = (float *)malloc(sizeof(float) * t->np);
  memcpy(t->pp, pol_params, sizeof(float) * t->np);
  if (val) {
    t->val = *val;
    t->nv = or_model_nparams(val);
    t->vp = (float *)malloc(sizeof(float) * t->nv);
    memcpy(t->vp, val_params, sizeof(float) * t->nv);
  }
  t->gamma = gamma;
  t->lambda = 0.95f; /* policy_gradient.h:286 */
  t->opt[0].kind = t->opt[1].kind = OR_OPT_SGD;
  t->opt[0].lr = lr_pi;
  t->opt[0].wd = wd_pi;
  t->opt[1].lr = lr_v;
  t->opt[1].wd = wd_v;
  t->beta = 1.0f;
  t->d_targ = 1e-9f;
  t->x = t->x0 = x0;
  const int BD = env->B * env->D;
  t->bins = (int32_t *)malloc(sizeof(int32_t) * (size_t)N * BD);
  t->item = (int32_t *)calloc((size_t)N * 3, sizeof(int32_t));
  t->steps = (int *)calloc(N, sizeof(int));
  t->cur = (int *)malloc(sizeof(int) * N);
  /* envs constructed in worker order: 2 engine draws each (bin_packing.h:50) */
  for (int i = 0; i < N; ++i) {
    or_env_construct(env, t->bins + (size_t)i * BD, t->item + (size_t)i * 3,
                     &t->x);
    t->cur[i] = -1;
  }
  return t;
}

static void traj_free(traj_t *tj) {
  free(tj->opening.bins);
  for (int i = 0; i < tj->n; ++i) {
    free(tj->tr[i].start.bins);
    free(tj->tr[i].end.bins);
    free(tj->tr[i].distrib);
  }
  free(tj->tr);
  free(tj);
}

void or_trainer_destroy(or_trainer *t) {
  if (!t) return;
  for (int i = 0; i < t->nlist; ++i) traj_free(t->list[i]);
  free(t->list);
  for (int b = 0; b < OR_BUF_COUNT; ++b) buf_clear(&t->buf[b]);
  free(t->pp);
  free(t->vp);
  free(t->bins);
  free(t->item);
  free(t->steps);
  free(t->cur);
  free(t->xs);
  or_opt_free(&t->opt[0]);
  or_opt_free(&t->opt[1]);
  free(t);
}

void or_trainer_set_optimizer(or_trainer *t, int which, int kind, float lr,
                              float wd, float beta1, float beta2) {
  or_opt *o = &t->opt[which ? 1 : 0];
  or_opt_free(o);
  o->kind = kind;
  o->lr = lr;
  o->wd = wd;
  o->b1 = beta1;
  o->b2 = beta2;
  o->t = 1.0f;
}

uint32_t or_trainer_rng(const or_trainer *t) { return t->x; }

void or_trainer_set_options(or_trainer *t, int adv_normalize,
                            int lr_scale_rows) {
  t->adv_normalize = adv_normalize;
  t->lr_scale_rows = lr_scale_rows;
}

/* optimizer step with the opt-in lr / rows scaling (rows = T * N) */
static void opt_step_scaled(or_trainer *t, or_opt *o, float *params,
                            const float *grad, size_t n) {
  const float lr = o->lr;
  if (t->lr_scale_rows) o->lr = (float)((double)lr / ((double)t->T * t->N));
  or_opt_step(o, params, grad, n);
  o->lr = lr;
}

/* Independent per-env streams: env i draws from x0 advanced by i * stride
 * (the device evaluators' and REINFORCE trainer's convention; env 0 is the
 * single-env reference run).  Re-constructs the envs (2 draws each). */
void or_trainer_set_env_streams(or_trainer *t, uint64_t stride,
                                int reconstruct) {
  const int BD = t->env.B * t->env.D;
  free(t->xs);
  t->xs = (uint32_t *)malloc(sizeof(uint32_t) * t->N);
  for (int i = 0; i < t->N; ++i) {
    if (!reconstruct) { /* keep the envs; streams from the current engine */
      t->xs[i] = or_minstd_jump(t->x, (uint64_t)i * stride);
      continue;
    }
    t->xs[i] = or_minstd_jump(t->x0, (uint64_t)i * stride);
    or_env_construct(&t->env, t->bins + (size_t)i * BD,
                     t->item + (size_t)i * 3, &t->xs[i]);
  }
}

/* Explicit per-env stream states (the envs are kept): env i draws from xs[i]
 * from the next rollout on.  A sample of envs [off, off + N) of a larger
 * reference-order job: xs[i] = the engine state at global env off + i's first
 * draw of the iteration (2 Ng + 4 T (off + i) after x0). */
void or_trainer_set_stream_states(or_trainer *t, const uint32_t *xs) {
  free(t->xs);
  t->xs = (uint32_t *)malloc(sizeof(uint32_t) * t->N);
  memcpy(t->xs, xs, sizeof(uint32_t) * t->N);
}

const uint32_t *or_trainer_env_streams(const or_trainer *t) { return t->xs; }

static uint32_t *env_rng(or_trainer *t, int i) {
  return t->xs ? &t->xs[i] : &t->x;
}

void or_trainer_get_params(const or_trainer *t, int which, float *out) {
  if (which == 0)
    memcpy(out, t->pp, sizeof(float) * t->np);
  else
    memcpy(out, t->vp, sizeof(float) * t->nv);
}

void or_trainer_set_params(or_trainer *t, int which, const float *in) {
  if (which == 0)
    memcpy(t->pp, in, sizeof(float) * t->np);
  else
    memcpy(t->vp, in, sizeof(float) * t->nv);
}

const void *or_trainer_buf(const or_trainer *t, int which, size_t *count) {
  if (which < 0 || which >= OR_BUF_COUNT) {
    *count = 0;
    return NULL;
  }
  *count = t->buf[which].count;
  return t->buf[which].data;
}

static const st_t *traj_last(const traj_t *tj) {
  return tj->n ? &tj->tr[tj->n - 1].end : &tj->opening;
}

/* replay_buffer::emplace_trajectory (rl.h:215-219) */
static int emplace_traj(or_trainer *t, st_t opening, int env) {
  if (t->nlist == t->caplist) {
    t->caplist = t->caplist ? 2 * t->caplist : 16;
    t->list = (traj_t **)realloc(t->list, sizeof(traj_t *) * t->caplist);
  }
  traj_t *tj = (traj_t *)calloc(1, sizeof(traj_t));
  tj->opening = opening;
  tj->env = env;
  t->list[t->nlist] = tj;
  return t->nlist++;
}

static void traj_add(traj_t *tj, tr_t tr) {
  if (tj->n == tj->cap) {
    tj->cap = tj->cap ? 2 * tj->cap : 8;
    tj->tr = (tr_t *)realloc(tj->tr, sizeof(tr_t) * tj->cap);
  }
  tj->tr[tj->n++] = tr;
}

/* xylo::agent::step (rl.h:325-349) with policy_gradient_policy::react
 * (policy_gradient.h:343-350) and discrete_action::from_vector (rl.h:27-30). */
static int agent_step(or_trainer *t, int i, int forced_choice) {
  const or_env_cfg *c = &t->env;
  const int B = c->B, D = c->D, BD = B * D;
  int32_t *bins = t->bins + (size_t)i * BD, *item = t->item + (size_t)i * 3;
  if (t->cur[i] < 0)
    t->cur[i] = emplace_traj(t, st_copy(t, bins, item, i, t->steps[i]), i);
  traj_t *tj = t->list[t->cur[i]];
  const st_t *prev = traj_last(tj);

  float *obs = (float *)malloc(sizeof(float) * 2 * D * B);
  or_obs(c, prev->bins, prev->item, obs);
  float *probs = (float *)malloc(sizeof(float) * B);
  or_model_eval(&t->pol, t->pp, obs, 1, 2 * D * B, probs);
  free(obs);
  int choice;
  if (forced_choice >= 0) {
    (void)or_canonical(env_rng(t, i)); /* the sampler's 2 engine draws */
    choice = forced_choice;
  } else {
    choice = or_discrete(env_rng(t, i), probs, B);
  }

  /* step log: state before apply (== prev, see rl.h:332-334) */
  int32_t done32;
  buf_append(&t->buf[OR_BUF_STEP_BINS], bins, BD, sizeof(int32_t));
  buf_append(&t->buf[OR_BUF_STEP_ITEM], item, D, sizeof(int32_t));
  buf_append(&t->buf[OR_BUF_STEP_CHOICE], &choice, 1, sizeof(int32_t));
  buf_append(&t->buf[OR_BUF_STEP_PCHOICE], probs + choice, 1, sizeof(float));

  or_env_apply(c, bins, item, choice, env_rng(t, i));
  t->steps[i]++;
  st_t curr = st_copy(t, bins, item, i, t->steps[i]);
  const int over = or_env_game_over(c, curr.bins);
  tr_t tr;
  tr.start = st_copy(t, prev->bins, prev->item, prev->env, prev->step);
  tr.end = curr;
  tr.choice = choice;
  tr.distrib = probs;
  tr.reward = over ? 0.0f : 1.0f; /* agent::get_reward bin_packing.h:102-106 */
  traj_add(tj, tr);
  done32 = over;
  buf_append(&t->buf[OR_BUF_STEP_DONE], &done32, 1, sizeof(int32_t));
  if (over) {
    or_env_reset(c, bins, item, env_rng(t, i));
    tj->frozen = 1;
    t->cur[i] = -1;
    return 0;
  }
  return 1;
}

void or_trainer_rollout(or_trainer *t, const int32_t *forced) {
  for (int b = OR_BUF_STEP_BINS; b <= OR_BUF_STEP_PCHOICE; ++b)
    buf_clear(&t->buf[b]);
  for (int i = 0; i < t->N; ++i) {
    if (t->algo == OR_PG) {
      /* pg_training.cc:221-225: play_one_episode x episodes */
      for (int e = 0; e < t->episodes; ++e)
        while (agent_step(t, i, -1))
          ;
    } else {
      /* agent::play_steps (rl.h:356-360) */
      for (int s = 0; s < t->T; ++s)
        agent_step(t, i, forced ? forced[(size_t)i * t->T + s] : -1);
    }
  }
  const int BD = t->env.B * t->env.D;
  buf_set(&t->buf[OR_BUF_FINAL_BINS], t->bins, (size_t)t->N * BD,
          sizeof(int32_t));
  buf_clear(&t->buf[OR_BUF_FINAL_ITEM]);
  for (int i = 0; i < t->N; ++i)
    buf_append(&t->buf[OR_BUF_FINAL_ITEM], t->item + (size_t)i * 3,
               t->env.D, sizeof(int32_t));
}

/* ---- loss gradients (functors handed to optimizer::step) ---- */
typedef struct {
  const float *labels;
} sq_ctx;
/* square_loss_grad (nn.h:548-550): output - label */
static void loss_square(void *ctx, const float *out, int rows, int cols,
                        float *g) {
  const sq_ctx *c = (const sq_ctx *)ctx;
  (void)cols;
  for (int r = 0; r < rows; ++r) g[r] = out[r] - c->labels[r];
}

typedef struct {
  const int *choice;
  const float *pold;
  const float *adv;
  int ppo;
  /* KL-PPO: old distributions [rows][cols], adaptive beta, target KL */
  const float *qold;
  float *beta;
  float d_targ;
  double d_avg; /* out: mean KL(q || p) of the call */
} pl_ctx;
/* PPO: surrogate_loss -> clipped_gradient (policy_gradient.h:28-38,
 * rl.h:54-74).  AC / PG: policy_loss -> softmax_gradient_log
 * (policy_gradient.h:16-26, rl.h:45-52). */
static void loss_kl(pl_ctx *c, const float *out, int rows, int cols,
                    float *g);
static void loss_policy(void *ctx, const float *out, int rows, int cols,
                        float *g) {
  pl_ctx *c = (pl_ctx *)ctx;
  if (c->qold) {
    loss_kl(c, out, rows, cols, g);
    return;
  }
  for (int r = 0; r < rows; ++r) {
    const float *p = out + (size_t)r * cols;
    float *o = g + (size_t)r * cols;
    const int ch = c->choice[r];
    const float A = c->adv[r];
    if (c->ppo) {
      const float eps = 0.2f;
      for (int j = 0; j < cols; ++j) o[j] = 0.0f;
      float ratio = p[ch] / c->pold[r];
      float clipped = ratio;
      if (ratio > (1 + eps))
        clipped = 1 + eps;
      else if (ratio < (1 - eps))
        clipped = 1 - eps;
      float a1 = clipped * A, a2 = ratio * A;
      float ig = (a1 < a2 ? a1 : a2) * -1;
      o[ch] = ig / p[ch];
    } else {
      for (int j = 0; j < cols; ++j) o[j] = p[j] * A;
      o[ch] -= A;
    }
  }
}

/* kl_regulated_loss (policy_gradient.h:41-85): softmax_gradient_log rows
 * (rl.h:45-52) + beta * softmax_cross_entropy_loss_grad(q, p) = beta (p - q)
 * (nn.h:584-586), then the mean KL(q || p) over all rows (kl_divergence,
 * :41-46) adapts beta for the next call: halve below d_targ / 1.5, double
 * above 1.5 d_targ, clamp to [1e-25, 0.1].  The gradient uses the beta from
 * before the update. */
static void loss_kl(pl_ctx *c, const float *out, int rows, int cols,
                    float *g) {
  const float beta = *c->beta;
  double dsum = 0.0;
  for (int r = 0; r < rows; ++r) {
    const float *p = out + (size_t)r * cols;
    const float *q = c->qold + (size_t)r * cols;
    float *o = g + (size_t)r * cols;
    const float A = c->adv[r];
    for (int j = 0; j < cols; ++j) o[j] = p[j] * A;
    o[c->choice[r]] -= A;
    double d = 0.0;
    for (int j = 0; j < cols; ++j) {
      o[j] += beta * (p[j] - q[j]);
      d += (double)q[j] * log((double)q[j] / (double)p[j]);
    }
    dsum += d;
  }
  const float d_avg = (float)(dsum / rows);
  c->d_avg = d_avg;
  float b = beta;
  if (fabsf(d_avg) < c->d_targ / 1.5f)
    b /= 2;
  else if (fabsf(d_avg) > c->d_targ * 1.5f)
    b *= 2;
  if (b < 1e-25f) b = 1e-25f;
  if (b > 0.1f) b = 0.1f;
  *c->beta = b;
}

void or_trainer_learn(or_trainer *t) {
  const or_env_cfg *c = &t->env;
  const int B = c->B, D = c->D, len = 2 * D * B;
  const int pg = t->algo == OR_PG;
  /* replay_buffer::sample_td (rl.h:222-234): all trajectories, list order */
  int ntr = 0;
  for (int k = 0; k < t->nlist; ++k) ntr += t->list[k]->n;
  const int rows = pg ? ntr : ntr + t->nlist;
  float *sm = (float *)malloc(sizeof(float) * (size_t)rows * len);
  int *choice = (int *)malloc(sizeof(int) * rows);
  float *pold = (float *)malloc(sizeof(float) * rows);
  int32_t *renv = (int32_t *)malloc(sizeof(int32_t) * rows);
  int32_t *rstep = (int32_t *)malloc(sizeof(int32_t) * rows);
  int32_t *rend = (int32_t *)malloc(sizeof(int32_t) * rows);
  float *qrows = (float *)malloc(sizeof(float) * (size_t)rows * B);
  /* state_matrix: transitions + one end row per trajectory, end-row action =
   * copy of the previous one (policy_gradient.h:168-180) */
  int r = 0;
  for (int k = 0; k < t->nlist; ++k) {
    traj_t *tj = t->list[k];
    for (int i = 0; i < tj->n; ++i) {
      tr_t *tr = &tj->tr[i];
      or_obs(c, tr->start.bins, tr->start.item, sm + (size_t)r * len);
      choice[r] = tr->choice;
      pold[r] = tr->distrib[tr->choice];
      memcpy(qrows + (size_t)r * B, tr->distrib, sizeof(float) * B);
      renv[r] = tr->start.env;
      rstep[r] = tr->start.step;
      rend[r] = 0;
      ++r;
    }
    if (!pg) {
      tr_t *bk = &tj->tr[tj->n - 1];
      or_obs(c, bk->end.bins, bk->end.item, sm + (size_t)r * len);
      choice[r] = choice[r - 1];
      pold[r] = pold[r - 1];
      memcpy(qrows + (size_t)r * B, qrows + (size_t)(r - 1) * B,
             sizeof(float) * B);
      renv[r] = bk->end.env;
      rstep[r] = bk->end.step;
      rend[r] = 1;
      ++r;
    }
  }
  buf_set(&t->buf[OR_BUF_ROWS], sm, (size_t)rows * len, sizeof(float));
  buf_set(&t->buf[OR_BUF_ROW_ENV], renv, rows, sizeof(int32_t));
  buf_set(&t->buf[OR_BUF_ROW_STEP], rstep, rows, sizeof(int32_t));
  buf_set(&t->buf[OR_BUF_ROW_IS_END], rend, rows, sizeof(int32_t));
  buf_set(&t->buf[OR_BUF_ROW_CHOICE], choice, rows, sizeof(int32_t));
  buf_set(&t->buf[OR_BUF_ROW_POLD], pold, rows, sizeof(float));
  buf_clear(&t->buf[OR_BUF_POLICY_GRADS]);

  float *adv = (float *)calloc(rows, sizeof(float));
  float *pgrad = (float *)malloc(sizeof(float) * t->np);
  if (pg) {
    /* policy_gradient_learner::get_advantages (policy_gradient.h:125-147):
     * discounted prefix sums written into the slice back-to-front. */
    float total = 0.0f;
    int cur = 0;
    for (int k = 0; k < t->nlist; ++k) {
      traj_t *tj = t->list[k];
      float reward = 0.0f;
      for (int i = 0; i < tj->n; ++i) {
        reward = tj->tr[i].reward + t->gamma * reward;
        adv[cur + tj->n - 1 - i] = reward;
      }
      total += adv[cur];
      cur += tj->n;
    }
    float avg = total / (float)t->nlist;
    for (int i = 0; i < rows; ++i) adv[i] = adv[i] - avg;
    pl_ctx pc = {choice, pold, adv, 0, NULL, NULL, 0, 0};
    or_model_grad(&t->pol, t->pp, sm, rows, len, loss_policy, &pc, pgrad);
    buf_append(&t->buf[OR_BUF_POLICY_GRADS], pgrad, t->np, sizeof(float));
    or_opt_step(&t->opt[0], t->pp, pgrad, t->np);
  } else {
    /* update_value_model (policy_gradient.h:196-218) */
    float *values = (float *)malloc(sizeof(float) * rows);
    float *targets = (float *)malloc(sizeof(float) * rows);
    or_model_eval(&t->val, t->vp, sm, rows, len, values);
    int cur = 0;
    for (int k = 0; k < t->nlist; ++k) {
      traj_t *tj = t->list[k];
      for (int i = 0; i < tj->n; ++i) {
        targets[cur] = tj->tr[i].reward + t->gamma * values[cur + 1];
        ++cur;
      }
      targets[cur] = values[cur];
      ++cur;
    }
    buf_set(&t->buf[OR_BUF_VALUES], values, rows, sizeof(float));
    buf_set(&t->buf[OR_BUF_TARGETS], targets, rows, sizeof(float));
    float *vgrad = (float *)malloc(sizeof(float) * t->nv);
    sq_ctx sc = {targets};
    float *vmag = (float *)malloc(sizeof(float) * t->nv);
    or_model_grad_mag(&t->val, t->vp, sm, rows, len, loss_square, &sc, vgrad,
                      vmag);
    buf_set(&t->buf[OR_BUF_VALUE_GRAD], vgrad, t->nv, sizeof(float));
    buf_set(&t->buf[OR_BUF_VALUE_GRAD_MAG], vmag, t->nv, sizeof(float));
    free(vmag);
    opt_step_scaled(t, &t->opt[1], t->vp, vgrad, t->nv);
    free(vgrad);

    /* calculate_advantage (policy_gradient.h:220-281), post-update values */
    or_model_eval(&t->val, t->vp, sm, rows, len, values);
    cur = 0;
    for (int k = 0; k < t->nlist; ++k) {
      cur += t->list[k]->n;
      if (t->list[k]->frozen) values[cur] = 0;
      ++cur;
    }
    float *deltas = (float *)calloc(rows, sizeof(float));
    cur = 0;
    for (int k = 0; k < t->nlist; ++k) {
      traj_t *tj = t->list[k];
      for (int i = 0; i < tj->n; ++i) {
        deltas[cur] = tj->tr[i].reward + t->gamma * values[cur + 1] -
                      values[cur];
        ++cur;
      }
      deltas[cur] = 0;
      ++cur;
    }
    const float lg = t->lambda * t->gamma;
    cur = 0;
    for (int k = 0; k < t->nlist; ++k) {
      traj_t *tj = t->list[k];
      const int end = cur + tj->n;
      for (int i = 0; i < tj->n; ++i) {
        adv[cur] = 0;
        float coef = 1;
        for (int j = cur; j < end; ++j) {
          adv[cur] += deltas[j] * coef;
          coef *= lg;
        }
        ++cur;
      }
      adv[cur] = 0;
      ++cur;
    }
    free(deltas);
    free(values);
    free(targets);
    if (t->adv_normalize) {
      /* opt-in (not in the reference): over the transition rows, population
       * statistics in double, A <- (A - mean) / (std + 1e-8) rounded once;
       * end rows keep A = 0 */
      double s1 = 0.0, s2 = 0.0, cnt = 0.0;
      for (int i = 0; i < rows; ++i)
        if (!rend[i]) {
          s1 += adv[i];
          s2 += (double)adv[i] * adv[i];
          cnt += 1.0;
        }
      const double mean = s1 / cnt;
      double var = s2 / cnt - mean * mean;
      if (var < 0) var = 0;
      const double inv = 1.0 / (sqrt(var) + 1e-8);
      for (int i = 0; i < rows; ++i)
        if (!rend[i]) adv[i] = (float)(((double)adv[i] - mean) * inv);
    }

    /* optimize_action: PPO k=4 surrogate steps (policy_gradient.h:297-307),
     * AC one policy_loss step (:187-194) */
    const int epochs = t->algo == OR_AC ? 1 : 4;
    pl_ctx pc = {choice, pold, adv, t->algo == OR_PPO, NULL, NULL, 0, 0};
    if (t->algo == OR_KLPPO) {
      pc.qold = qrows;
      pc.beta = &t->beta;
      pc.d_targ = t->d_targ;
    }
    buf_clear(&t->buf[OR_BUF_KL]);
    buf_clear(&t->buf[OR_BUF_POLICY_GRADS_MAG]);
    float *pmag = (float *)malloc(sizeof(float) * t->np);
    for (int e = 0; e < epochs; ++e) {
      const float beta_used = t->beta;
      or_model_grad_mag(&t->pol, t->pp, sm, rows, len, loss_policy, &pc,
                        pgrad, pmag);
      buf_append(&t->buf[OR_BUF_POLICY_GRADS], pgrad, t->np, sizeof(float));
      buf_append(&t->buf[OR_BUF_POLICY_GRADS_MAG], pmag, t->np,
                 sizeof(float));
      if (t->algo == OR_KLPPO) {
        const float kl[3] = {beta_used, (float)pc.d_avg, t->beta};
        buf_append(&t->buf[OR_BUF_KL], kl, 3, sizeof(float));
      }
      opt_step_scaled(t, &t->opt[0], t->pp, pgrad, t->np);
    }
    free(pmag);
  }
  buf_set(&t->buf[OR_BUF_ADVANTAGES], adv, rows, sizeof(float));
  free(adv);
  free(pgrad);
  free(sm);
  free(choice);
  free(pold);
  free(qrows);
  free(renv);
  free(rstep);
  free(rend);

  /* replay_buffer::forget (rl.h:274-291) */
  int w = 0;
  for (int k = 0; k < t->nlist; ++k) {
    traj_t *tj = t->list[k];
    if (tj->frozen) {
      traj_free(tj);
      continue;
    }
    /* keep the last state as the new opening; the agent keeps pointing at it */
    st_t last = tj->tr[tj->n - 1].end;
    tj->tr[tj->n - 1].end.bins = NULL;
    free(tj->opening.bins);
    tj->opening = last;
    for (int i = 0; i < tj->n; ++i) {
      free(tj->tr[i].start.bins);
      free(tj->tr[i].end.bins);
      free(tj->tr[i].distrib);
    }
    tj->n = 0;
    t->cur[tj->env] = w;
    t->list[w++] = tj;
  }
  t->nlist = w;
}

void or_policy_grad_rows(const or_model *m, const float *params, const float *x,
                         int rows, int xcols, const int32_t *choice,
                         const float *pold, const float *adv, int algo,
                         float *grad) {
  int *ch = (int *)malloc(sizeof(int) * (rows > 0 ? rows : 1));
  for (int r = 0; r < rows; ++r) ch[r] = choice[r];
  pl_ctx pc = {ch, pold, adv, algo == OR_PPO, NULL, NULL, 0, 0};
  or_model_grad(m, params, x, rows, xcols, loss_policy, &pc, grad);
  free(ch);
}

void or_value_grad_rows(const or_model *m, const float *params, const float *x,
                        int rows, int xcols, const float *targets, float *grad) {
  sq_ctx sc = {targets};
  or_model_grad(m, params, x, rows, xcols, loss_square, &sc, grad);
}

void or_policy_grad_rows_mag(const or_model *m, const float *params,
                             const float *x, int rows, int xcols,
                             const int32_t *choice, const float *pold,
                             const float *adv, int algo, float *grad,
                             float *mag) {
  int *ch = (int *)malloc(sizeof(int) * (rows > 0 ? rows : 1));
  for (int r = 0; r < rows; ++r) ch[r] = choice[r];
  pl_ctx pc = {ch, pold, adv, algo == OR_PPO, NULL, NULL, 0, 0};
  or_model_grad_mag(m, params, x, rows, xcols, loss_policy, &pc, grad, mag);
  free(ch);
}

void or_value_grad_rows_mag(const or_model *m, const float *params,
                            const float *x, int rows, int xcols,
                            const float *targets, float *grad, float *mag) {
  sq_ctx sc = {targets};
  or_model_grad_mag(m, params, x, rows, xcols, loss_square, &sc, grad, mag);
}

/* deep_agent.cc:25-41 / policy_gradient_deterministic_policy
 * (policy_gradient.h:356-373): argmax over the model output. */
double or_eval_argmax(const or_env_cfg *c, const or_model *pol,
                      const float *params, long episodes, uint32_t *x) {
  const int B = c->B, D = c->D;
  int32_t bins[128 * 3], item[3];
  float obs[2 * 3 * 128], out[128];
  double total = 0;
  or_env_construct(c, bins, item, x);
  for (long e = 0; e < episodes; ++e) {
    for (;;) {
      or_obs(c, bins, item, obs);
      or_model_eval(pol, params, obs, 1, 2 * D * B, out);
      int ch = or_argmax(out, B);
      or_env_apply(c, bins, item, ch, x);
      int over = or_env_game_over(c, bins);
      if (over) {
        or_env_reset(c, bins, item, x);
        break;
      }
      total += 1.0;
    }
  }
  return total;
}

/* The reference's heuristic agents (firstfit_agent.cc:10-28,
 * bestfit_agent.cc:10-30, minwaste_agent.cc:10-39, random_policy rl.h:
 * 305-316) playing `episodes` episodes on one env seeded at *x (constructed
 * first, 2 draws); returns the total reward.  Generalised to D dims as the
 * device kernel is (bestfit sums item/bin over the dims in order; minwaste's
 * 0 score = residual with one dim at cap/2 and the others 0). */
double or_heuristic_eval(const or_env_cfg *c, int kind, long episodes,
                         uint32_t *x, int32_t *lens) {
  const int B = c->B, D = c->D;
  int32_t bins[128 * 3], item[3];
  float sc[128];
  double total = 0;
  or_env_construct(c, bins, item, x);
  for (long e = 0; e < episodes; ++e) {
    int32_t len = 0;
    for (;;) {
      int ch = 0;
      if (kind == OR_HEUR_RANDOM) {
        for (int i = 0; i < B; ++i) sc[i] = (float)(1.0 / B);
        ch = or_discrete(x, sc, B);
      } else {
        for (int i = 0; i < B; ++i) {
          int fits = 1;
          for (int d = 0; d < D; ++d) fits &= item[d] <= bins[i * D + d];
          if (kind == OR_HEUR_FIRSTFIT) {
            sc[i] = fits ? 1.0f : 0.0f;
          } else if (kind == OR_HEUR_BESTFIT) {
            float v = -1.0f;
            if (fits) {
              v = (float)item[0] / (float)bins[i * D];
              for (int d = 1; d < D; ++d)
                v = v + (float)item[d] / (float)bins[i * D + d];
            }
            sc[i] = v;
          } else {
            float v = -1.0f;
            if (fits) {
              int half = 0, zero = 0;
              for (int d = 0; d < D; ++d) {
                const int r = bins[i * D + d] - item[d];
                half += r == c->cap / 2;
                zero += r == 0;
              }
              v = (half == 1 && zero == D - 1) ? 0.0f : 1.0f;
            }
            sc[i] = v;
          }
        }
        ch = or_argmax(sc, B);
      }
      or_env_apply(c, bins, item, ch, x);
      ++len;
      if (or_env_game_over(c, bins)) {
        or_env_reset(c, bins, item, x);
        break;
      }
      total += 1.0;
    }
    if (lens) lens[e] = len;
  }
  return total;
}
