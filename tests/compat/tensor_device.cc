// Device-resident tensors of the drop-in xylo/tensor.h (tensors created with
// on_device = true, in HBM): every operation on them runs the HIP kernels
// behind xh_tensor_* and must give what the same operation gives on host
// tensors of the same values (the host loops are the reference's,
// tests/compat/tensor_ops.cc holds them to the reference's own build).
// Drop-in only (to_host / to_device are extensions).  Prints one line per
// check, "ok <name> <err>" or "FAIL <name> <err>", and exits 1 on a failure;
// run by tests/test_gpu_tensor.py.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>

#include <xylo/tensor.h>

namespace {

int g_fail = 0;
uint32_t g_state = 777u;
float rnd() {
  g_state = g_state * 1664525u + 1013904223u;
  return (float)(g_state >> 8) / 16777216.0f * 2.0f - 1.0f;
}
xylo::vector rvec(std::size_t n, float lo = -1.0f, float hi = 1.0f) {
  xylo::vector v(n);
  for (std::size_t i = 0; i < n; ++i) v[i] = lo + (rnd() + 1.0f) * 0.5f * (hi - lo);
  return v;
}
xylo::matrix rmat(std::size_t r, std::size_t c) {
  xylo::matrix m(std::array<std::size_t, 2>{r, c});
  xylo::vector_view f = flatten(m);
  for (std::size_t i = 0; i < f.size(); ++i) f[i] = rnd();
  return m;
}

// |x - y| <= tol * max(1, |y|) entry by entry (y: the host result)
void check(const std::string &name, xylo::vector_view dev_or_host,
           xylo::vector_view host, double tol = 1e-5) {
  const xylo::vector d = xylo::to_host<1>(dev_or_host);
  double worst = 0.0;
  bool bad = d.size() != host.size();
  for (std::size_t i = 0; !bad && i < host.size(); ++i) {
    const double e = std::fabs((double)d[i] - host[i]) /
                     std::fmax(1.0, std::fabs((double)host[i]));
    if (!(e <= tol)) bad = true;
    worst = std::fmax(worst, e);
  }
  std::printf("%s %s %.3g\n", bad ? "FAIL" : "ok", name.c_str(), worst);
  g_fail |= bad;
}
void check_s(const std::string &name, double x, double y, double tol = 1e-5) {
  const double e = std::fabs(x - y) / std::fmax(1.0, std::fabs(y));
  const bool bad = !(e <= tol);
  std::printf("%s %s %.3g (%.9g vs %.9g)\n", bad ? "FAIL" : "ok", name.c_str(),
              e, x, y);
  g_fail |= bad;
}
void check_i(const std::string &name, long x, long y) {
  std::printf("%s %s %ld %ld\n", x == y ? "ok" : "FAIL", name.c_str(), x, y);
  g_fail |= x != y;
}

void vectors(std::size_t n) {
  const std::string t = "n" + std::to_string(n) + "_";
  xylo::vector h1 = rvec(n), h2 = rvec(n, 0.5f, 2.0f);
  xylo::vector d1 = xylo::to_device(h1), d2 = xylo::to_device(h2);
  check_i(t + "on_device", d1.on_device(), 1);
  check(t + "round_trip", d1, h1, 0.0);
  check(t + "add", d1 + d2, h1 + h2, 0.0);
  check(t + "sub", d1 - d2, h1 - h2, 0.0);
  check(t + "mul", d1 * d2, h1 * h2, 0.0);
  check(t + "div", d1 / d2, h1 / h2, 0.0);
  check(t + "add_s", d1 + 0.25f, h1 + 0.25f, 0.0);
  check(t + "sub_s", d1 - 0.25f, h1 - 0.25f, 0.0);
  check(t + "mul_s", d1 * 3.5f, h1 * 3.5f, 0.0);
  check(t + "div_s", d1 / 3.5f, h1 / 3.5f, 0.0);
  check(t + "abs", abs(d1), abs(h1), 0.0);
  check(t + "sqrt", sqrt(d2), sqrt(h2), 0.0);
  check(t + "sin", sin(d1), sin(h1), 1e-6);
  check(t + "exp", exp(d1), exp(h1), 1e-6);
  check(t + "log", log(d2), log(h2), 1e-6);
  xylo::vector dc(d1), hc(h1);
  for (auto *p : {&dc, &hc}) {
    *p += 1.5f;
    *p -= (p == &dc ? xylo::vector_view(d2) : xylo::vector_view(h2));
    *p *= 0.75f;
    *p /= 1.25f;  // the reference's scalar-first quirk, on both sides
    *p -= 0.125f;
    *p *= (p == &dc ? xylo::vector_view(d2) : xylo::vector_view(h2));
  }
  check(t + "compound", dc, hc, 0.0);
  // reductions: the device sums in double, the host in float partial sums
  check_s(t + "sum", sum(d1), sum(h1), 1e-4);
  check_s(t + "dot", dot(d1, d2), dot(h1, h2), 1e-4);
  check_s(t + "mean", mean(d1), mean(h1), 1e-5);
  check_s(t + "variance", variance(d1), variance(h1), 1e-4);
  check_s(t + "stddev", xylo::vector_view(d1).stddev(),
          xylo::vector_view(h1).stddev(), 1e-4);
  check_s(t + "max", max(d1), max(h1), 0.0);
  check_i(t + "argmax", (long)argmax(d1), (long)argmax(h1));
  // fill, assignment, views into device memory
  xylo::vector df(n, true), hf(n);
  df = 2.5f;
  hf = 2.5f;
  check(t + "fill", df, hf, 0.0);
  df = xylo::vector_view(d1);
  check(t + "assign_view", df, h1, 0.0);
  check(t + "slice", slice(xylo::vector_view(d1), n / 3, n / 4),
        slice(xylo::vector_view(h1), n / 3, n / 4), 0.0);
  check_i(t + "equal", xylo::vector_view(d1) == xylo::vector_view(d1), 1);
  check_i(t + "equal_copy", xylo::vector_view(xylo::to_device(h1)) ==
                                xylo::vector_view(d1), 1);
  check_i(t + "unequal", xylo::vector_view(d1) == xylo::vector_view(d2), 0);
}

void gemms(std::size_t M, std::size_t N, std::size_t K) {
  const std::string t = "g" + std::to_string(M) + "x" + std::to_string(N) + "x" +
                        std::to_string(K) + "_";
  xylo::matrix a = rmat(M, K), b = rmat(N, K), c = rmat(K, N);
  xylo::matrix da = xylo::to_device(a), db = xylo::to_device(b),
               dc = xylo::to_device(c);
  // the host loops (below the device threshold the drop-in keeps them)
  xylo::matrix mt(std::array<std::size_t, 2>{M, N});
  for (std::size_t i = 0; i < M; ++i)
    for (std::size_t j = 0; j < N; ++j) {
      double s = 0;
      for (std::size_t k = 0; k < K; ++k)
        s += (double)flatten(a)[i * K + k] * flatten(b)[j * K + k];
      flatten(mt)[i * N + j] = (float)s;
    }
  check(t + "matmul_transposed", flatten(::matmul_transposed(da, db)),
        flatten(mt), 2e-5);
  xylo::matrix mm(std::array<std::size_t, 2>{M, N});
  for (std::size_t i = 0; i < M; ++i)
    for (std::size_t j = 0; j < N; ++j) {
      double s = 0;
      for (std::size_t k = 0; k < K; ++k)
        s += (double)flatten(a)[i * K + k] * flatten(c)[k * N + j];
      flatten(mm)[i * N + j] = (float)s;
    }
  check(t + "matmul", flatten(::matmul(da, dc)), flatten(mm), 2e-5);
  xylo::matrix into(std::array<std::size_t, 2>{M, N}, true);
  xylo::matmul_transposed(da, db, into);
  check(t + "matmul_transposed_into", flatten(into), flatten(mt), 2e-5);
  check(t + "transpose", flatten(::transpose(da)), flatten(::transpose(a)), 0.0);
  xylo::matrix s1 = ::transpose(da);
  check_i(t + "transpose_on_device", s1.on_device(), 1);
  check(t + "mat_add", flatten(da + da), flatten(a + a), 0.0);
  xylo::matrix dm(da);
  dm += 1.0f;
  dm *= da;
  xylo::matrix hm(a);
  hm += 1.0f;
  hm *= a;
  check(t + "mat_compound", flatten(dm), flatten(hm), 0.0);
  check(t + "row", xylo::matrix_view(da)[M / 2], xylo::matrix_view(a)[M / 2], 0.0);
}

}  // namespace

int main() {
  vectors(1000);
  vectors(1 << 20);
  vectors((1 << 22) + 3);  // an odd tail for the float4 maps
  gemms(13, 11, 17);
  gemms(300, 190, 257);
  gemms(1027, 65, 96);
  // the engine's draws land in a device vector as in a host one
  xylo::default_generator().seed(99);
  xylo::vector hn(100);
  normal_distribution(0.0f, 1.0f, hn);
  xylo::default_generator().seed(99);
  xylo::vector dn(100, true);
  normal_distribution(0.0f, 1.0f, dn);
  check("normal_draws", dn, hn, 0.0);
  xylo::vector p(5);
  for (int i = 0; i < 5; ++i) p[i] = 0.1f + 0.2f * i;
  xylo::default_generator().seed(5);
  const long h = (long)discrete_distribution(p);
  xylo::default_generator().seed(5);
  const long d = (long)discrete_distribution(xylo::to_device(p));
  check_i("discrete_draw", d, h);
  // a host operand and a device operand do not mix
  bool threw = false;
  try {
    xylo::vector x = rvec(8), y = xylo::to_device(rvec(8));
    (void)(x + y);
  } catch (const xeno::error &) {
    threw = true;
  }
  check_i("mixed_throws", threw, 1);
  std::printf("%s\n", g_fail ? "tensor_device FAILED" : "tensor_device ok");
  return g_fail ? 1 : 0;
}
