// Every operation of xylo/tensor.h, written against the reference's API only,
// so that this one source compiles unchanged against the reference
// (/root/reference/xylo/tensor.h + tensor.cc: tests/golden/make_tensor_golden.py
// writes tests/golden/tensor_ops.npz from that build) and against the drop-in
// layer (include/xylo_compat/xylo/tensor.h: make compat ->
// build/compat/tensor_ops, run by tests/test_gpu_tensor.py).
//
// Output: one line per result, "<name> f <n> v0 v1 ..." (floats, %.9g),
// "<name> i <n> v0 ..." (integers: sizes, shapes, indices, draws, flags) or
// "<name> s <text>" (streamable output).  The sizes cover both sides of the
// drop-in's device thresholds (GEMMs from 2^22 multiply-adds, reductions
// from 2^20 floats).
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include <xeno/exception.h>
#include <xylo/tensor.h>

namespace {

uint32_t g_state = 12345u;
float rnd() {  // [-1, 1), a fixed LCG (not the library's engine)
  g_state = g_state * 1664525u + 1013904223u;
  return (float)(g_state >> 8) / 16777216.0f * 2.0f - 1.0f;
}

void emit_f(const std::string &name, const float *p, std::size_t n) {
  std::printf("%s f %zu", name.c_str(), n);
  for (std::size_t i = 0; i < n; ++i) std::printf(" %.9g", (double)p[i]);
  std::printf("\n");
}
void emit_v(const std::string &name, xylo::vector_view v) {
  emit_f(name, v.data(), v.size());
}
// a matrix: its shape, then its values (above 8192 of them every k-th, k
// recorded: keeps the fixture small, the GEMM outputs are compared per entry)
void emit_m(const std::string &name, xylo::matrix_view m) {
  std::printf("%s_shape i 2 %zu %zu\n", name.c_str(), m.num_rows(), m.num_cols());
  xylo::vector_view f = m.flatten();
  const std::size_t k = f.size() > 8192 ? (f.size() + 8191) / 8192 : 1;
  if (k == 1) {
    emit_f(name, f.data(), f.size());
    return;
  }
  std::vector<float> s;
  for (std::size_t i = 0; i < f.size(); i += k) s.push_back(f[i]);
  std::printf("%s_stride i 1 %zu\n", name.c_str(), k);
  emit_f(name, s.data(), s.size());
}
void emit_s(const std::string &name, float x) { emit_f(name, &x, 1); }
void emit_i(const std::string &name, const std::vector<long> &v) {
  std::printf("%s i %zu", name.c_str(), v.size());
  for (long x : v) std::printf(" %ld", x);
  std::printf("\n");
}
void emit_t(const std::string &name, const std::string &text) {
  std::printf("%s s %s\n", name.c_str(), text.c_str());
}

xylo::matrix random_matrix(std::size_t r, std::size_t c) {
  xylo::matrix m(std::array<std::size_t, 2>{r, c});
  xylo::vector_view f = flatten(m);
  for (std::size_t i = 0; i < f.size(); ++i) f[i] = rnd();
  return m;
}
xylo::vector random_vector(std::size_t n, float lo = -1.0f, float hi = 1.0f) {
  xylo::vector v(n);
  for (std::size_t i = 0; i < n; ++i) v[i] = lo + (rnd() + 1.0f) * 0.5f * (hi - lo);
  return v;
}

template <class F> long throws(F f) {
  try {
    f();
  } catch (const xeno::error &) {
    return 1;
  }
  return 0;
}

// the GEMMs and the transpose (tensor.cc:209-230, 322-336)
void gemms(const std::string &tag, std::size_t M, std::size_t N, std::size_t K) {
  xylo::matrix a = random_matrix(M, K), b = random_matrix(N, K);
  xylo::matrix c = random_matrix(K, N);
  emit_m(tag + "_mt", ::matmul_transposed(a, b));
  xylo::matrix out(std::array<std::size_t, 2>{M, N});
  xylo::matmul_transposed(a, b, out);
  emit_m(tag + "_mt_into", out);
  emit_m(tag + "_mm", ::matmul(a, c));
  xylo::matrix out2(std::array<std::size_t, 2>{M, N});
  xylo::matmul(a, c, out2);
  emit_m(tag + "_mm_into", out2);
  emit_m(tag + "_tr", ::transpose(a));
  xylo::matrix t(std::array<std::size_t, 2>{K, M});
  xylo::transpose(a, t);
  emit_m(tag + "_tr_into", t);
}

// reductions and elementwise maps on vectors (tensor.cc:152-206, 256-317,
// 371-557)
void vectors(const std::string &tag, std::size_t n) {
  xylo::vector v1 = random_vector(n), v2 = random_vector(n, 0.5f, 2.0f);
  xylo::vector_view w1(v1), w2(v2);
  emit_s(tag + "_dot_m", w1.dot(w2));
  emit_s(tag + "_dot", dot(v1, v2));
  emit_s(tag + "_sum_m", w1.sum());
  emit_s(tag + "_sum", sum(v1));
  emit_s(tag + "_mean_m", w1.mean());
  emit_s(tag + "_mean", mean(v1));
  emit_s(tag + "_var_m", w1.variance());
  emit_s(tag + "_var", variance(v1));
  emit_s(tag + "_sd_m", w1.stddev());
  emit_s(tag + "_sd", stddev(v1));
  emit_s(tag + "_cv_m", w2.coef_variance());
  emit_s(tag + "_cv", coef_variance(v2));
  emit_s(tag + "_max", max(v1));
  emit_i(tag + "_argmax", {(long)w1.argmax(), (long)argmax(v1),
                           (long)argmax(v2)});
  if (n <= 4096) {  // the arithmetic operators (host maps at every size)
    emit_v(tag + "_add", v1 + v2);
    emit_v(tag + "_sub", v1 - v2);
    emit_v(tag + "_mul", v1 * v2);
    emit_v(tag + "_div", v1 / v2);
    emit_v(tag + "_add_s", v1 + 0.25f);
    emit_v(tag + "_sub_s", v1 - 0.25f);
    emit_v(tag + "_mul_s", v1 * 3.5f);
    emit_v(tag + "_div_s", v1 / 3.5f);
    emit_v(tag + "_abs", abs(v1));
    emit_v(tag + "_sin", sin(v1));
    emit_v(tag + "_exp", exp(v1));
    emit_v(tag + "_log", log(v2));
    emit_v(tag + "_sqrt", sqrt(v2));
    xylo::vector o(n);
    xylo::add(v1, v2, o);
    emit_v(tag + "_add_into", o);
    xylo::minus(v1, v2, o);
    emit_v(tag + "_sub_into", o);
    xylo::multiply(v1, v2, o);
    emit_v(tag + "_mul_into", o);
    xylo::divide(v1, v2, o);
    emit_v(tag + "_div_into", o);
    xylo::abs(v1, o);
    emit_v(tag + "_abs_into", o);
    xylo::sin(v1, o);
    emit_v(tag + "_sin_into", o);
    xylo::exp(v1, o);
    emit_v(tag + "_exp_into", o);
    xylo::log(v2, o);
    emit_v(tag + "_log_into", o);
    xylo::sqrt(v2, o);
    emit_v(tag + "_sqrt_into", o);
    xylo::vector c(v1);
    c += 1.5f;
    c -= v2;
    c *= 0.75f;
    c *= v2;
    c /= 1.25f;
    c /= v2;
    c -= 0.125f;
    c += v1;
    emit_v(tag + "_compound", c);
  }
}

}  // namespace

int main() {
  xylo::default_generator().seed(20241008);

  // shapes, views, indexing (tensor.h:69-422)
  xylo::tensor<3> t3({3, 4, 5});
  for (std::size_t i = 0; i < t3.size(); ++i) t3.data()[i] = (float)i;
  emit_i("t3_shape", {(long)t3.shape()[0], (long)t3.shape()[1],
                      (long)t3.shape()[2], (long)t3.rank(), (long)t3.size()});
  xylo::matrix_view t3_1 = t3[1];
  emit_m("t3_1", t3_1);
  emit_v("t3_1_2", t3[1][2]);
  xylo::tensor_view<3> v3(t3);
  emit_v("t3_flat", v3.flatten());
  emit_v("t3_view_2_3", v3[2][3]);
  xylo::matrix m = random_matrix(6, 7);
  xylo::matrix_view mv(m);
  emit_i("m_shape", {(long)mv.num_rows(), (long)mv.num_cols(), (long)mv.rank(),
                     (long)mv.size(), (long)m.rank(), (long)m.size()});
  long rows = 0;
  float rowsum = 0.0f;
  for (xylo::vector_view row : mv) {
    ++rows;
    rowsum += sum(row);
  }
  emit_i("m_rows", {rows});
  emit_s("m_rowsum", rowsum);
  emit_m("m_slice", slice(mv, 2, 3));
  emit_v("v_slice", slice(flatten(m), 5, 9));
  emit_m("m_fold", fold<2>(flatten(m), {7, 6}));
  emit_m("m_fold2", flatten(m).fold(14, 3));
  std::vector<float> raw(12);
  for (std::size_t i = 0; i < raw.size(); ++i) raw[i] = 0.5f * (float)i;
  xylo::vector_view borrowed = xylo::borrow_vector(raw);
  emit_i("borrowed", {(long)borrowed.borrowed(), (long)borrowed.size()});
  emit_m("borrowed_fold", borrowed.fold(3, 4));
  xylo::vector copied(borrowed);
  copied[3] = -1.0f;
  emit_v("copied", copied);
  emit_v("raw_after_copy", borrowed);

  // assignment (tensor.cc:128-136, 152-156)
  xylo::vector a(5);
  a = 2.5f;
  emit_v("assign_scalar", a);
  xylo::vector b = random_vector(5);
  a = xylo::vector_view(b);
  emit_v("assign_view", a);
  xylo::vector c5 = random_vector(5);
  a = c5;
  emit_v("assign_vector", a);
  xylo::vector_view av(a);
  av = 7.0f;
  emit_v("assign_view_scalar", a);
  xylo::matrix dst(std::array<std::size_t, 2>{2, 5});
  dst[0] = 0.0f;  // (the reference leaves fresh memory uninitialised)
  dst[1] = xylo::vector_view(b);
  emit_m("assign_row", dst);
  emit_i("shape_errors",
         {throws([&] { a = xylo::vector(4); }),
          throws([&] { dot(xylo::vector(3), xylo::vector(4)); }),
          throws([&] { xylo::vector o(2); xylo::add(b, c5, o); }),
          throws([&] { ::matmul_transposed(random_matrix(2, 3), random_matrix(2, 4)); }),
          throws([&] { xylo::matrix o(std::array<std::size_t, 2>{3, 3});
                       xylo::transpose(random_matrix(2, 3), o); })});

  // equality (tensor.cc:483-491)
  xylo::vector e1 = random_vector(9), e2(e1);
  xylo::vector_view ev1(e1);
  const bool eq_same = ev1 == xylo::vector_view(e1);
  const bool eq_copy = e1 == e2;
  e2[4] += 1.0f;
  const bool eq_diff = e1 == e2;
  const bool eq_size = e1 == xylo::vector(8);
  emit_i("equality", {eq_same, eq_copy, eq_diff, eq_size});

  // argmax keeps the first of equal maxima (tensor.cc:464-466)
  xylo::vector ties(6);
  ties = 1.0f;
  ties[2] = 3.0f;
  ties[4] = 3.0f;
  emit_i("argmax_ties", {(long)argmax(ties), (long)xylo::vector_view(ties).argmax()});

  // matrices: elementwise and compound (tensor.cc:232-251, 338-368)
  xylo::matrix m1 = random_matrix(5, 8), m2 = random_matrix(5, 8);
  emit_m("mat_add", m1 + m2);
  emit_m("mat_sub", m1 - m2);
  xylo::matrix mo(std::array<std::size_t, 2>{5, 8});
  xylo::add(m1, m2, mo);
  emit_m("mat_add_into", mo);
  xylo::minus(m1, m2, mo);
  emit_m("mat_sub_into", mo);
  xylo::multiply(m1, m2, mo);
  emit_m("mat_mul_into", mo);
  xylo::matrix m2p(m2);
  m2p += 3.0f;
  xylo::divide(m1, m2p, mo);
  emit_m("mat_div_into", mo);
  xylo::matrix mc(m1);
  mc += 0.5f;
  mc += m2;
  mc -= 0.25f;
  mc -= m1;
  mc *= 2.0f;
  mc *= m2;
  mc /= 4.0f;
  mc /= m2p;
  emit_m("mat_compound", mc);

  // the GEMMs on both sides of the device threshold (2^22 multiply-adds)
  gemms("g_small", 13, 11, 17);
  gemms("g_mid", 64, 48, 40);
  gemms("g_large", 300, 190, 257);
  gemms("g_tall", 1027, 65, 96);
  // reductions on both sides of theirs (2^20 floats)
  vectors("v_small", 1000);
  vectors("v_4k", 4096);
  vectors("v_large", 1100000);

  // the engine's distributions (tensor.cc:191-200, 467-481)
  xylo::vector nv(64), uv(64), nv2(32), uv2(32);
  normal_distribution(0.5f, 2.0f, nv);
  uniform_distribution(-3.0f, 1.0f, uv);
  xylo::vector_view(nv2).normal_distribution(1.0f, 0.5f);
  xylo::vector_view(uv2).uniform_distribution(2.0f, 4.0f);
  emit_v("normal", nv);
  emit_v("uniform", uv);
  emit_v("normal_m", nv2);
  emit_v("uniform_m", uv2);
  xylo::vector probs(7);
  for (std::size_t i = 0; i < 7; ++i) probs[i] = 0.05f + 0.1f * (float)i;
  std::vector<long> draws;
  for (int i = 0; i < 200; ++i) draws.push_back((long)discrete_distribution(probs));
  emit_i("discrete", draws);

  // streamable (tensor.h:489-523)
  xylo::vector sv(3);
  sv[0] = 1.5f;
  sv[1] = -2.0f;
  sv[2] = 0.125f;
  emit_t("streamable_v", xeno::string::streamable(xylo::vector_view(sv)));
  xylo::matrix sm(std::array<std::size_t, 2>{2, 2});
  flatten(sm) = 0.0f;
  flatten(sm)[0] = 1.0f;
  flatten(sm)[3] = 4.0f;
  std::string smt = xeno::string::streamable(xylo::matrix_view(sm));
  for (char &ch : smt)
    if (ch == '\n') ch = '|';
  emit_t("streamable_m", smt);
  std::printf("done i 1 1\n");
  return 0;
}
