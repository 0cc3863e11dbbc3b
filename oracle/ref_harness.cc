// oracle/ref_harness.cc -- TEST INFRASTRUCTURE ONLY (never part of the product).
//
// Drives the *real* reference (beehover/dependence_free_rl) compiled from its
// own sources under /root/reference (see oracle/Makefile, target `ref`), to
//   (1) emit golden vectors (tests/golden/*.npz via tests/golden/make_golden.py)
//   (2) time the reference's single-threaded CPU path (bench.py cpu_baseline,
//       kind "reference").
// Nothing here is copied from the reference: it only #includes the reference
// headers and links the reference's tensor.cc / logging.cc.
//
// Reference entry points exercised (file:line under /root/reference):
//   xylo::default_generator            xylo/tensor.cc:71-75
//   ::discrete_distribution            xylo/tensor.cc:467-470
//   bp::environment / bp::agent        apps/bin_packing/bin_packing.h:46-107
//   xylo::agent::step                  xylo/rl.h:325-349
//   xylo::replay_buffer                xylo/rl.h:213-296
//   xylo::actor_critic_learner         xylo/policy_gradient.h:150-287
//   xylo::ppo_learner                  xylo/policy_gradient.h:289-308
//   xylo::policy_gradient_learner      xylo/policy_gradient.h:89-148
//   xylo::model / layers / sgd         xylo/nn.h:60-628
//
// The 64-bin / 1-D / 3-D configurations of BASELINE.json cannot use
// bin_packing.h (num_bins is a constexpr 8, D is fixed at 2), so this harness
// supplies `gen_env<B,D>`: the same environment semantics generalised to B bins
// and D dims (capacity 8 per dim; items (4,2)/(1,2) at D=2, (4)/(1) at D=1,
// (4,2,2)/(1,2,1) at D=3; P(first)=0.4).  mode=envcheck proves gen_env<8,2>
// produces bit-identical trajectories and RNG consumption to bp::environment,
// and that gen_env<64,2> / gen_env<128,2> reproduce it on any 8 of their bins
// (envcheck_injected).  D = 1 and D = 3 have no reference env to compare with.
//
// XH_REF_BP64 (oracle/Makefile, ref_harness_bp64): the same harness compiled
// against a copy of the reference's apps/bin_packing/bin_packing.h whose only
// change is num_bins (:12) = 64, generated in a scratch directory of the
// build and deleted after it (never committed, never shipped).  Its learn /
// bench modes at B = 64, D = 2 then drive the reference's own bp::environment
// and bp::agent -- BASELINE config 3's env pinned by the reference's code,
// not by gen_env.  Only those modes exist in that build.
#ifndef XH_REF_BP64
#define XH_REF_BP64 0
#endif
#include <apps/bin_packing/bin_packing.h>  // pulls xylo/nn.h, rl.h, policy_gradient.h
#if XH_REF_BP64
static_assert(bp::num_bins == 64, "ref_harness_bp64: bin_packing.h copy with num_bins = 64");
#endif

#include <xeno/sys/file_descriptor.h>

// The heuristic policies of the reference's own agent programs
// (firstfit_agent.cc:10-28, bestfit_agent.cc:10-30, minwaste_agent.cc:10-39),
// compiled from those files where they lie; their main() is renamed and never
// called (mode=heuristic drives the policies with a seeded engine instead).
#if !XH_REF_BP64
namespace ref_firstfit {
#define main firstfit_main
#include <apps/bin_packing/firstfit_agent.cc>
#undef main
}  // namespace ref_firstfit
namespace ref_bestfit {
#define main bestfit_main
#include <apps/bin_packing/bestfit_agent.cc>
#undef main
}  // namespace ref_bestfit
namespace ref_minwaste {
#define main minwaste_main
#include <apps/bin_packing/minwaste_agent.cc>
#undef main
}  // namespace ref_minwaste
#endif

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace {

// ---------------------------------------------------------------- output ---
// Record file: repeated [u32 name_len][name][u8 dtype][u32 ndim][u64 dims..][raw]
struct recorder {
  FILE *f = nullptr;
  explicit recorder(const std::string &path) {
    f = std::fopen(path.c_str(), "wb");
    if (!f) {
      std::perror("open out");
      std::exit(2);
    }
  }
  ~recorder() {
    if (f) std::fclose(f);
  }
  void put(const std::string &name, char dt, const std::vector<uint64_t> &dims,
           const void *data, std::size_t elsize) {
    uint32_t nl = name.size();
    std::fwrite(&nl, 4, 1, f);
    std::fwrite(name.data(), 1, nl, f);
    std::fwrite(&dt, 1, 1, f);
    uint32_t nd = dims.size();
    std::fwrite(&nd, 4, 1, f);
    uint64_t n = 1;
    for (auto d : dims) {
      std::fwrite(&d, 8, 1, f);
      n *= d;
    }
    if (n) std::fwrite(data, elsize, n, f);
  }
  void f32(const std::string &n, const std::vector<float> &v,
           std::vector<uint64_t> dims = {}) {
    if (dims.empty()) dims = {v.size()};
    put(n, 'f', dims, v.data(), 4);
  }
  void f64(const std::string &n, const std::vector<double> &v) {
    put(n, 'd', {v.size()}, v.data(), 8);
  }
  void i32(const std::string &n, const std::vector<int32_t> &v,
           std::vector<uint64_t> dims = {}) {
    if (dims.empty()) dims = {v.size()};
    put(n, 'i', dims, v.data(), 4);
  }
  void u32(const std::string &n, const std::vector<uint32_t> &v) {
    put(n, 'u', {v.size()}, v.data(), 4);
  }
};

std::map<std::string, std::string> parse_args(int argc, char **argv) {
  std::map<std::string, std::string> m;
  for (int i = 2; i < argc; ++i) {
    std::string a = argv[i];
    auto p = a.find('=');
    if (p == std::string::npos) continue;
    m[a.substr(0, p)] = a.substr(p + 1);
  }
  return m;
}
long iarg(std::map<std::string, std::string> &m, const char *k, long d) {
  return m.count(k) ? std::stol(m[k]) : d;
}
double darg(std::map<std::string, std::string> &m, const char *k, double d) {
  return m.count(k) ? std::stod(m[k]) : d;
}
std::vector<int> listarg(std::map<std::string, std::string> &m, const char *k,
                         std::vector<int> d) {
  if (!m.count(k)) return d;
  std::vector<int> r;
  std::stringstream ss(m[k]);
  std::string tok;
  while (std::getline(ss, tok, ',')) r.push_back(std::stoi(tok));
  return r;
}

uint32_t engine_state() {
  std::ostringstream os;
  os << xylo::default_generator();
  return static_cast<uint32_t>(std::stoul(os.str()));
}

std::vector<float> to_std(xylo::vector_view v) {
  return std::vector<float>(v.begin(), v.end());
}
std::vector<float> to_std(const xylo::matrix &m) {
  xylo::matrix_view mv(m);
  xylo::vector_view f = mv.flatten();
  return std::vector<float>(f.begin(), f.end());
}

// --------------------------------------------- generalised environment -----
template <std::size_t D> struct item_table;
template <> struct item_table<1> {
  static constexpr std::array<int, 1> a{4}, b{1};
};
template <> struct item_table<2> {
  static constexpr std::array<int, 2> a{4, 2}, b{1, 2};
};
template <> struct item_table<3> {
  static constexpr std::array<int, 3> a{4, 2, 2}, b{1, 2, 1};
};
constexpr int kCapacity = 8;

template <std::size_t B, std::size_t D> struct gen_obs {
  static std::size_t length() { return 2 * D * B; }
  std::array<std::array<int, D>, B> bins{};
  std::array<int, D> item{};
  // Tags (not part of the observation vector): which env / how many applies.
  int tag_env = -1;
  int tag_step = -1;
  void to_vector(xylo::vector_view o) const {
    xylo::matrix_view m = xylo::fold<2>(o, {B, 2 * D});
    for (std::size_t i = 0; i < B; ++i)
      for (std::size_t d = 0; d < D; ++d) {
        m[i][d] = float(bins[i][d]) / kCapacity;
        m[i][D + d] = float(item[d]) / kCapacity;
      }
  }
};

struct step_log {
  int env, step;
  std::vector<int> bins, item;  // state before apply
  int choice;
  std::vector<float> distrib;
  int done;
};

template <std::size_t B, std::size_t D>
class gen_env
    : public xylo::environment<xylo::discrete_action<B>, gen_obs<B, D>> {
public:
  using A = xylo::discrete_action<B>;
  using S = gen_obs<B, D>;
  gen_env(int index, std::vector<step_log> *log)
      : index_(index), log_(log), dist_(0.4) {
    fill_bins();
    get_item();
  }
  void apply(const A &a, std::size_t) override {
    if (log_) {
      step_log l;
      l.env = index_;
      l.step = steps_;
      for (auto &b : s_.bins)
        for (auto v : b) l.bins.push_back(v);
      for (auto v : s_.item) l.item.push_back(v);
      l.choice = a.choice;
      if (a.distrib) l.distrib = to_std(*a.distrib);
      l.done = 0;
      log_->push_back(l);
    }
    ++steps_;
    auto &bin = s_.bins[a.choice];
    bool neg = false;
    for (std::size_t d = 0; d < D; ++d) {
      bin[d] -= s_.item[d];
      neg |= bin[d] < 0;
    }
    if (neg) {
      if (log_) log_->back().done = 1;
      return;
    }
    get_item();
  }
  S view(std::size_t) const override {
    S s = s_;
    s.tag_env = index_;
    s.tag_step = steps_;
    return s;
  }
  void reset(std::size_t) override {
    fill_bins();
    get_item();
  }

private:
  void fill_bins() {
    for (auto &b : s_.bins) b.fill(kCapacity);
  }
  void get_item() {
    s_.item = dist_(xylo::default_generator()) ? item_table<D>::a
                                               : item_table<D>::b;
  }
  int index_;
  int steps_ = 0;
  std::vector<step_log> *log_;
  S s_;
  std::bernoulli_distribution dist_;
};

template <std::size_t B, std::size_t D>
class gen_agent
    : public xylo::agent<xylo::discrete_action<B>, gen_obs<B, D>> {
public:
  using base = xylo::agent<xylo::discrete_action<B>, gen_obs<B, D>>;
  using base::base;

private:
  bool game_over(const gen_obs<B, D> &ob) override {
    for (const auto &b : ob.bins)
      for (auto v : b)
        if (v < 0) return true;
    return false;
  }
  float get_reward(const gen_obs<B, D> &, const gen_obs<B, D> &ob) override {
    return game_over(ob) ? 0.0f : 1.0f;
  }
};

// Records every flat gradient handed to the optimizer (nn.h:594-605); the
// update itself is the reference optimizer's own next_parameters.
struct grad_log {
  std::vector<std::vector<float>> grads;
  bool record = true;
};

template <class Base>
struct recording : Base, grad_log {
  template <class... Args>
  recording(xylo::model &m, Args... args) : Base(m, args...) {}

protected:
  xylo::vector next_parameters(const xylo::vector &p, const xylo::vector &g,
                               float rate) override {
    if (record) grads.push_back(std::vector<float>(g.begin(), g.end()));
    return Base::next_parameters(p, g, rate);
  }
};
using recording_sgd = recording<xylo::sgd_optimizer>;

// opt = sgd | momentum | adam (nn.h:616-698).  Owns the concrete object
// (xylo::optimizer has no virtual destructor).
struct opt_holder {
  std::unique_ptr<recording_sgd> sgd;
  std::unique_ptr<recording<xylo::momentum_optimizer>> mom;
  std::unique_ptr<recording<xylo::adam_optimizer>> adam;
  xylo::optimizer *opt = nullptr;
  grad_log *log = nullptr;
  opt_holder(const std::string &kind, xylo::model &m, float lr, float wd) {
    if (kind == "momentum") {
      mom = std::make_unique<recording<xylo::momentum_optimizer>>(m, lr);
      opt = mom.get();
      log = mom.get();
    } else if (kind == "adam") {
      adam = std::make_unique<recording<xylo::adam_optimizer>>(m, lr);
      opt = adam.get();
      log = adam.get();
    } else {
      sgd = std::make_unique<recording_sgd>(m, lr, wd);
      opt = sgd.get();
      log = sgd.get();
    }
  }
};

// --------------------------------------------------------------- models ----
enum head_kind { head_none = 0, head_softmax = 1, head_softmax_xent = 2 };

void build_perbin(xylo::model &m, int in, const std::vector<int> &widths,
                  head_kind head) {
  int prev = in;
  for (int w : widths) {
    m.add_layer(std::make_unique<xylo::convolution1d_1_layer>(prev, w));
    m.add_layer(std::make_unique<xylo::relu_activation>());
    prev = w;
  }
  m.add_layer(std::make_unique<xylo::convolution1d_1_layer>(prev, 1));
  if (head == head_softmax)
    m.add_layer(std::make_unique<xylo::softmax_layer>());
  else if (head == head_softmax_xent)
    m.add_layer(std::make_unique<xylo::softmax_cross_entropy_layer>());
}

void build_full(xylo::model &m, int in, const std::vector<int> &widths, int out,
                head_kind head) {
  int prev = in;
  for (int w : widths) {
    m.add_layer(std::make_unique<xylo::full_layer>(prev, w));
    m.add_layer(std::make_unique<xylo::relu_activation>());
    prev = w;
  }
  m.add_layer(std::make_unique<xylo::full_layer>(prev, out));
  if (head == head_softmax)
    m.add_layer(std::make_unique<xylo::softmax_layer>());
  else if (head == head_softmax_xent)
    m.add_layer(std::make_unique<xylo::softmax_cross_entropy_layer>());
}

#if !XH_REF_BP64
// ------------------------------------------------------------ mode: rng ----
int mode_rng(std::map<std::string, std::string> &a) {
  recorder rec(a["out"]);
  uint32_t seed = iarg(a, "seed", 42);
  long n = iarg(a, "n", 100000);
  auto &g = xylo::default_generator();

  g.seed(seed);
  std::vector<uint32_t> raw(n);
  for (auto &v : raw) v = g();
  rec.u32("raw", raw);

  g.seed(seed);
  std::vector<double> canon(n);
  for (auto &v : canon) v = std::generate_canonical<double, 53>(g);
  rec.f64("canonical", canon);

  g.seed(seed);
  std::bernoulli_distribution bd(0.4);
  std::vector<int32_t> bern(n);
  for (auto &v : bern) v = bd(g);
  rec.i32("bernoulli", bern);

  // discrete_distribution (tensor.cc:467-470) over float probability vectors
  // of several widths. Probabilities come from an independent mt19937 so the
  // minstd stream is consumed by the sampler only.
  for (int width : {8, 32, 64, 128}) {
    std::mt19937 pg(width);
    std::uniform_real_distribution<float> u(0.0f, 1.0f);
    long m = n / 4;
    std::vector<float> probs(m * width);
    std::vector<int32_t> pick(m);
    g.seed(seed + width);
    for (long i = 0; i < m; ++i) {
      xylo::vector v({(std::size_t)width});
      float s = 0;
      for (int j = 0; j < width; ++j) {
        float x = u(pg);
        // Make a few probability vectors very peaked / sparse.
        if (i % 7 == 0) x = x * x * x * x;
        if (i % 11 == 0 && j % 3 == 0) x = 0.0f;
        v[j] = x;
        s += x;
      }
      for (int j = 0; j < width; ++j) {
        v[j] = v[j] / s;
        probs[i * width + j] = v[j];
      }
      pick[i] = ::discrete_distribution(v);
    }
    rec.f32("disc_probs_" + std::to_string(width), probs,
            {(uint64_t)m, (uint64_t)width});
    rec.i32("disc_pick_" + std::to_string(width), pick);
    rec.u32("disc_state_after_" + std::to_string(width), {engine_state()});
  }
  return 0;
}

// ------------------------------------------------------- mode: envcheck ----
// A uniform 8-way choice (random_policy<8>'s react: the same engine draws)
// placed on 8 distinct bins `slot` of a B-bin env.
template <std::size_t B>
class injected_policy
    : public xylo::policy<xylo::discrete_action<B>, gen_obs<B, 2>> {
public:
  explicit injected_policy(const std::vector<int> &slot) : slot_(slot) {}
  xylo::discrete_action<B> react(const gen_obs<B, 2> &) const override {
    xylo::random_policy<8, gen_obs<8, 2>> rp;
    xylo::discrete_action<B> a;
    a.choice = slot_[rp.react(gen_obs<8, 2>{}).choice];
    return a;
  }

private:
  std::vector<int> slot_;
};

// gen_env<B,2> (B = 64, 128: the benchmark shapes) driven by the reference
// run's choices placed on 8 random distinct bins: those bins must follow the
// reference env's 8 bins transition for transition, every other bin must stay
// full, and rewards, episode ends and the engine must agree.  With the slots
// redrawn per seed, every bin index of the larger env gets exercised.
template <std::size_t B>
bool envcheck_injected(uint32_t seed, long steps, uint32_t x_end,
                       const std::vector<int32_t> &choice,
                       const std::vector<int32_t> &reward,
                       const std::vector<int32_t> &end_bins) {
  std::vector<int> perm(B);
  for (std::size_t i = 0; i < B; ++i) perm[i] = (int)i;
  std::mt19937 pick(seed * 7919u + (uint32_t)B);
  std::shuffle(perm.begin(), perm.end(), pick);
  std::vector<int> slot(perm.begin(), perm.begin() + 8);

  auto &g = xylo::default_generator();
  g.seed(seed);
  injected_policy<B> pol(slot);
  gen_env<B, 2> genv(0, nullptr);
  xylo::replay_buffer<xylo::discrete_action<B>, gen_obs<B, 2>> rb;
  gen_agent<B, 2> ag(pol, genv, rb);
  for (long i = 0; i < steps; ++i) ag.step();
  bool same = engine_state() == x_end;
  std::vector<int> owner(B, -1);
  for (int b = 0; b < 8; ++b) owner[slot[b]] = b;
  std::size_t k = 0;
  for (auto &traj : rb.sample_td())
    for (auto &tr : traj) {
      if (k >= choice.size()) return false;
      same &= tr.action.choice == (std::size_t)slot[choice[k]];
      same &= (int)tr.reward == reward[k];
      for (std::size_t b = 0; b < B; ++b)
        for (int d = 0; d < 2; ++d) {
          int want = owner[b] < 0 ? kCapacity
                                  : end_bins[(k * 8 + owner[b]) * 2 + d];
          same &= tr.end_state.bins[b][d] == want;
        }
      ++k;
    }
  return same && k == choice.size();
}

// bp::environment (the reference env) vs gen_env<8,2>: identical trajectories;
// vs gen_env<64,2> and gen_env<128,2> through envcheck_injected.
int mode_envcheck(std::map<std::string, std::string> &a) {
  recorder rec(a["out"]);
  uint32_t seed = iarg(a, "seed", 7);
  long steps = iarg(a, "steps", 20000);
  auto &g = xylo::default_generator();

  xylo::random_policy<bp::num_bins, bp::observation> rp;
  xylo::random_policy<8, gen_obs<8, 2>> rp2;

  g.seed(seed);
  uint32_t x0 = engine_state();
  bp::environment env;
  xylo::replay_buffer<bp::action, bp::observation> rb;
  bp::agent ag(rp, env, rb);
  for (long i = 0; i < steps; ++i) ag.step();
  uint32_t x_end = engine_state();

  std::vector<int32_t> start_bins, start_item, choice, reward, end_bins,
      end_item, frozen;
  for (auto &traj : rb.sample_td()) {
    for (auto &tr : traj) {
      for (auto &b : tr.start_state->bins) {
        start_bins.push_back(b.first);
        start_bins.push_back(b.second);
      }
      start_item.push_back(tr.start_state->item.first);
      start_item.push_back(tr.start_state->item.second);
      choice.push_back(tr.action.choice);
      reward.push_back((int)tr.reward);
      for (auto &b : tr.end_state.bins) {
        end_bins.push_back(b.first);
        end_bins.push_back(b.second);
      }
      end_item.push_back(tr.end_state.item.first);
      end_item.push_back(tr.end_state.item.second);
      frozen.push_back(traj.frozen());
    }
  }
  uint64_t nt = choice.size();
  rec.u32("x0", {x0});
  rec.u32("x_end", {x_end});
  rec.i32("start_bins", start_bins, {nt, 8, 2});
  rec.i32("start_item", start_item, {nt, 2});
  rec.i32("choice", choice);
  rec.i32("reward", reward);
  rec.i32("end_bins", end_bins, {nt, 8, 2});
  rec.i32("end_item", end_item, {nt, 2});
  rec.i32("frozen", frozen);

  // The same with the generalised env: must be bit-identical.
  g.seed(seed);
  gen_env<8, 2> genv(0, nullptr);
  xylo::replay_buffer<xylo::discrete_action<8>, gen_obs<8, 2>> rb2;
  gen_agent<8, 2> ag2(rp2, genv, rb2);
  for (long i = 0; i < steps; ++i) ag2.step();
  std::size_t k = 0;
  bool same = engine_state() == x_end;
  for (auto &traj : rb2.sample_td())
    for (auto &tr : traj) {
      same &= tr.action.choice == (std::size_t)choice[k];
      for (int b = 0; b < 8; ++b)
        for (int d = 0; d < 2; ++d)
          same &= tr.end_state.bins[b][d] == end_bins[(k * 8 + b) * 2 + d];
      ++k;
    }
  same &= k == nt;
  rec.i32("gen_env_identical", {same ? 1 : 0});
  bool same64 = envcheck_injected<64>(seed, steps, x_end, choice, reward, end_bins);
  bool same128 = envcheck_injected<128>(seed, steps, x_end, choice, reward, end_bins);
  rec.i32("gen_env64_identical", {same64 ? 1 : 0});
  rec.i32("gen_env128_identical", {same128 ? 1 : 0});
  std::fprintf(stderr,
               "envcheck: %llu transitions, gen_env identical=%d, "
               "gen_env<64,2> injected=%d, gen_env<128,2> injected=%d\n",
               (unsigned long long)nt, same, same64, same128);
  return same && same64 && same128 ? 0 : 1;
}

// -------------------------------------------------------- mode: deep -------
// apps/bin_packing/deep_agent.cc: weights.20, argmax policy, seed-driven.
int mode_deep(std::map<std::string, std::string> &a) {
  recorder rec(a["out"]);
  uint32_t seed = iarg(a, "seed", 1);
  long episodes = iarg(a, "episodes", 1000);
  // main=1: exactly deep_agent.cc's order -- the engine is seeded before the
  // model is built (its He init draws), no logits section, no reseed.
  const bool as_main = iarg(a, "main", 0) != 0;
  if (as_main) xylo::default_generator().seed(seed);
  xylo::model m;
  build_perbin(m, 4, {128, 64}, head_none);
  xeno::sys::mmap f = xeno::sys::mmap<float>(a["weights"]);
  xylo::vector_view v = xylo::borrow_vector(f.span());
  m.set_parameters(v);
  rec.f32("params", to_std(m.parameters()));
  if (!as_main) {
  // Logits for a few fixed observations (bins, item) -> golden Dense forward.
  std::vector<float> obs_all, logits_all;
  xylo::default_generator().seed(seed + 1000);
  std::mt19937 sg(5);
  for (int i = 0; i < 64; ++i) {
    bp::observation o(bp::environment::capacity);
    for (auto &b : o.bins) {
      b.first = (int)(sg() % 9);
      b.second = (int)(sg() % 9);
    }
    o.item = (sg() % 2) ? std::pair<int, int>{4, 2} : std::pair<int, int>{1, 2};
    if (i == 0) {
      for (auto &b : o.bins) b = {8, 8};
      o.item = {4, 2};
    }
    xylo::vector x = xylo::to_vector(o);
    xylo::matrix z = m.eval(xylo::fold<2>(x, {1, x.size()}));
    for (float q : x) obs_all.push_back(q);
    for (float q : to_std(z)) logits_all.push_back(q);
  }
  rec.f32("obs", obs_all, {64, 32});
  rec.f32("logits", logits_all, {64, 8});
  xylo::default_generator().seed(seed);
  }
  uint32_t x0 = engine_state();
  xylo::policy_gradient_deterministic_policy<bp::action, bp::observation> pol(
      m);
  bp::environment env;
  xylo::replay_buffer<bp::action, bp::observation> rb;
  bp::agent ag(pol, env, rb);
  for (long i = 0; i < episodes; ++i) ag.play_one_episode();
  auto exp = rb.sample_td();
  float total = xylo::total_rewards<bp::action, bp::observation>(exp);
  std::vector<int32_t> lens;
  for (auto &t : exp) lens.push_back(t.size());
  rec.u32("x0", {x0});
  rec.f32("total_reward", {total});
  rec.i32("episode_len", lens);
  std::fprintf(stderr, "deep: %ld episodes total reward %g\n", episodes,
               total);
  return 0;
}

// ------------------------------------------------------ mode: driver -------
// The model + env construction prologue of ppo_training.cc:9-43 (algo=ppo)
// or ac_training.cc (algo=ac) after seeding the engine: initial parameters
// and the engine state once the workers' envs exist.  Pins the drop-in
// layer's initialisation against the reference's (tests/test_compat.py).
int mode_driver(std::map<std::string, std::string> &a) {
  recorder rec(a["out"]);
  xylo::default_generator().seed(iarg(a, "seed", 1));
  const bool ac = a["algo"] == "ac";
  xylo::model pol, val;
  build_perbin(pol, 4, ac ? std::vector<int>{64, 32} : std::vector<int>{128, 64},
               ac ? head_softmax_xent : head_softmax);
  build_full(val, 4 * bp::num_bins, {64, 32}, 1, head_none);
  const uint32_t x_models = engine_state();
  std::vector<bp::environment> envs;
  const long n = iarg(a, "workers", ac ? 16 : 8);
  envs.reserve(n);
  for (long i = 0; i < n; ++i) envs.emplace_back();
  rec.f32("policy_init", to_std(pol.parameters()));
  rec.f32("value_init", to_std(val.parameters()));
  rec.u32("x_models", {x_models});
  rec.u32("x_envs", {engine_state()});
  std::vector<int32_t> items;
  for (auto &e : envs) {
    bp::observation o = e.view(0);
    items.push_back(o.item.first);
    items.push_back(o.item.second);
  }
  rec.i32("items", items);
  return 0;
}

// ------------------------------------------------------ mode: random -------
// random_agent.cc's loop (rounds x 100 episodes of xylo::random_policy),
// seeded: per-round average reward.
int mode_random(std::map<std::string, std::string> &a) {
  recorder rec(a["out"]);
  xylo::default_generator().seed(iarg(a, "seed", 1));
  const long rounds = iarg(a, "rounds", 3), episodes = iarg(a, "episodes", 100);
  std::vector<float> avg;
  for (long r = 0; r < rounds; ++r) {
    xylo::random_policy<bp::num_bins, bp::observation> policy;
    bp::environment env;
    xylo::replay_buffer<bp::action, bp::observation> rb;
    bp::agent agent(policy, env, rb);
    for (long i = 0; i < episodes; ++i) agent.play_one_episode();
    auto exp = rb.sample_td();
    avg.push_back(xylo::total_rewards<bp::action, bp::observation>(exp) /
                  double(episodes));
    rb.forget();
  }
  rec.f32("round_avg", avg);
  return 0;
}

// ---------------------------------------------------- mode: heuristic ------
// The agent programs' loop (firstfit_agent.cc:30-46 & co.): per round a new
// env + replay buffer, `episodes` episodes, average reward; seeded.  Records
// the per-round averages and round 0's episode lengths.
int mode_heuristic(std::map<std::string, std::string> &a) {
  recorder rec(a["out"]);
  xylo::default_generator().seed(iarg(a, "seed", 1));
  const long rounds = iarg(a, "rounds", 2), episodes = iarg(a, "episodes", 100);
  const std::string kind = a["policy"];
  ref_firstfit::firstfit_policy ff;
  ref_bestfit::bestfit_policy bf;
  ref_minwaste::minwaste_policy mw;
  xylo::random_policy<bp::num_bins, bp::observation> rnd;
  const xylo::policy<bp::action, bp::observation> *pol =
      kind == "firstfit" ? (const xylo::policy<bp::action, bp::observation> *)&ff
      : kind == "bestfit" ? (const xylo::policy<bp::action, bp::observation> *)&bf
      : kind == "minwaste"
          ? (const xylo::policy<bp::action, bp::observation> *)&mw
          : (const xylo::policy<bp::action, bp::observation> *)&rnd;
  std::vector<float> avg;
  std::vector<int32_t> lens;
  std::vector<uint32_t> x_round;
  for (long r = 0; r < rounds; ++r) {
    x_round.push_back(engine_state());
    bp::environment env;
    xylo::replay_buffer<bp::action, bp::observation> rb;
    bp::agent agent(*pol, env, rb);
    for (long i = 0; i < episodes; ++i) agent.play_one_episode();
    auto exp = rb.sample_td();
    avg.push_back(xylo::total_rewards<bp::action, bp::observation>(exp) /
                  double(episodes));
    if (r == 0)
      for (auto &t : exp) lens.push_back(t.size());
    rb.forget();
  }
  rec.f32("round_avg", avg);
  rec.i32("episode_len", lens);
  rec.u32("x_round", x_round);
  return 0;
}

#endif  // !XH_REF_BP64

// ------------------------------------------------------- mode: learn -------
struct learn_cfg {
  std::string algo;  // ppo | klppo | ac | pg
  int N, T, iters;
  std::vector<int> widths, vwidths;
  float lr_pi, lr_v, wd_pi, wd_v, gamma;
  uint32_t seed;
  bool record;
  int episodes;  // pg: episodes per worker per iteration
  std::string opt_pi = "sgd", opt_v = "sgd";  // sgd | momentum | adam
};

// The env / agent / observation types a learner run drives: the reference's
// own bp::environment / bp::agent where the shape is theirs (D = 2 and B =
// bp::num_bins: 8 in the plain build, 64 in the XH_REF_BP64 build), gen_env
// for every other shape.
template <std::size_t B, std::size_t D> struct gen_world {
  using A = xylo::discrete_action<B>;
  using S = gen_obs<B, D>;
  using env = gen_env<B, D>;
  using agent = gen_agent<B, D>;
  static constexpr bool real_env = false;
  static void bins_of(const S &s, std::vector<int32_t> &out) {
    for (auto &b : s.bins) out.insert(out.end(), b.begin(), b.end());
  }
  static void item_of(const S &s, std::vector<int32_t> &out) {
    out.insert(out.end(), s.item.begin(), s.item.end());
  }
};

// bp::environment with the per-apply log the golden's step records come from
// (the env's own apply runs unchanged).
class logged_bp_env : public bp::environment {
public:
  logged_bp_env(int index, std::vector<step_log> *log)
      : index_(index), log_(log) {}
  void apply(const bp::action &a, std::size_t id) override {
    if (log_) {
      step_log l;
      l.env = index_;
      l.step = steps_;
      const bp::observation s = view(id);
      for (auto &b : s.bins) {
        l.bins.push_back(b.first);
        l.bins.push_back(b.second);
      }
      l.item = {s.item.first, s.item.second};
      l.choice = a.choice;
      if (a.distrib) l.distrib = to_std(*a.distrib);
      l.done = 0;
      log_->push_back(l);
    }
    ++steps_;
    bp::environment::apply(a, id);
    if (log_)
      for (auto &b : view(id).bins)
        if (b.first < 0 || b.second < 0) log_->back().done = 1;
  }

private:
  int index_;
  int steps_ = 0;
  std::vector<step_log> *log_;
};

struct bp_world {
  using A = bp::action;
  using S = bp::observation;
  using env = logged_bp_env;
  using agent = bp::agent;
  static constexpr bool real_env = true;
  static void bins_of(const S &s, std::vector<int32_t> &out) {
    for (auto &b : s.bins) {
      out.push_back(b.first);
      out.push_back(b.second);
    }
  }
  static void item_of(const S &s, std::vector<int32_t> &out) {
    out.push_back(s.item.first);
    out.push_back(s.item.second);
  }
};

// The replay buffer's trajectory list (rl.h:213-296) replayed from the apply
// log: a trajectory opens at an env's first step and after each game over,
// forget() drops the frozen ones and keeps the open ones from their last
// state.  Gives each learner row its (env, step) when the observation type
// carries no tags (bp::observation).
struct traj_book {
  struct entry {
    int env, start, n;
    bool frozen;
  };
  std::vector<entry> list;
  std::vector<int> open;
  explicit traj_book(int n_env) : open(n_env, -1) {}
  void on_apply(const step_log &l) {
    int &o = open[l.env];
    if (o < 0) {
      list.push_back({l.env, l.step, 0, false});
      o = (int)list.size() - 1;
    }
    ++list[o].n;
    if (l.done) {
      list[o].frozen = true;
      o = -1;
    }
  }
  void forget() {
    std::vector<entry> keep;
    std::fill(open.begin(), open.end(), -1);
    for (auto e : list) {
      if (e.frozen) continue;
      e.start += e.n;
      e.n = 0;
      open[e.env] = (int)keep.size();
      keep.push_back(e);
    }
    list = std::move(keep);
  }
};

template <class W, std::size_t B, std::size_t D>
int run_learn(learn_cfg c, recorder *rec, double *steps_per_s) {
  using A = typename W::A;
  using S = typename W::S;
  auto &g = xylo::default_generator();
  g.seed(c.seed);
  const int f0 = 2 * D;

  xylo::model pol, val;
  const bool pg = c.algo == "pg";
  if (pg)
    build_full(pol, B * f0, c.widths, B, head_softmax_xent);
  else
    build_perbin(pol, f0, c.widths,
                 c.algo == "ac" ? head_softmax_xent : head_softmax);
  if (!pg) build_full(val, B * f0, c.vwidths, 1, head_none);
  opt_holder hold_pi(c.opt_pi, pol, c.lr_pi, c.wd_pi),
      hold_v(c.opt_v, val, c.lr_v, c.wd_v);
  grad_log *log_pi = hold_pi.log, *log_v = hold_v.log;
  xylo::optimizer &opt_pi = *hold_pi.opt, &opt_v = *hold_v.opt;
  log_pi->record = log_v->record = rec != nullptr;

  if (rec) {
    rec->f32("init_policy", to_std(pol.parameters()));
    if (!pg) rec->f32("init_value", to_std(val.parameters()));
  }
  const uint32_t x0 = engine_state();
  if (rec) {
    rec->u32("x0", {x0});
    // 1: the reference's own bp::environment / bp::agent drove this run
    rec->i32("env_is_reference", {W::real_env ? 1 : 0});
  }

  std::vector<step_log> log;
  std::vector<typename W::env> envs;
  envs.reserve(c.N);
  for (int i = 0; i < c.N; ++i) envs.emplace_back(i, rec ? &log : nullptr);
  traj_book book(c.N);
  xylo::replay_buffer<A, S> rb;
  xylo::policy_gradient_policy<A, S> policy(pol);
  std::vector<typename W::agent> agents;
  agents.reserve(c.N);
  for (int i = 0; i < c.N; ++i) agents.emplace_back(policy, envs[i], rb);

  std::unique_ptr<xylo::actor_critic_learner<A, S>> ac;
  std::unique_ptr<xylo::policy_gradient_learner<A, S>> pgl;
  if (c.algo == "ppo")
    ac = std::make_unique<xylo::ppo_learner<A, S>>(rb, pol, opt_pi, val, opt_v,
                                                   c.gamma);
  else if (c.algo == "klppo")  // ppo2_training.cc
    ac = std::make_unique<xylo::kl_ppo_learner<A, S>>(rb, pol, opt_pi, val,
                                                      opt_v, c.gamma);
  else if (c.algo == "ac")
    ac = std::make_unique<xylo::actor_critic_learner<A, S>>(
        rb, pol, opt_pi, val, opt_v, c.gamma);
  else
    pgl = std::make_unique<xylo::policy_gradient_learner<A, S>>(rb, pol,
                                                                opt_pi,
                                                                c.gamma);

  long total_steps = 0;
  double secs = 0;
  for (int it = 0; it < c.iters; ++it) {
    std::string p = "it" + std::to_string(it) + "_";
    std::size_t log0 = log.size();
    auto t0 = std::chrono::steady_clock::now();
    // Rollout: workers stepped one after another (the deterministic order).
    for (auto &agt : agents) {
      if (pg) {
        for (int e = 0; e < c.episodes; ++e) agt.play_one_episode();
      } else {
        agt.play_steps(c.T);
      }
    }
    std::size_t n_steps = 0;
    for (auto &traj : rb.sample_td()) n_steps += traj.size();
    total_steps += n_steps;

    if (!rec) {
      // Timed path: the reference learner, untouched.
      if (pg)
        pgl->step();
      else
        ac->step();
      rb.forget();
      secs += std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                            t0)
                  .count();
      continue;
    }

    // ---- Recorded path: the body of learn() (policy_gradient.h:159-185 /
    // 95-123), via the learners' public methods, with every intermediate.
    auto exp = rb.sample_td();
    for (std::size_t k = log0; k < log.size(); ++k) book.on_apply(log[k]);
    if (book.list.size() != exp.size()) {
      std::fprintf(stderr, "traj_book: %zu trajectories, replay buffer %zu\n",
                   book.list.size(), exp.size());
      return 3;
    }
    std::size_t ti = 0;
    std::size_t ntr = 0;
    for (auto &t : exp) ntr += t.size();
    const std::size_t rows = pg ? ntr : ntr + exp.size();
    xylo::matrix sm({rows, S::length()});
    std::vector<A> actions;
    std::vector<int32_t> tag_env, tag_step, is_end, frozen, choice;
    std::vector<float> reward;
    std::size_t r = 0;
    for (auto &traj : exp) {
      const traj_book::entry &be = book.list[ti++];
      if ((std::size_t)be.n != traj.size()) {
        std::fprintf(stderr, "traj_book: trajectory of %d transitions, "
                     "replay buffer %zu\n", be.n, traj.size());
        return 3;
      }
      int k = 0;
      for (auto &tr : traj) {
        tr.start_state->to_vector(sm[r++]);
        actions.push_back(tr.action);
        if constexpr (W::real_env) {
          tag_env.push_back(be.env);
          tag_step.push_back(be.start + k);
        } else {
          tag_env.push_back(tr.start_state->tag_env);
          tag_step.push_back(tr.start_state->tag_step);
          if (be.env != tr.start_state->tag_env ||
              be.start + k != tr.start_state->tag_step) {
            std::fprintf(stderr, "traj_book disagrees with the tags\n");
            return 3;
          }
        }
        ++k;
        is_end.push_back(0);
        frozen.push_back(traj.frozen());
        choice.push_back(tr.action.choice);
        reward.push_back(tr.reward);
      }
      if (!pg) {
        actions.push_back(actions.back());
        traj.back().end_state.to_vector(sm[r++]);
        if constexpr (W::real_env) {
          tag_env.push_back(be.env);
          tag_step.push_back(be.start + be.n);
        } else {
          tag_env.push_back(traj.back().end_state.tag_env);
          tag_step.push_back(traj.back().end_state.tag_step);
        }
        is_end.push_back(1);
        frozen.push_back(traj.frozen());
        choice.push_back(actions.back().choice);
        reward.push_back(0.0f);
      }
    }
    rec->f32(p + "rows", to_std(sm), {rows, S::length()});
    rec->i32(p + "row_env", tag_env);
    rec->i32(p + "row_step", tag_step);
    rec->i32(p + "row_is_end", is_end);
    rec->i32(p + "row_frozen", frozen);
    rec->i32(p + "row_choice", choice);
    rec->f32(p + "row_reward", reward);

    // Per-step log in env-major order (this iteration only).
    {
      std::vector<int32_t> lb, li, lc, ld, le, ls;
      std::vector<float> lp;
      for (std::size_t k = log0; k < log.size(); ++k) {
        auto &l = log[k];
        lb.insert(lb.end(), l.bins.begin(), l.bins.end());
        li.insert(li.end(), l.item.begin(), l.item.end());
        lc.push_back(l.choice);
        ld.push_back(l.done);
        le.push_back(l.env);
        ls.push_back(l.step);
        lp.insert(lp.end(), l.distrib.begin(), l.distrib.end());
      }
      uint64_t ns = lc.size();
      rec->i32(p + "step_bins", lb, {ns, B, D});
      rec->i32(p + "step_item", li, {ns, D});
      rec->i32(p + "step_choice", lc);
      rec->i32(p + "step_done", ld);
      rec->i32(p + "step_env", le);
      rec->i32(p + "step_index", ls);
      rec->f32(p + "step_distrib", lp, {ns, B});
    }

    log_pi->grads.clear();
    log_v->grads.clear();
    if (pg) {
      xylo::vector adv = pgl->get_advantages(exp);
      rec->f32(p + "advantages", to_std(adv));
      pgl->learn();  // same batch (sample_td is non-destructive)
    } else {
      rec->f32(p + "values_before", to_std(val.eval(sm)));
      ac->update_value_model(exp, sm);
      rec->f32(p + "value_grad", log_v->grads.at(0));
      rec->f32(p + "value_params", to_std(val.parameters()));
      xylo::vector adv = ac->calculate_advantage(exp, sm);
      rec->f32(p + "advantages", to_std(adv));
      ac->optimize_action(sm, actions, adv);
    }
    std::vector<float> gall;
    for (auto &gv : log_pi->grads) gall.insert(gall.end(), gv.begin(), gv.end());
    rec->f32(p + "policy_grads", gall,
             {log_pi->grads.size(),
              log_pi->grads.empty() ? 0 : log_pi->grads[0].size()});
    rec->f32(p + "policy_params", to_std(pol.parameters()));
    rb.forget();
    book.forget();
    rec->u32(p + "x_end", {engine_state()});
    {
      std::vector<int32_t> fb, fi;
      for (auto &e : envs) {
        S s = e.view(0);
        W::bins_of(s, fb);
        W::item_of(s, fi);
      }
      rec->i32(p + "final_bins", fb, {(uint64_t)c.N, B, D});
      rec->i32(p + "final_item", fi, {(uint64_t)c.N, D});
    }
  }
  if (steps_per_s) *steps_per_s = secs > 0 ? total_steps / secs : 0;
  if (!rec)
    std::printf("{\"env_steps\": %ld, \"seconds\": %.6f, \"env_steps_per_s\": "
                "%.3f}\n",
                total_steps, secs, secs > 0 ? total_steps / secs : 0.0);
  return 0;
}

int mode_learn(std::map<std::string, std::string> &a, bool bench) {
  learn_cfg c;
  c.algo = a.count("algo") ? a["algo"] : "ppo";
  c.N = iarg(a, "N", 8);
  c.T = iarg(a, "T", 4);
  c.iters = iarg(a, "iters", 2);
  c.widths = listarg(a, "widths", {128, 64});
  c.vwidths = listarg(a, "vwidths", {64, 32});
  c.lr_pi = darg(a, "lr_pi", c.algo == "ac" ? 1e-5 : 1e-4);
  c.lr_v = darg(a, "lr_v", c.algo == "ac" ? 1e-4 : 1e-5);
  c.wd_pi = darg(a, "wd_pi", 0.0);
  c.wd_v = darg(a, "wd_v", 0.0);
  c.gamma = darg(a, "gamma", 0.99);
  c.seed = iarg(a, "seed", 42);
  c.episodes = iarg(a, "episodes", 1);
  if (a.count("opt_pi")) c.opt_pi = a["opt_pi"];
  if (a.count("opt_v")) c.opt_v = a["opt_v"];
  int B = iarg(a, "B", 8), D = iarg(a, "D", 2);
  std::unique_ptr<recorder> rec;
  if (!bench) rec = std::make_unique<recorder>(a["out"]);
  c.record = !bench;
  recorder *r = rec.get();
  if (B == (int)bp::num_bins && D == 2)
    return run_learn<bp_world, bp::num_bins, 2>(c, r, nullptr);
#define XH_CASE(b, d)                                                          \
  if (B == b && D == d) return run_learn<gen_world<b, d>, b, d>(c, r, nullptr);
  XH_CASE(8, 1)
  XH_CASE(16, 2)
  XH_CASE(32, 1)
#if !XH_REF_BP64
  XH_CASE(64, 2)
#endif
  XH_CASE(128, 3)
#undef XH_CASE
  std::fprintf(stderr, "unsupported B=%d D=%d\n", B, D);
  return 2;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr,
                 "usage: ref_harness rng|envcheck|deep|learn|bench key=value...\n");
    return 2;
  }
  auto a = parse_args(argc, argv);
  std::string mode = argv[1];
#if !XH_REF_BP64
  if (mode == "rng") return mode_rng(a);
  if (mode == "envcheck") return mode_envcheck(a);
  if (mode == "deep") return mode_deep(a);
  if (mode == "driver") return mode_driver(a);
  if (mode == "random") return mode_random(a);
  if (mode == "heuristic") return mode_heuristic(a);
#endif
  if (mode == "learn") return mode_learn(a, false);
  if (mode == "bench") return mode_learn(a, true);
  std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
  return 2;
}
