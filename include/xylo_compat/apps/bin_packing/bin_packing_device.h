// apps/bin_packing/bin_packing_device.h (xylo-hip drop-in layer): the device
// session behind bp:: (see bin_packing.h for the behaviour).  Everything
// here calls the C ABI of include/xylo_hip.h; a non-zero status becomes a
// xeno::error.
#ifndef XYLO_HIP_COMPAT_BIN_PACKING_DEVICE_H_
#define XYLO_HIP_COMPAT_BIN_PACKING_DEVICE_H_

#include <cinttypes>
#include <set>

namespace bp {
namespace device {

inline void check(int status, const char *what) {
  if (status != XH_OK)
    throw xeno::error(std::string("xylo-hip: ") + what + ": " + xh_last_error());
}

// ---- minstd_rand0 state access (the engine of tensor.cc:71-75) ----------
inline std::uint32_t engine_state(const std::default_random_engine &e) {
  std::ostringstream os;  // libstdc++ streams the engine's state word
  os << e;
  return std::uint32_t(std::stoul(os.str()));
}
inline std::uint32_t minstd_jump(std::uint32_t x, std::uint64_t n) {
  const std::uint64_t m = 2147483647ull;
  std::uint64_t r = 1, b = 16807;
  for (; n; n >>= 1, b = b * b % m)
    if (n & 1) r = r * b % m;
  return std::uint32_t(r * x % m);
}

// ---- the process-wide device context (xylo/nn.h) ------------------------
inline xh_ctx *context() { return xylo::detail::hip_context(); }

struct trainer {
  xh_trainer *h = nullptr;
  xh_config cfg{};
  int policy_n = 0, value_n = 0;
  explicit trainer(const xh_config &c) : cfg(c) {
    check(xh_trainer_create(context(), &cfg, &h), "xh_trainer_create");
    policy_n = int(xh_trainer_num_params(h, XH_POLICY));
    value_n = int(xh_trainer_num_params(h, XH_VALUE));
  }
  ~trainer() { xh_trainer_destroy(h); }
  trainer(const trainer &) = delete;
  void operator=(const trainer &) = delete;
};

// ---- model descriptions -> device shapes --------------------------------
struct policy_shape {
  int h1 = 0, h2 = 0;
  int head = -1;  // -1: logits (deep_agent.cc), else layer_kind of the head
};
inline policy_shape parse_policy(const xylo::model &m) {
  using K = xylo::layer_kind;
  auto ls = m.layers();
  auto is = [&](std::size_t i, K k) { return i < ls.size() && ls[i]->kind() == k; };
  policy_shape s;
  const bool ok = ls.size() >= 5 && is(0, K::conv1d_1) && is(1, K::relu) &&
                  is(2, K::conv1d_1) && is(3, K::relu) && is(4, K::conv1d_1) &&
                  ls[0]->input_size() == 4 && ls[4]->output_size() == 1 &&
                  ls[1 + 1]->input_size() == ls[0]->output_size() &&
                  ls[4]->input_size() == ls[2]->output_size() &&
                  (ls.size() == 5 || (ls.size() == 6 && (is(5, K::softmax) ||
                                                         is(5, K::softmax_xent))));
  if (!ok)
    throw xeno::error("xylo-hip: the device policy is the per-bin network "
                      "conv1d_1(4,h1)-relu-conv1d_1(h1,h2)-relu-conv1d_1(h2,1)"
                      "[-softmax]");
  s.h1 = int(ls[0]->output_size());
  s.h2 = int(ls[2]->output_size());
  if (ls.size() == 6) s.head = int(ls[5]->kind());
  return s;
}
// REINFORCE's policy (pg_training.cc:10-20): full(4B,h1)-relu
// [-full(h1,h2)-relu]-full(.,B)-softmax_cross_entropy.
inline policy_shape parse_full_policy(const xylo::model &m) {
  using K = xylo::layer_kind;
  auto ls = m.layers();
  auto is = [&](std::size_t i, K k) { return i < ls.size() && ls[i]->kind() == k; };
  policy_shape s;
  const std::size_t n = ls.size();
  bool ok = (n == 4 || n == 6) && is(0, K::full) && is(1, K::relu) &&
            is(n - 2, K::full) && is(n - 1, K::softmax_xent) &&
            ls[0]->input_size() == observation::length() &&
            ls[n - 2]->output_size() == num_bins;
  if (ok && n == 6)
    ok = is(2, K::full) && is(3, K::relu) &&
         ls[2]->input_size() == ls[0]->output_size() &&
         ls[4]->input_size() == ls[2]->output_size();
  if (ok && n == 4) ok = ls[2]->input_size() == ls[0]->output_size();
  if (!ok)
    throw xeno::error("xylo-hip: the device REINFORCE policy is full(4*num_bins,"
                      "h1)-relu[-full(h1,h2)-relu]-full(.,num_bins)-"
                      "softmax_cross_entropy_layer");
  s.h1 = int(ls[0]->output_size());
  s.h2 = n == 6 ? int(ls[2]->output_size()) : 0;
  s.head = int(K::softmax_xent);
  return s;
}

// non-throwing forms: can the device take this model?
template <class F>
bool parses(F &&f) {
  try {
    f();
    return true;
  } catch (const xeno::error &) {
    return false;
  }
}
inline std::pair<int, int> parse_value(const xylo::model &m);
inline bool device_policy(const xylo::model &m) {
  return parses([&] { parse_policy(m); });
}
inline bool device_full_policy(const xylo::model &m) {
  return parses([&] { parse_full_policy(m); });
}
inline bool device_value(const xylo::model &m) {
  return parses([&] { parse_value(m); });
}
// The fused device learner takes this description: library optimizers, the
// per-bin policy with the learner's head (REINFORCE: the full policy) and the
// device value net.
inline bool fusable(const xylo::learner_desc &d) {
  auto lib_opt = [](const xylo::optimizer *o) {
    return !o || o->kind() != xylo::optimizer_kind::custom;
  };
  if (!d.action_model || !lib_opt(d.action_optimizer) ||
      !lib_opt(d.value_optimizer))
    return false;
  if (d.kind == xylo::learner_kind::reinforce)
    return device_full_policy(*d.action_model);
  if (!d.value_model || !device_policy(*d.action_model) ||
      !device_value(*d.value_model))
    return false;
  const int want = int(d.kind == xylo::learner_kind::actor_critic
                           ? xylo::layer_kind::softmax_xent
                           : xylo::layer_kind::softmax);
  return parse_policy(*d.action_model).head == want;
}

inline std::pair<int, int> parse_value(const xylo::model &m) {
  using K = xylo::layer_kind;
  auto ls = m.layers();
  const bool ok = ls.size() == 5 && ls[0]->kind() == K::full &&
                  ls[1]->kind() == K::relu && ls[2]->kind() == K::full &&
                  ls[3]->kind() == K::relu && ls[4]->kind() == K::full &&
                  ls[0]->input_size() == observation::length() &&
                  ls[4]->output_size() == 1;
  if (!ok)
    throw xeno::error("xylo-hip: the device value net is full(4*num_bins,v1)-"
                      "relu-full(v1,v2)-relu-full(v2,1)");
  return {int(ls[0]->output_size()), int(ls[2]->output_size())};
}

class session;
inline std::set<session *> &live_sessions() {
  static std::set<session *> s;
  return s;
}
inline void flush_all();

// Per-model cache of an eval-only trainer (models never trained here, e.g.
// deep_agent.cc's weights.20).
struct eval_binding {
  std::unique_ptr<trainer> tr;
  std::uint64_t version = ~0ull;
};

using rb_t = xylo::replay_buffer<action, observation>;
using agent_t = xylo::agent<action, observation>;

class session {
 public:
  session() { live_sessions().insert(this); }
  ~session() {
    live_sessions().erase(this);
    try {
      if (learner_.action_model) learner_.action_model->unbind_device(this);
      if (learner_.value_model) learner_.value_model->unbind_device(this);
    } catch (...) {
    }
    for (environment *e : envs_)
      if (e) e->bind(nullptr, -1);
  }

  void attach(const xylo::learner_desc &d) {
    learner_ = d;
    has_learner_ = true;
  }

  // agent.play_steps(n) with a stochastic device policy.
  void request_steps(environment &env, xylo::model &m, int n) {
    if (learned_unforgotten_)
      throw xeno::error("xylo-hip: call replay_buffer.forget() after "
                        "learner.step() before playing again (device windows "
                        "do not accumulate)");
    if (state_ == rolled)
      throw xeno::error("xylo-hip: play_steps() again before learner.step()");
    if (!has_learner_ || learner_.action_model != &m)
      throw xeno::error("xylo-hip: construct the learner of this replay "
                        "buffer (with the policy's model) before playing");
    if (env.bound_session() && env.bound_session() != this)
      throw xeno::error("xylo-hip: env is bound to another replay buffer");
    flush_evals();
    if (state_ == idle) {
      window_.clear();
      T_ = n;
      state_ = pending;
    }
    if (n != T_)
      throw xeno::error("xylo-hip: every agent plays the same number of steps "
                        "per window");
    if (tr_) {  // same agents, same order as the first window
      if (window_.size() >= envs_.size() || envs_[window_.size()] != &env)
        throw xeno::error("xylo-hip: the set / order of agents changed "
                          "between windows");
    } else if (!first_window_.insert(&env).second) {
      throw xeno::error("xylo-hip: an env played twice in one window");
    }
    window_.push_back(&env);
  }

  void request_episodes(agent_t &a, environment &env, xylo::model &m, int k) {
    if (env.bound_session())
      throw xeno::error("xylo-hip: evaluation env is bound to a training "
                        "window");
    if (!evals_.empty() && evals_.back().agent == &a)
      evals_.back().episodes += k;
    else
      evals_.push_back({&a, &env, &m, k});
  }

  // agent.play_one_episode() with a stochastic device policy and a REINFORCE
  // learner: the window is every agent's whole episodes, played on the
  // device at the next flush (pg_training.cc:52-62).
  void request_train_episodes(environment &env, xylo::model &m, int k) {
    if (learned_unforgotten_)
      throw xeno::error("xylo-hip: call replay_buffer.forget() after "
                        "learner.step() before playing again (device windows "
                        "do not accumulate)");
    if (state_ == rolled)
      throw xeno::error("xylo-hip: play_one_episode() again before "
                        "learner.step()");
    if (!has_learner_ || learner_.action_model != &m ||
        learner_.kind != xylo::learner_kind::reinforce)
      throw xeno::error("xylo-hip: training episodes need the replay buffer's "
                        "policy_gradient_learner (REINFORCE) constructed with "
                        "the policy's model before playing");
    if (env.bound_session() && env.bound_session() != this)
      throw xeno::error("xylo-hip: env is bound to another replay buffer");
    flush_evals();
    if (state_ == idle) {
      window_.clear();
      episodes_.clear();
      state_ = pending;
    }
    if (!window_.empty() && window_.back() == &env) {
      episodes_.back() += k;
      return;
    }
    if (tr_) {
      if (window_.size() >= envs_.size() || envs_[window_.size()] != &env)
        throw xeno::error("xylo-hip: the set / order of agents changed "
                          "between windows");
    } else if (!first_window_.insert(&env).second) {
      throw xeno::error("xylo-hip: an env played in two separate runs of one "
                        "window");
    }
    window_.push_back(&env);
    episodes_.push_back(k);
  }

  // Runs deferred device work in request order.
  void flush() {
    roll();
    flush_evals();
  }

  void learn(rb_t &, const xylo::learner_desc &d) {
    attach(d);
    flush_all();
    if (state_ != rolled)
      throw xeno::error("xylo-hip: learner.step() without new experience");
    push_params();
    sync_rates();
    check(xh_trainer_learn(tr_->h), "xh_trainer_learn");
    state_ = idle;
    learned_unforgotten_ = true;
    learner_.action_model->mark_device_newer(this);
    if (learner_.value_model) learner_.value_model->mark_device_newer(this);
    ++steps_;
    if (const char *p = std::getenv("XYLO_HIP_DUMP")) {
      const std::string k = "." + std::to_string(steps_) + ".bin";
      write_params(std::string(p) + ".policy" + k, XH_POLICY);
      if (!pg()) write_params(std::string(p) + ".value" + k, XH_VALUE);
    }
    maybe_exit();
  }

  void forget() {
    flush_all();
    if (tr_ && state_ == rolled) {
      // the window was never learned on the device (a learner of the
      // caller's own read it through sample_td, or nobody did): forget() is
      // the trainer's shift of the final states to the next start states
      check(xh_trainer_forget(tr_->h), "xh_trainer_forget");
      state_ = idle;
      ++steps_;
    }
    learned_unforgotten_ = false;
  }

  // learner.step() of a composed learner (policy_gradient.h) consumed the
  // window on the host: the trainer forgets it as its own learn() would
  void learned_on_host() {
    flush_all();
    if (!tr_) return;  // host-stepped experience: nothing on the device
    if (state_ != rolled)
      throw xeno::error("xylo-hip: learner.step() without new experience");
    check(xh_trainer_forget(tr_->h), "xh_trainer_forget");
    state_ = idle;
    learned_unforgotten_ = true;
    ++steps_;
  }

  bool composed() const { return learner_.fused && !learner_.fused(); }

  // replay_buffer.sample_td(): the window's trajectories from the device.
  void materialise(rb_t &rb) {
    flush_all();
    if (!tr_ || materialised_ || (state_ != rolled && !learned_unforgotten_))
      return;
    if (pg()) {
      materialise_episodes(rb);
      return;
    }
    const int N = int(envs_.size()), T = T_, B = int(num_bins);
    std::vector<std::int8_t> bins(std::size_t(T + 1) * N * B * 2),
        items(std::size_t(T + 1) * N * 4);
    std::vector<std::int32_t> act(std::size_t(T) * N);
    std::vector<std::uint8_t> done(std::size_t(T) * N);
    get(XH_BUF_BINS, bins);
    get(XH_BUF_ITEMS, items);
    get(XH_BUF_ACTION, act);
    get(XH_BUF_DONE, done);
    // the sampling distributions (discrete_action::distrib) when the
    // trainer recorded them for a composed learner's loss
    std::vector<float> qold;
    if (tr_->cfg.record_distrib) {
      qold.resize(std::size_t(T) * N * B);
      get(XH_BUF_QOLD, qold);
    }
    auto state = [&](int t, int e) {
      observation o;
      const std::int8_t *b = &bins[(std::size_t(t) * N + e) * B * 2];
      for (int i = 0; i < B; ++i) o.bins[i] = {b[2 * i], b[2 * i + 1]};
      const std::int8_t *it = &items[(std::size_t(t) * N + e) * 4];
      o.item = {it[0], it[1]};
      return o;
    };
    auto &list = rb.trajectories();
    list.clear();
    for (int e = 0; e < N; ++e) {
      xylo::trajectory<action, observation> *traj = nullptr;
      for (int t = 0; t < T; ++t) {
        if (!traj) traj = &rb.emplace_trajectory(state(t, e));
        action a;
        a.choice = std::size_t(act[std::size_t(t) * N + e]);
        if (!qold.empty())
          a.distrib = xylo::vector(xylo::vector_view(
              qold.data() + (std::size_t(t) * N + e) * B, std::size_t(B)));
        const bool over = done[std::size_t(t) * N + e] != 0;
        observation end = state(over ? t : t + 1, e);
        if (over) {  // the overflowed view before reset (rl.h:336-343)
          end.bins[a.choice].first -= end.item.first;
          end.bins[a.choice].second -= end.item.second;
        }
        traj->add_transition(std::move(a), over ? 0.0f : 1.0f, std::move(end));
        if (over) {
          traj->freeze();
          traj = nullptr;
        }
      }
    }
    materialised_ = true;
  }

  // REINFORCE window: each env's whole episodes (all frozen), env by env.
  void materialise_episodes(rb_t &rb) {
    const int N = int(envs_.size()), T = T_, B = int(num_bins);
    std::vector<std::int8_t> bins(std::size_t(T + 1) * N * B * 2),
        items(std::size_t(T + 1) * N * 4);
    std::vector<std::int32_t> act(std::size_t(T) * N), len(N);
    std::vector<std::uint8_t> done(std::size_t(T) * N);
    get(XH_BUF_BINS, bins);
    get(XH_BUF_ITEMS, items);
    get(XH_BUF_ACTION, act);
    get(XH_BUF_DONE, done);
    get(XH_BUF_LEN, len);
    auto &list = rb.trajectories();
    list.clear();
    for (int e = 0; e < N; ++e) {
      xylo::trajectory<action, observation> *traj = nullptr;
      for (int t = 0; t < len[e]; ++t) {
        if (!traj) traj = &rb.emplace_trajectory(state_at(bins, items, t, e));
        action a;
        a.choice = std::size_t(act[std::size_t(t) * N + e]);
        const bool over = done[std::size_t(t) * N + e] != 0;
        observation end = state_at(bins, items, over ? t : t + 1, e);
        if (over) {
          end.bins[a.choice].first -= end.item.first;
          end.bins[a.choice].second -= end.item.second;
        }
        traj->add_transition(std::move(a), over ? 0.0f : 1.0f, std::move(end));
        if (over) {
          traj->freeze();
          traj = nullptr;
        }
      }
    }
    materialised_ = true;
  }

  observation state_at(const std::vector<std::int8_t> &bins,
                       const std::vector<std::int8_t> &items, int t, int e) {
    const int N = int(envs_.size()), B = int(num_bins);
    observation o;
    const std::int8_t *b = &bins[(std::size_t(t) * N + e) * B * 2];
    for (int i = 0; i < B; ++i) o.bins[i] = {b[2 * i], b[2 * i + 1]};
    const std::int8_t *it = &items[(std::size_t(t) * N + e) * 4];
    o.item = {it[0], it[1]};
    return o;
  }

  // env.apply / env.reset of a device-bound env by host code: the new state
  // is what that env's next rollout starts from (xh_trainer_set_env_state);
  // the current window's trajectories are untouched.
  void set_env_state(int index, const observation &o) {
    flush_all();
    if (pg())
      throw xeno::error("xylo-hip: host apply / reset of an env bound to a "
                        "REINFORCE window is not supported");
    const int B = int(num_bins);
    std::vector<std::int8_t> b(std::size_t(B) * 2), it(2);
    for (int i = 0; i < B; ++i) {
      b[2 * i] = std::int8_t(o.bins[i].first);
      b[2 * i + 1] = std::int8_t(o.bins[i].second);
    }
    it[0] = std::int8_t(o.item.first);
    it[1] = std::int8_t(o.item.second);
    check(xh_trainer_set_env_state(tr_->h, index, 1, b.data(), it.data()),
          "xh_trainer_set_env_state");
    overrides_[index] = o;
  }

  // env.view() of a device-bound env: its current state on the device.
  observation device_view(int index) {
    flush_all();
    auto ov = overrides_.find(index);
    if (ov != overrides_.end()) return ov->second;
    const int N = int(envs_.size()), B = int(num_bins);
    std::vector<std::int8_t> bins(std::size_t(T_ + 1) * N * B * 2),
        items(std::size_t(T_ + 1) * N * 4);
    get(XH_BUF_BINS, bins);
    get(XH_BUF_ITEMS, items);
    int slot = slot_;
    if (pg()) {  // after its last episode an env holds its post-reset state
      std::vector<std::int32_t> len(N);
      get(XH_BUF_LEN, len);
      slot = len[index];
    }
    observation o;
    const std::size_t row = std::size_t(slot) * N + index;
    for (int i = 0; i < B; ++i)
      o.bins[i] = {bins[row * B * 2 + 2 * i], bins[row * B * 2 + 2 * i + 1]};
    o.item = {items[row * 4], items[row * 4 + 1]};
    return o;
  }

  void env_gone(int index) {
    if (index >= 0 && index < int(envs_.size())) envs_[index] = nullptr;
  }

  trainer *training_trainer() { return tr_.get(); }
  void push_params() {
    if (!tr_) return;
    push(*learner_.action_model, XH_POLICY, pol_version_);
    // a composed learner's value net never runs on this trainer
    if (learner_.value_model && !tr_->cfg.record_distrib)
      push(*learner_.value_model, XH_VALUE, val_version_);
  }
  bool pg() const { return tr_ && tr_->cfg.algo == XH_PG; }

 private:
  enum { idle, pending, rolled } state_ = idle;

  struct eval_req {
    agent_t *agent;
    environment *env;
    xylo::model *model;
    int episodes;
  };

  template <typename V> void get(int which, V &v) {
    check(xh_trainer_get_buffer(tr_->h, which, v.data(),
                                v.size() * sizeof(v[0])),
          "xh_trainer_get_buffer");
  }

  void push(xylo::model &m, int which, std::uint64_t &version) {
    if (m.device_owner() == this && m.host_version() == version) return;
    xylo::vector p = m.parameters();  // pulls from another owner if needed
    check(xh_trainer_set_params(tr_->h, which, p.data(), p.size()),
          "xh_trainer_set_params");
    version = m.host_version();
    trainer *t = tr_.get();
    m.bind_device(this, [t, which](std::span<float> out) {
      check(xh_trainer_get_params(t->h, which, out.data(), out.size()),
            "xh_trainer_get_params");
    });
  }

  void ensure_trainer_pg() {
    const int N = int(window_.size());
    for (int k : episodes_)
      if (k != episodes_[0])
        throw xeno::error("xylo-hip: every agent plays the same number of "
                          "episodes per window");
    if (tr_) {
      if (window_.size() != envs_.size())
        throw xeno::error("xylo-hip: fewer agents played than in the first "
                          "window");
      if (episodes_[0] != tr_->cfg.steps)
        throw xeno::error("xylo-hip: episodes per window changed");
      return;
    }
    const policy_shape ps = parse_full_policy(*learner_.action_model);
    xh_config c;
    xh_config_default(&c, XH_PG, int(num_bins), 2, N, episodes_[0]);
    c.policy_h1 = ps.h1;
    c.policy_h2 = ps.h2;
    c.lr_policy = learner_.action_optimizer->rate();
    c.wd_policy = learner_.action_optimizer->weight_decay();
    c.gamma = learner_.gamma;
    tr_ = std::make_unique<trainer>(c);
    set_optimizers();
    T_ = int(xh_trainer_buffer_bytes(tr_->h, XH_BUF_ACTION) / (4 * std::size_t(N)));
    upload_host_states();
    if (const char *p = std::getenv("XYLO_HIP_DUMP"))
      write_params(std::string(p) + ".policy.0.bin", XH_POLICY);
  }

  // optimizer::set_rate between steps (nn.h:591) reaches the device
  void sync_rates() {
    for (int which : {XH_POLICY, XH_VALUE}) {
      xylo::optimizer *o = which == XH_POLICY ? learner_.action_optimizer
                                              : learner_.value_optimizer;
      if (!o) continue;
      const float want = o->rate();
      const float have = which == XH_POLICY ? tr_->cfg.lr_policy : tr_->cfg.lr_value;
      if (want != have) {
        check(xh_trainer_set_learning_rate(tr_->h, which, want),
              "xh_trainer_set_learning_rate");
        (which == XH_POLICY ? tr_->cfg.lr_policy : tr_->cfg.lr_value) = want;
      }
    }
  }

  void set_optimizers() {
    for (int which : {XH_POLICY, XH_VALUE}) {
      xylo::optimizer *o = which == XH_POLICY ? learner_.action_optimizer
                                              : learner_.value_optimizer;
      if (!o || o->kind() == xylo::optimizer_kind::sgd) continue;
      const int kind = o->kind() == xylo::optimizer_kind::adam ? XH_OPT_ADAM
                                                               : XH_OPT_MOMENTUM;
      check(xh_trainer_set_optimizer(tr_->h, which, kind, o->rate(), 0.0f,
                                     o->beta1(), o->beta2()),
            "xh_trainer_set_optimizer");
    }
  }

  // slot 0 <- the host envs' states (drawn by their constructors); binds them
  void upload_host_states() {
    const int N = int(window_.size()), B = int(num_bins);
    std::vector<std::int8_t> bins(std::size_t(T_ + 1) * N * B * 2, 0),
        items(std::size_t(T_ + 1) * N * 4, 0);
    for (int e = 0; e < N; ++e) {
      const observation &o = window_[e]->host_state();
      for (int i = 0; i < B; ++i) {
        bins[(std::size_t(e) * B + i) * 2] = std::int8_t(o.bins[i].first);
        bins[(std::size_t(e) * B + i) * 2 + 1] = std::int8_t(o.bins[i].second);
      }
      items[std::size_t(e) * 4] = std::int8_t(o.item.first);
      items[std::size_t(e) * 4 + 1] = std::int8_t(o.item.second);
      window_[e]->bind(this, e);
    }
    check(xh_trainer_set_buffer(tr_->h, XH_BUF_BINS, bins.data(), bins.size()),
          "xh_trainer_set_buffer");
    check(xh_trainer_set_buffer(tr_->h, XH_BUF_ITEMS, items.data(),
                                items.size()),
          "xh_trainer_set_buffer");
    envs_ = window_;
    first_window_.clear();
    pol_version_ = val_version_ = ~0ull;
    push_params();
  }

  void ensure_trainer() {
    const int N = int(window_.size());
    if (tr_) {
      if (window_.size() != envs_.size())
        throw xeno::error("xylo-hip: fewer agents played than in the first "
                          "window");
      if (T_ != tr_->cfg.steps)
        throw xeno::error("xylo-hip: steps per window changed");
      return;
    }
    const policy_shape ps = parse_policy(*learner_.action_model);
    // a composed learner (policy_gradient.h) learns on the host: the trainer
    // only rolls out, recording the sampling distributions its loss reads
    const bool composed = this->composed();
    const auto vs = composed ? std::pair<int, int>{64, 32}
                             : parse_value(*learner_.value_model);
    const bool ac = learner_.kind == xylo::learner_kind::actor_critic;
    const bool klppo = learner_.kind == xylo::learner_kind::kl_ppo;
    const int want_head = int(ac ? xylo::layer_kind::softmax_xent
                                 : xylo::layer_kind::softmax);
    if (!composed && ps.head != want_head)
      throw xeno::error(ac ? "xylo-hip: ac_learner needs a "
                             "softmax_cross_entropy_layer head"
                           : "xylo-hip: ppo_learner / kl_ppo_learner need a "
                             "softmax_layer head");
    xh_config c;
    xh_config_default(&c, composed ? XH_PPO : ac ? XH_AC : klppo ? XH_KLPPO : XH_PPO,
                      int(num_bins), 2, N, T_);
    c.record_distrib = composed ? 1 : 0;
    c.policy_h1 = ps.h1;
    c.policy_h2 = ps.h2;
    c.value_h1 = vs.first;
    c.value_h2 = vs.second;
    c.lr_policy = learner_.action_optimizer->rate();
    c.lr_value = learner_.value_optimizer->rate();
    c.wd_policy = learner_.action_optimizer->weight_decay();
    c.wd_value = learner_.value_optimizer->weight_decay();
    c.gamma = learner_.gamma;
    c.lambda = learner_.lambda;
    tr_ = std::make_unique<trainer>(c);
    // momentum / adam optimizers (nn.h:630-698) run on the device too; their
    // state starts at zero with the first learn(), as the reference's does
    set_optimizers();
    // initial env states: slot 0 from the host envs (drawn by their ctors)
    const int B = int(num_bins);
    std::vector<std::int8_t> bins(std::size_t(T_ + 1) * N * B * 2, 0),
        items(std::size_t(T_ + 1) * N * 4, 0);
    for (int e = 0; e < N; ++e) {
      const observation &o = window_[e]->host_state();
      for (int i = 0; i < B; ++i) {
        bins[(std::size_t(e) * B + i) * 2] = std::int8_t(o.bins[i].first);
        bins[(std::size_t(e) * B + i) * 2 + 1] = std::int8_t(o.bins[i].second);
      }
      items[std::size_t(e) * 4] = std::int8_t(o.item.first);
      items[std::size_t(e) * 4 + 1] = std::int8_t(o.item.second);
      window_[e]->bind(this, e);
    }
    check(xh_trainer_set_buffer(tr_->h, XH_BUF_BINS, bins.data(), bins.size()),
          "xh_trainer_set_buffer");
    check(xh_trainer_set_buffer(tr_->h, XH_BUF_ITEMS, items.data(),
                                items.size()),
          "xh_trainer_set_buffer");
    envs_ = window_;
    first_window_.clear();
    pol_version_ = val_version_ = ~0ull;
    push_params();
    if (const char *p = std::getenv("XYLO_HIP_DUMP")) {
      write_params(std::string(p) + ".policy.0.bin", XH_POLICY);
      write_params(std::string(p) + ".value.0.bin", XH_VALUE);
    }
  }

  void roll() {
    if (state_ != pending) return;
    if (!episodes_.empty()) {
      roll_episodes();
      return;
    }
    ensure_trainer();
    push_params();
    auto &eng = xylo::detail::raw_generator();
    const std::uint32_t x = engine_state(eng);
    if (steps_ == 0) x_first_ = x;
    check(xh_trainer_seed_streams(tr_->h, x), "xh_trainer_seed_streams");
    eng.seed(minstd_jump(x, 4ull * T_ * envs_.size()));
    check(xh_trainer_rollout(tr_->h), "xh_trainer_rollout");
    overrides_.clear();  // the rollout started from them
    state_ = rolled;
    materialised_ = false;
    slot_ = T_;
  }

  // REINFORCE window: env g plays on the engine state advanced by g * 2^26
  // draws (env 0 continues the host engine exactly, as one reference worker
  // does); the host engine then takes the last env's final stream state.
  void roll_episodes() {
    ensure_trainer_pg();
    push_params();
    auto &eng = xylo::detail::raw_generator();
    const std::uint32_t x = engine_state(eng);
    if (steps_ == 0) x_first_ = x;
    check(xh_trainer_seed_streams(tr_->h, x), "xh_trainer_seed_streams");
    check(xh_trainer_rollout(tr_->h), "xh_trainer_rollout");
    std::vector<std::uint32_t> rng(envs_.size());
    get(XH_BUF_RNG, rng);
    eng.seed(rng.back());
    state_ = rolled;
    materialised_ = false;
    episodes_.clear();
  }

  void flush_evals() {
    std::vector<eval_req> todo;
    todo.swap(evals_);
    for (eval_req &r : todo) run_eval(r);
  }

  // agent.play_one_episode() x k with an argmax policy, on the device.
  static void run_eval(eval_req &r) {
    const policy_shape ps = parse_policy(*r.model);
    const int B = int(num_bins), G = B <= 64 ? 64 / B : 0;
    if (G == 0)
      throw xeno::error("xylo-hip: device evaluation needs num_bins <= 64");
    trainer *t = nullptr;
    for (session *s : live_sessions())
      if (r.model->device_owner() == s && s->training_trainer()) {
        s->push_params();
        t = s->training_trainer();
      }
    if (!t) {
      auto slot = std::static_pointer_cast<eval_binding>(r.model->device_slot);
      if (!slot) {
        slot = std::make_shared<eval_binding>();
        r.model->device_slot = slot;
      }
      if (!slot->tr || slot->tr->cfg.policy_h1 != ps.h1 ||
          slot->tr->cfg.policy_h2 != ps.h2) {
        xh_config c;
        xh_config_default(&c, XH_PPO, B, 2, G, 1);
        c.policy_h1 = ps.h1;
        c.policy_h2 = ps.h2;
        slot->tr = std::make_unique<trainer>(c);
        slot->version = ~0ull;
      }
      if (slot->version != r.model->host_version() ||
          r.model->device_owner() != nullptr) {
        xylo::vector p = r.model->parameters();
        check(xh_trainer_set_params(slot->tr->h, XH_POLICY, p.data(), p.size()),
              "xh_trainer_set_params");
        slot->version = r.model->host_version();
      }
      t = slot->tr.get();
    }
    const observation &o = r.env->host_state();
    for (const auto &b : o.bins)
      if (b != observation::capacity)
        throw xeno::error("xylo-hip: device episodes start from a fresh or "
                          "reset env");
    std::vector<std::int32_t> init(std::size_t(G) * 2);
    for (int e = 0; e < G; ++e) {
      init[2 * e] = o.item.first;
      init[2 * e + 1] = o.item.second;
    }
    auto &eng = xylo::detail::raw_generator();
    const long cap = long(r.episodes) * (B * 8 * 2 + 2);
    std::vector<std::int32_t> trace(std::size_t(cap > 0 ? cap : 1));
    std::vector<double> totals(G);
    std::vector<long> steps(G);
    std::vector<std::uint32_t> rng(G);
    xh_eval ev{};
    ev.n_envs = G;
    ev.episodes = r.episodes;
    ev.argmax_probs = ps.head >= 0 ? 1 : 0;
    ev.rng_state = engine_state(eng);
    ev.init_items = init.data();
    ev.rng_out = rng.data();
    ev.totals = totals.data();
    ev.steps = steps.data();
    ev.trace = trace.data();
    ev.trace_cap = cap;
    check(xh_trainer_evaluate(t->h, &ev), "xh_trainer_evaluate");
    // replay the device's choices through the host env (engine draws,
    // trajectories and rewards exactly as agent::step makes them)
    double total = 0;
    long n = 0;
    for (int ep = 0; ep < r.episodes; ++ep) {
      for (;;) {
        if (n >= steps[0] || n >= cap)
          throw xeno::error("xylo-hip: device episode trace too short");
        action a;
        a.choice = std::size_t(trace[std::size_t(n++)]);
        const bool open = r.agent->step_with(std::move(a));
        if (!open) break;
        total += 1.0;
      }
    }
    if (n != steps[0] || total != totals[0] || engine_state(eng) != rng[0])
      throw xeno::error("xylo-hip: device evaluation disagrees with the host "
                        "replay");
  }

  void write_params(const std::string &path, int which) {
    std::vector<float> p(which == XH_POLICY ? tr_->policy_n : tr_->value_n);
    check(xh_trainer_get_params(tr_->h, which, p.data(), p.size()),
          "xh_trainer_get_params");
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char *>(p.data()), p.size() * sizeof(float));
  }

  void maybe_exit() {
    const char *m = std::getenv("XYLO_HIP_MAX_STEPS");
    if (!m || steps_ < std::atol(m)) return;
    if (const char *p = std::getenv("XYLO_HIP_DUMP")) {
      std::ofstream j(std::string(p) + ".json");
      j << "{\"x0\": " << x_first_ << ", \"num_envs\": " << envs_.size()
        << ", \"steps\": " << T_ << ", \"learner_steps\": " << steps_
        << ", \"algo\": \""
        << (tr_->cfg.algo == XH_AC      ? "ac"
            : tr_->cfg.algo == XH_KLPPO ? "klppo"
            : tr_->cfg.algo == XH_PG    ? "pg"
                                        : "ppo")
        << "\", \"h1\": " << tr_->cfg.policy_h1 << ", \"h2\": "
        << tr_->cfg.policy_h2 << ", \"v1\": " << tr_->cfg.value_h1
        << ", \"v2\": " << tr_->cfg.value_h2 << ", \"lr_policy\": "
        << tr_->cfg.lr_policy << ", \"lr_value\": " << tr_->cfg.lr_value
        << ", \"bins\": " << num_bins << "}\n";
    }
    std::fflush(nullptr);
    std::exit(0);
  }

  xylo::learner_desc learner_{};
  bool has_learner_ = false;
  std::unique_ptr<trainer> tr_;
  std::vector<environment *> window_, envs_;
  std::set<environment *> first_window_;
  std::vector<eval_req> evals_;
  std::vector<int> episodes_;  // REINFORCE window: episodes per env
  int T_ = 0, slot_ = 0;
  bool materialised_ = false, learned_unforgotten_ = false;
  long steps_ = 0;
  std::uint32_t x_first_ = 0;
  std::uint64_t pol_version_ = ~0ull, val_version_ = ~0ull;
  std::map<int, observation> overrides_;  // host apply / reset since the roll
};

inline void flush_all() {
  static bool busy = false;
  if (busy) return;
  busy = true;
  try {
    for (session *s : std::vector<session *>(live_sessions().begin(),
                                             live_sessions().end()))
      s->flush();
  } catch (...) {
    busy = false;
    throw;
  }
  busy = false;
}

inline session &session_of(rb_t &rb) {
  auto &p = rb.device_state();
  if (!p) {
    p = std::make_shared<session>();
    xylo::detail::engine_flush_hook() = &flush_all;
  }
  return *std::static_pointer_cast<session>(p);
}

}  // namespace device

inline environment::~environment() {
  if (bound_) bound_->env_gone(index_);
}

inline observation environment::view(std::size_t) const {
  if (bound_) return bound_->device_view(index_);
  return state_;
}

inline void environment::bound_write(const observation &s) {
  bound_->set_env_state(index_, s);
}

}  // namespace bp

namespace xylo {

template <> struct device_traits<bp::action, bp::observation> {
  static constexpr bool enabled = true;
  using A = bp::action;
  using S = bp::observation;

  static void attach(replay_buffer<A, S> &rb, const learner_desc &d) {
    bp::device::session_of(rb).attach(d);
  }
  static void learn(replay_buffer<A, S> &rb, const learner_desc &d) {
    bp::device::session_of(rb).learn(rb, d);
  }
  static bool fusable(const learner_desc &d) { return bp::device::fusable(d); }
  static void learned_on_host(replay_buffer<A, S> &rb) {
    if (rb.device_state()) bp::device::session_of(rb).learned_on_host();
  }
  static bool play_steps(agent<A, S> &a, std::size_t n) {
    auto *p = dynamic_cast<const policy_gradient_policy<A, S> *>(&a.bound_policy());
    auto *env = dynamic_cast<bp::environment *>(&a.bound_env());
    // a policy network the device rollout cannot run steps on the host
    // (react() -> model::eval, still on the device)
    if (!p || !env || !bp::device::device_policy(p->device_model())) return false;
    bp::device::session_of(a.bound_buffer()).request_steps(*env, p->device_model(),
                                                           int(n));
    return true;
  }
  static bool play_episodes(agent<A, S> &a, int k) {
    auto *env = dynamic_cast<bp::environment *>(&a.bound_env());
    if (!env) return false;
    if (auto *sp = dynamic_cast<const policy_gradient_policy<A, S> *>(
            &a.bound_policy())) {  // REINFORCE training episodes
      if (!bp::device::device_full_policy(sp->device_model())) return false;
      bp::device::session_of(a.bound_buffer())
          .request_train_episodes(*env, sp->device_model(), k);
      return true;
    }
    auto *p = dynamic_cast<const policy_gradient_deterministic_policy<A, S> *>(
        &a.bound_policy());
    if (!p) return false;
    bp::device::session_of(a.bound_buffer())
        .request_episodes(a, *env, p->device_model(), k);
    return true;
  }
  // A host-policy step of a device-bound env goes through the env's device
  // view / apply / reset; only recording it into the replay buffer whose
  // device window that env belongs to is refused (the window's trajectories
  // are the device's).
  static void before_host_step(agent<A, S> &a) {
    bp::device::flush_all();
    if (auto *env = dynamic_cast<bp::environment *>(&a.bound_env()))
      if (env->bound_session() &&
          a.bound_buffer().device_state().get() == env->bound_session())
        throw xeno::error("xylo-hip: host step of a device-bound env into "
                          "its own device window's replay buffer");
  }
  static void materialise(replay_buffer<A, S> &rb) {
    if (rb.device_state()) bp::device::session_of(rb).materialise(rb);
  }
  static void forget(replay_buffer<A, S> &rb) {
    if (rb.device_state()) bp::device::session_of(rb).forget();
  }
};

}  // namespace xylo

#endif  // XYLO_HIP_COMPAT_BIN_PACKING_DEVICE_H_
