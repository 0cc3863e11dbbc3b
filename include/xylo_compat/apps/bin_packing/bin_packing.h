// apps/bin_packing/bin_packing.h (xylo-hip drop-in layer).
//
// The reference's bin-packing types (bin_packing.h:10-153) -- observation,
// environment, agent, pg/ac/ppo/kl_ppo learners -- with the same names and
// constructors, plus the device session that runs them on the GPU through the
// C ABI (include/xylo_hip.h):
//
//   * agent.play_steps(T) with a policy_gradient_policy enqueues the agent's
//     env into the current window; the first engine draw or learner.step()
//     after that runs ONE batched rollout of every enqueued env
//     (xh_trainer_rollout), with each env's draws at the position the
//     reference's sequential order gives it (xh_trainer_seed_streams);
//   * learner.step() runs the learner on the device (xh_trainer_learn) and
//     leaves the parameters there; model::parameters() pulls them lazily;
//   * agent.play_one_episode() with a policy_gradient_deterministic_policy
//     plays on the device (xh_trainer_evaluate) and the chosen actions are
//     replayed through the host env to fill the replay buffer, so the
//     trajectories, rewards and engine state are the reference's;
//   * replay_buffer.sample_td() materialises the window's trajectories from
//     the device buffers.
// Agents with host policies (random / firstfit / bestfit / minwaste) step the
// host env exactly as in the reference.
//
// Knobs (environment): XYLO_SEED (engine seed, tensor.h), XYLO_HIP_DEVICE,
// XYLO_HIP_MAX_STEPS=n (exit(0) after n learner steps) and XYLO_HIP_DUMP=
// prefix (write <prefix>.json + raw float32 parameter files at that exit).
#ifndef XYLO_HIP_COMPAT_BIN_PACKING_H_
#define XYLO_HIP_COMPAT_BIN_PACKING_H_

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <memory>
#include <random>
#include <sstream>
#include <string>
#include <typeinfo>
#include <vector>

#include <xylo/nn.h>
#include <xylo/policy_gradient.h>
#include <xylo_hip.h>

#ifndef XYLO_BP_NUM_BINS
#define XYLO_BP_NUM_BINS 8
#endif

namespace bp {

constexpr std::size_t num_bins = XYLO_BP_NUM_BINS;

using action = xylo::discrete_action<num_bins>;

struct observation {
  static std::size_t length() { return 4 * num_bins; }

  static constexpr std::pair<int, int> capacity{8, 8};

  observation(const std::pair<int, int> &bin_shape)
      : bins(num_bins, bin_shape), item{0, 0} {}
  observation() : observation(capacity) {}

  std::string to_string() const {
    std::ostringstream oss;
    oss << "item: " << xeno::string::streamable(item) << "; ";
    oss << "bins: " << xeno::string::streamable(bins);
    return oss.str();
  }

  // bin_packing.h:31-40: per bin [bin / cap, item / cap].
  void to_vector(xylo::vector_view o) const {
    for (std::size_t i = 0; i < bins.size(); ++i) {
      o[4 * i + 0] = float(bins[i].first) / capacity.first;
      o[4 * i + 1] = float(bins[i].second) / capacity.second;
      o[4 * i + 2] = float(item.first) / capacity.first;
      o[4 * i + 3] = float(item.second) / capacity.second;
    }
  }

  std::vector<std::pair<int, int>> bins;
  std::pair<int, int> item;
};

namespace device {
class session;
}

class environment : public xylo::environment<action, observation> {
 public:
  static constexpr std::pair<int, int> capacity{8, 8};
  static constexpr std::pair<int, int> shape1{4, 2};
  static constexpr std::pair<int, int> shape2{1, 2};

  environment() : state_(capacity), dist_(0.4) { get_item(); }
  environment(environment &&o)
      : state_(std::move(o.state_)), dist_(o.dist_) {
    if (o.bound_) throw xeno::error("moving a device-bound environment");
  }
  environment(const environment &) = delete;
  ~environment() override;

  // bin_packing.h:53-64.  A device-bound env's state lives in the trainer's
  // HBM buffers: it is viewed from there, changed here with the same engine
  // draws, and written back as the state its next rollout starts from.
  void apply(const action &a, std::size_t) override {
    if (bound_) {
      observation s = view(0);
      apply_to(s, a);
      bound_write(s);
      return;
    }
    apply_to(state_, a);
  }
  observation view(std::size_t) const override;
  // bin_packing.h:67-70
  void reset(std::size_t) override {
    observation s(capacity);
    s.item = draw_item();
    if (bound_)
      bound_write(s);
    else
      state_ = std::move(s);
  }

  // ---- device binding ----------------------------------------------------
  const observation &host_state() const { return state_; }
  device::session *bound_session() const { return bound_; }
  void bind(device::session *s, int index) {
    bound_ = s;
    index_ = index;
  }
  int bound_index() const { return index_; }

 private:
  void apply_to(observation &s, const action &a) {
    std::pair<int, int> &bin = s.bins[a.choice];
    bin.first -= s.item.first;
    bin.second -= s.item.second;
    if (bin.first < 0 || bin.second < 0) return;
    s.item = draw_item();
  }
  void bound_write(const observation &s);  // bin_packing_device.h
  // bin_packing.h:76-81: 2 engine draws (generate_canonical<double>).
  std::pair<int, int> draw_item() {
    return dist_(xylo::default_generator()) ? shape1 : shape2;
  }
  void get_item() { state_.item = draw_item(); }

  observation state_;
  std::bernoulli_distribution dist_;
  device::session *bound_ = nullptr;
  int index_ = -1;
};

// bin_packing.h:84-107
class agent : public xylo::agent<action, observation> {
 public:
  agent(const xylo::policy<action, observation> &p, environment &env,
        xylo::replay_buffer<action, observation> &rb)
      : xylo::agent<action, observation>(p, env, rb) {}

 protected:
  bool game_over(const observation &ob) override {
    for (const auto &bin : ob.bins)
      if (bin.first < 0 || bin.second < 0) return true;
    return false;
  }
  float get_reward(const observation &, const observation &ob) override {
    return game_over(ob) ? 0 : 1;
  }
};

// bin_packing.h:109-152
class pg_learner : public xylo::policy_gradient_learner<action, observation> {
 public:
  pg_learner(xylo::replay_buffer<action, observation> &rb,
             xylo::model &action_model, xylo::optimizer &action_optimizer,
             float gamma = 0.99)
      : xylo::policy_gradient_learner<action, observation>(
            rb, action_model, action_optimizer, gamma) {}

 protected:
  // this exact class runs the fused device learner (policy_gradient.h)
  bool device_fused() const override {
    return typeid(*this) == typeid(pg_learner) &&
           xylo::detail::device_fusable<action, observation>(this->desc());
  }
};

class ac_learner : public xylo::actor_critic_learner<action, observation> {
 public:
  ac_learner(xylo::replay_buffer<action, observation> &rb,
             xylo::model &action_model, xylo::optimizer &action_optimizer,
             xylo::model &value_model, xylo::optimizer &value_optimizer,
             float gamma = 0.99)
      : xylo::actor_critic_learner<action, observation>(
            rb, action_model, action_optimizer, value_model, value_optimizer,
            gamma) {}

 protected:
  // this exact class runs the fused device learner (policy_gradient.h)
  bool device_fused() const override {
    return typeid(*this) == typeid(ac_learner) &&
           xylo::detail::device_fusable<action, observation>(this->desc());
  }
};

class ppo_learner : public xylo::ppo_learner<action, observation> {
 public:
  ppo_learner(xylo::replay_buffer<action, observation> &rb,
              xylo::model &action_model, xylo::optimizer &action_optimizer,
              xylo::model &value_model, xylo::optimizer &value_optimizer,
              float gamma = 0.99)
      : xylo::ppo_learner<action, observation>(rb, action_model,
                                               action_optimizer, value_model,
                                               value_optimizer, gamma) {}

 protected:
  // this exact class runs the fused device learner (policy_gradient.h)
  bool device_fused() const override {
    return typeid(*this) == typeid(ppo_learner) &&
           xylo::detail::device_fusable<action, observation>(this->desc());
  }
};

class kl_ppo_learner : public xylo::kl_ppo_learner<action, observation> {
 public:
  kl_ppo_learner(xylo::replay_buffer<action, observation> &rb,
                 xylo::model &action_model, xylo::optimizer &action_optimizer,
                 xylo::model &value_model, xylo::optimizer &value_optimizer,
                 float gamma = 0.99)
      : xylo::kl_ppo_learner<action, observation>(rb, action_model,
                                                  action_optimizer, value_model,
                                                  value_optimizer, gamma) {}

 protected:
  // this exact class runs the fused device learner (policy_gradient.h)
  bool device_fused() const override {
    return typeid(*this) == typeid(kl_ppo_learner) &&
           xylo::detail::device_fusable<action, observation>(this->desc());
  }
};

}  // namespace bp

#include <apps/bin_packing/bin_packing_device.h>

#endif  // XYLO_HIP_COMPAT_BIN_PACKING_H_
