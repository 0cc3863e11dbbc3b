// xylo/rl.h (xylo-hip drop-in layer): actions (discrete_action with its loss
// gradients; the reference's continuous_action, rl.h:77-109, is not carried:
// no bin-packing app or learner on this path uses it), trajectories, replay buffer (sample_td,
// sample_transitions, forget), environment / policy / agent / learner
// interfaces (rl.h:17-392), same names and signatures.
//
// Device hook: `device_traits<A, S>` (disabled by default).  When an app
// header specialises it (apps/bin_packing/bin_packing.h does for the
// bin-packing types), agent::play_steps / play_one_episode with a device
// policy only *enqueue* work, the learner runs on the device, and the replay
// buffer materialises host trajectories from the device buffers on demand.
// Agents with host policies (firstfit_agent.cc & co.) step the host env
// exactly as the reference does.
#ifndef XYLO_HIP_COMPAT_RL_H_
#define XYLO_HIP_COMPAT_RL_H_

#include <algorithm>
#include <cmath>
#include <exception>
#include <functional>
#include <iterator>
#include <list>
#include <memory>
#include <mutex>
#include <optional>
#include <random>
#include <vector>

#include <xylo/nn.h>
#include <xylo/tensor.h>

namespace xylo {

template <typename A, typename S> struct device_traits {
  static constexpr bool enabled = false;
};

template <typename T> vector to_vector(const T &t) {
  vector result({t.length()});
  t.to_vector(result);
  return result;
}

// rl.h:22-75.  The per-action loss gradients are the reference's host
// expressions (one row each); the batched forms the learners use
// (policy_loss / surrogate_loss / kl_regulated_loss, policy_gradient.h) run
// on the device.
template <std::size_t range> struct discrete_action {
  static std::size_t cardinality() { return range; }
  std::size_t choice = 0;
  std::optional<vector> distrib;

  void from_vector(vector_view a) {
    choice = discrete_distribution(a);
    distrib = vector(a);
  }
  void from_vector_deterministic(vector_view a) { choice = argmax(a); }

  // rl.h:33-42
  void gradient_log(vector_view input, vector_view output,
                    float advantage) const {
    if (input.size() != range || output.size() != range)
      throw std::exception();
    output = 0;
    float log_action_grad = 1 / input[choice];
    float weighted_grad = log_action_grad * advantage * -1;
    float importance_grad = input[choice] / (*distrib)[choice] * weighted_grad;
    output[choice] = importance_grad;
  }

  // rl.h:44-52
  void softmax_gradient_log(vector_view input, vector_view output,
                            float advantage) const {
    if (input.size() != range || output.size() != range)
      throw std::exception();
    for (std::size_t i = 0; i < range; ++i) output[i] = input[i] * advantage;
    output[choice] -= advantage;
  }

  // rl.h:54-74 (epsilon 0.2)
  void clipped_gradient(vector_view input, vector_view output,
                        float advantage) const {
    constexpr float epsilon = 0.2;
    if (input.size() != range || output.size() != range)
      throw std::exception();
    output = 0;
    float ratio = input[choice] / (*distrib)[choice];
    float clipped_ratio = ratio;
    if (ratio > (1 + epsilon)) {
      clipped_ratio = 1 + epsilon;
    } else if (ratio < (1 - epsilon)) {
      clipped_ratio = 1 - epsilon;
    }
    float importance_grad =
        std::min(clipped_ratio * advantage, ratio * advantage) * -1;
    output[choice] = importance_grad / input[choice];
  }
};

template <typename A, typename S> struct transition {
  transition() = default;
  transition(const S &, A &&a, float r, S &&curr)
      : action(std::move(a)), reward(r), end_state(std::move(curr)) {}

  const S *start_state = nullptr;
  A action;
  float reward = 0;
  S end_state;
};

template <typename A, typename S> struct trajectory {
  trajectory(S &&o) : opening(std::move(o)), frozen(false) {}

  void add_transition(A &&a, float r, S &&curr) {
    transitions.emplace_back(last_state(), std::move(a), r, std::move(curr));
  }
  const S &last_state() {
    return transitions.empty() ? opening : transitions.back().end_state;
  }
  std::size_t size() const { return transitions.size(); }
  void fill_reference() {
    const S *prev = &opening;
    for (auto &tr : transitions) {
      tr.start_state = prev;
      prev = &tr.end_state;
    }
  }
  void freeze() {
    frozen = true;
    fill_reference();
  }

  S opening;
  std::list<transition<A, S>> transitions;
  bool frozen;
};

template <typename A, typename S> class environment {
 public:
  virtual ~environment() = default;
  virtual void apply(const A &action, std::size_t id) = 0;
  virtual S view(std::size_t id) const = 0;
  virtual void reset(std::size_t id) = 0;
};

template <typename A, typename S> class td {
 public:
  using container = std::list<transition<A, S>>;
  td(const trajectory<A, S> &traj)
      : frozen_(traj.frozen), size_(traj.transitions.size()),
        begin_(traj.transitions.begin()), end_(traj.transitions.end()),
        back_(&traj.transitions.back()) {}

  typename container::const_iterator begin() const { return begin_; }
  typename container::const_iterator end() const { return end_; }
  std::size_t size() const { return size_; }
  bool frozen() const { return frozen_; }
  const transition<A, S> &front() const { return *begin_; }
  const transition<A, S> &back() const { return *back_; }

 private:
  bool frozen_;
  std::size_t size_;
  typename container::const_iterator begin_, end_;
  const transition<A, S> *back_;
};

template <typename A, typename S>
float total_rewards(const std::vector<td<A, S>> &experience) {
  float result = 0;
  for (const auto &traj : experience)
    for (const auto &tr : traj) result += tr.reward;
  return result;
}

template <typename A, typename S>
using transition_ref = std::reference_wrapper<transition<A, S>>;

template <typename A, typename S> class replay_buffer {
 public:
  trajectory<A, S> &emplace_trajectory(S &&s) {
    std::lock_guard l(mutex_);
    trajectories_.emplace_back(std::move(s));
    return trajectories_.back();
  }

  // rl.h:222-233: one td per trajectory, in list order.  Device-played
  // experience is materialised first.
  std::vector<td<A, S>> sample_td(std::size_t = -1, std::size_t = -1) {
    if constexpr (device_traits<A, S>::enabled)
      device_traits<A, S>::materialise(*this);
    std::vector<td<A, S>> result;
    for (auto &traj : trajectories_) {
      if (traj.size() == 0) continue;
      traj.fill_reference();
      result.emplace_back(traj);
    }
    return result;
  }

  // rl.h:236-272: n transitions drawn uniformly (with replacement) over the
  // buffer's transitions, from a std::random_device-seeded mt19937 as the
  // reference draws them (not reproducible run to run, as there).
  std::vector<transition_ref<A, S>> sample_transitions(std::size_t n) {
    if constexpr (device_traits<A, S>::enabled)
      device_traits<A, S>::materialise(*this);
    std::vector<transition_ref<A, S>> result;
    result.reserve(n);
    std::size_t total = 0;
    for (trajectory<A, S> &traj : trajectories_) total += traj.size();
    if (n && !total) throw xeno::error("sample_transitions: empty replay buffer");
    std::random_device rd;
    std::mt19937 gen(rd());
    std::uniform_int_distribution<> distrib(0, int(total) - 1);
    for (std::size_t i = 0; i < n; ++i) {
      std::size_t index = std::size_t(distrib(gen)), start = 0;
      transition<A, S> *p_trans = nullptr;
      for (trajectory<A, S> &traj : trajectories_) {
        const std::size_t end = start + traj.size();
        if (index < end) {
          auto pos = traj.transitions.begin();
          std::advance(pos, index - start);
          p_trans = &*pos;
          break;
        }
        start = end;
      }
      result.emplace_back(*p_trans);
    }
    return result;
  }

  // rl.h:274-291: drop frozen trajectories, keep the last state of open ones.
  void forget() {
    if constexpr (device_traits<A, S>::enabled)
      device_traits<A, S>::forget(*this);
    for (auto pos = trajectories_.begin(); pos != trajectories_.end();) {
      if (pos->frozen) {
        pos = trajectories_.erase(pos);
        continue;
      }
      if (!pos->transitions.empty()) {
        pos->opening = std::move(pos->transitions.back().end_state);
        pos->transitions.clear();
      }
      ++pos;
    }
  }

  std::list<trajectory<A, S>> &trajectories() { return trajectories_; }
  std::shared_ptr<void> &device_state() { return device_state_; }

 private:
  std::mutex mutex_;
  std::list<trajectory<A, S>> trajectories_;
  std::shared_ptr<void> device_state_;
};

template <typename A, typename S> class policy {
 public:
  virtual ~policy() = default;
  virtual A react(const S &state) const = 0;
};

// rl.h:298-312: uniform categorical (2 engine draws per react).
template <std::size_t N, typename S>
class random_policy : public policy<discrete_action<N>, S> {
 public:
  discrete_action<N> react(const S &) const override {
    vector v({N});
    v = 1.0f / N;
    discrete_action<N> a;
    a.from_vector(v);
    return a;
  }
};

template <typename A, typename S> class agent {
 public:
  explicit agent(const policy<A, S> &p, environment<A, S> &env,
                 replay_buffer<A, S> &rb, std::size_t id = 0)
      : id_(id), policy_(p), env_(env), replay_buffer_(rb) {}
  virtual ~agent() = default;

  // rl.h:325-349 (host stepping; device policies never come here).
  bool step() {
    if constexpr (device_traits<A, S>::enabled)
      device_traits<A, S>::before_host_step(*this);
    return step_with(policy_.react(curr_state()));
  }

  void play_one_episode() {
    if constexpr (device_traits<A, S>::enabled)
      if (device_traits<A, S>::play_episodes(*this, 1)) return;
    while (step()) {
    }
  }

  void play_steps(std::size_t n) {
    if constexpr (device_traits<A, S>::enabled)
      if (device_traits<A, S>::play_steps(*this, n)) return;
    for (std::size_t i = 0; i < n; ++i) step();
  }

  std::size_t id() { return id_; }

  // ---- used by device_traits ---------------------------------------------
  const policy<A, S> &bound_policy() const { return policy_; }
  environment<A, S> &bound_env() { return env_; }
  replay_buffer<A, S> &bound_buffer() { return replay_buffer_; }

  // One transition with a given action (the tail of rl.h:325-349); the
  // device path replays device-chosen actions through it.
  bool step_with(A &&action) {
    if (!curr_traj_)
      curr_traj_ = &replay_buffer_.emplace_trajectory(env_.view(id_));
    const S &previous_state = curr_traj_->last_state();
    env_.apply(action, id_);
    S curr_state = env_.view(id_);
    const float r = get_reward(previous_state, curr_state);
    curr_traj_->add_transition(std::move(action), r, std::move(curr_state));
    if (game_over(curr_traj_->last_state())) {
      env_.reset(id_);
      curr_traj_->freeze();
      curr_traj_ = nullptr;
      return false;
    }
    return true;
  }
  void drop_open_trajectory() { curr_traj_ = nullptr; }

 protected:
  virtual bool game_over(const S &state) = 0;
  virtual float get_reward(const S &state1, const S &state2) = 0;

  std::size_t id_;
  const policy<A, S> &policy_;
  environment<A, S> &env_;
  replay_buffer<A, S> &replay_buffer_;
  trajectory<A, S> *curr_traj_ = nullptr;

 private:
  S curr_state() {
    if (!curr_traj_)
      curr_traj_ = &replay_buffer_.emplace_trajectory(env_.view(id_));
    return curr_traj_->last_state();
  }
};

template <typename A, typename S> class learner {
 public:
  explicit learner(replay_buffer<A, S> &rb, model &policy_model,
                   optimizer &policy_optimizer, float gamma = 0.99)
      : replay_buffer_(rb), policy_model_(policy_model),
        policy_optimizer_(policy_optimizer), gamma_(gamma) {}
  virtual ~learner() = default;

  void step() { learn(); }
  virtual void learn() = 0;

 protected:
  replay_buffer<A, S> &replay_buffer_;
  model &policy_model_;
  optimizer &policy_optimizer_;
  float gamma_;
};

}  // namespace xylo

#endif  // XYLO_HIP_COMPAT_RL_H_
