// xylo/policy_gradient.h (xylo-hip drop-in layer): the loss functions,
// learners and policies of policy_gradient.h:14-373 with the reference's
// names, constructors and public members.
//
// Two ways a learner's learn() runs:
//   fused     the library's own learner classes on a device-bound replay
//             buffer (the bin-packing types, device_traits): the whole update
//             -- value step, TD targets, GAE, k epochs, optimizer steps -- is
//             one device trainer call (xh_trainer_learn);
//   composed  everything else -- a learner class of the caller's own (e.g. one
//             that overrides optimize_action), custom layers or optimizers,
//             other action / state types: the reference's learn() body on the
//             host, whose pieces run on the device (model::eval / forward /
//             gradient, the batched loss gradients below, optimizer
//             next_parameters; include/xylo_hip.h).
// device_fused() picks between them: the exact library class and a device
// learner that can take the models and optimizers.
#ifndef XYLO_HIP_COMPAT_POLICY_GRADIENT_H_
#define XYLO_HIP_COMPAT_POLICY_GRADIENT_H_

#include <cmath>
#include <functional>
#include <typeinfo>

#include <xylo/rl.h>
#include <xylo/tensor.h>

namespace xylo {

// What a device learner needs to know about its host-side description.
enum class learner_kind { reinforce, actor_critic, ppo, kl_ppo };

struct learner_desc {
  learner_kind kind;
  model *action_model;
  optimizer *action_optimizer;
  model *value_model;          // nullptr for REINFORCE
  optimizer *value_optimizer;  // nullptr for REINFORCE
  float gamma;
  float lambda = 0.95f;        // policy_gradient.h:286
  // evaluated once the learner is constructed: false = the composed path
  std::function<bool()> fused;
};

namespace detail {
template <typename A, typename S>
void device_learn(replay_buffer<A, S> &rb, const learner_desc &d) {
  if constexpr (device_traits<A, S>::enabled) {
    device_traits<A, S>::learn(rb, d);
  } else {
    (void)rb;
    (void)d;
    throw xeno::error("xylo-hip: no device learner for these action/state "
                      "types (specialise xylo::device_traits)");
  }
}
template <typename A, typename S>
void device_attach(replay_buffer<A, S> &rb, const learner_desc &d) {
  if constexpr (device_traits<A, S>::enabled) device_traits<A, S>::attach(rb, d);
}
// whether the device learner of these types can take this description
template <typename A, typename S>
bool device_fusable(const learner_desc &d) {
  if constexpr (device_traits<A, S>::enabled)
    return device_traits<A, S>::fusable(d);
  else
    return (void)d, false;
}
// a composed learn() consumed the device window (the trainer forgets it)
template <typename A, typename S>
void device_learned_on_host(replay_buffer<A, S> &rb) {
  if constexpr (device_traits<A, S>::enabled)
    device_traits<A, S>::learned_on_host(rb);
}

// One flat row per action: choice, sampling distribution (if needed),
// advantage -> the device's batched loss gradient (xh_action_loss_grad).
template <typename A>
matrix action_loss(int kind, const std::vector<A> &actions,
                   vector_view advantages, matrix_view orig, float param) {
  const std::size_t rows = actions.size(), range = A::cardinality();
  if (orig.num_rows() != rows || orig.num_cols() != range ||
      advantages.size() < rows)
    throw std::exception();  // as the reference's per-row size checks
  matrix result({rows, range});
  if (!rows) return result;
  std::vector<std::int32_t> choice(rows);
  std::vector<float> q;
  const bool need_q = kind != XH_LOSS_SOFTMAX_GRADIENT_LOG;
  if (need_q) q.resize(rows * range);
  for (std::size_t i = 0; i < rows; ++i) {
    choice[i] = std::int32_t(actions[i].choice);
    if (!need_q) continue;
    if (!actions[i].distrib || actions[i].distrib->size() != range)
      throw xeno::error("xylo-hip: an action without its sampling distribution");
    std::copy(actions[i].distrib->begin(), actions[i].distrib->end(),
              q.begin() + i * range);
  }
  hip_check(xh_action_loss_grad(hip_context(), kind, int(rows), int(range),
                                choice.data(), need_q ? q.data() : nullptr,
                                advantages.data(), orig.flatten().data(), param,
                                matrix_view(result).flatten().data()),
            "action loss gradient");
  return result;
}
}  // namespace detail

// policy_gradient.h:15-22
template <typename A, typename S>
inline std::size_t num_transitions(const std::vector<td<A, S>> &experience) {
  std::size_t result = 0;
  for (const auto &traj : experience) result += traj.size();
  return result;
}

// policy_gradient.h:24-34: softmax_gradient_log per row (on the device)
template <typename A>
inline matrix policy_loss(const std::vector<A> &actions, vector_view advantages,
                          matrix_view orig_action_matrix) {
  return detail::action_loss(XH_LOSS_SOFTMAX_GRADIENT_LOG, actions, advantages,
                             orig_action_matrix, 0.0f);
}

// policy_gradient.h:36-46: clipped_gradient per row (on the device)
template <typename A>
inline matrix surrogate_loss(const std::vector<A> &actions,
                             vector_view advantages,
                             matrix_view orig_action_matrix) {
  return detail::action_loss(XH_LOSS_CLIPPED, actions, advantages,
                             orig_action_matrix, 0.2f);
}

// policy_gradient.h:48-53: D_KL(P || Q)
inline float kl_divergence(vector_view p, vector_view q) {
  if (p.size() != q.size()) throw std::exception();
  float s = 0.0f;
  for (std::size_t i = 0; i < p.size(); ++i) s += p[i] * std::log(p[i] / q[i]);
  return s;
}

// policy_gradient.h:55-85: softmax_gradient_log + beta (p - q) per row (on
// the device, with the beta the call starts from), then beta adapted to the
// mean KL of the batch (host).
template <typename A>
inline matrix kl_regulated_loss(const std::vector<A> &actions,
                                vector_view advantages, float d_targ,
                                float &beta, matrix_view orig_action_matrix) {
  matrix result = detail::action_loss(XH_LOSS_KL_REGULATED, actions, advantages,
                                      orig_action_matrix, beta);
  float d_average = 0;
  for (std::size_t i = 0; i < actions.size(); ++i)
    d_average += kl_divergence(*actions[i].distrib, orig_action_matrix[i]);
  d_average /= actions.size();
  if (std::abs(d_average) < d_targ / 1.5) {
    beta /= 2;
  } else if (std::abs(d_average) > d_targ * 1.5) {
    beta *= 2;
  }
  beta = std::max<float>(beta, 1e-25);
  beta = std::min<float>(beta, 0.1);
  return result;
}

// REINFORCE (policy_gradient.h:88-147).
template <typename A, typename S>
class policy_gradient_learner : public learner<A, S> {
 public:
  policy_gradient_learner(replay_buffer<A, S> &rb, model &action_model,
                          optimizer &action_optimizer, float gamma = 1)
      : learner<A, S>(rb, action_model, action_optimizer, gamma) {
    detail::device_attach(rb, desc());
  }

  void learn() override {
    if (device_fused()) {
      detail::device_learn(this->replay_buffer_, desc());
      return;
    }
    // policy_gradient.h:95-123
    std::vector<td<A, S>> experience = this->replay_buffer_.sample_td();
    matrix state_matrix({num_transitions(experience), S::length()});
    std::size_t curr = 0;
    std::vector<A> actions;
    for (const auto &traj : experience)
      for (const auto &transition : traj) {
        transition.start_state->to_vector(state_matrix[curr]);
        actions.push_back(transition.action);
        ++curr;
      }
    vector advantages = get_advantages(experience);
    this->policy_optimizer_.step(state_matrix, [&](matrix_view v) -> matrix {
      return policy_loss(actions, advantages, v);
    });
    detail::device_learned_on_host(this->replay_buffer_);
  }

  // policy_gradient.h:125-146: reversed discounted rewards-to-go minus the
  // mean trajectory return
  vector get_advantages(const std::vector<td<A, S>> &experience) {
    vector rewards_to_go({num_transitions(experience)});
    const float discount = this->gamma_;
    float total_reward = 0;
    std::size_t curr = 0;
    for (const auto &traj : experience) {
      vector_view reward_slice = slice(rewards_to_go, curr, traj.size());
      // the reference's loop: the first transition's reward lands in the last
      // slot, one slot down per transition
      std::size_t k = reward_slice.size();
      float reward = 0;
      for (auto traj_pos = traj.begin(); traj_pos != traj.end() && k > 0;) {
        reward = (traj_pos++)->reward + discount * reward;
        reward_slice[--k] = reward;
      }
      total_reward += reward_slice[0];
      curr += traj.size();
    }
    const float avg_reward = total_reward / experience.size();
    for (float &r : rewards_to_go) r = r - avg_reward;
    return rewards_to_go;
  }

 protected:
  virtual bool device_fused() const {
    return typeid(*this) == typeid(policy_gradient_learner) &&
           detail::device_fusable<A, S>(desc());
  }
  learner_desc desc() const {
    auto *self = const_cast<policy_gradient_learner *>(this);
    return {learner_kind::reinforce, &self->policy_model_,
            &self->policy_optimizer_, nullptr, nullptr, this->gamma_, 0.95f,
            [self] { return self->device_fused(); }};
  }
};

// Online actor-critic (policy_gradient.h:150-288).
template <typename A, typename S>
class actor_critic_learner : public learner<A, S> {
 public:
  actor_critic_learner(replay_buffer<A, S> &rb, model &action_model,
                       optimizer &action_optimizer, model &value_model,
                       optimizer &value_optimizer, float gamma = 0.99)
      : learner<A, S>(rb, action_model, action_optimizer, gamma),
        value_model_(value_model), value_optimizer_(value_optimizer) {
    detail::device_attach(rb, desc());
  }

  void learn() override {
    if (device_fused()) {
      detail::device_learn(this->replay_buffer_, desc());
      return;
    }
    // policy_gradient.h:159-185
    std::vector<td<A, S>> experience = this->replay_buffer_.sample_td();
    const std::size_t total_num_transitions = num_transitions(experience);
    matrix state_matrix(
        {total_num_transitions + experience.size(), S::length()});
    std::vector<A> actions;
    std::size_t curr = 0;
    for (const auto &traj : experience) {
      for (const auto &transition : traj) {
        transition.start_state->to_vector(state_matrix[curr++]);
        actions.push_back(transition.action);
      }
      actions.push_back(actions.back());
      traj.back().end_state.to_vector(state_matrix[curr++]);
    }
    update_value_model(experience, state_matrix);
    vector advantage = calculate_advantage(experience, state_matrix);
    optimize_action(state_matrix, actions, advantage);
    detail::device_learned_on_host(this->replay_buffer_);
  }

  // policy_gradient.h:187-194
  virtual void optimize_action(matrix_view state_matrix,
                               const std::vector<A> &actions,
                               vector_view advantage) {
    this->policy_optimizer_.step(state_matrix, [&](matrix_view v) -> matrix {
      return policy_loss(actions, advantage, v);
    });
  }

  // policy_gradient.h:196-218: TD targets r + gamma V(next) (the end rows
  // keep their own value), one value optimizer step on the square loss
  void update_value_model(const std::vector<td<A, S>> &experience,
                          matrix_view state_matrix) {
    matrix value_matrix = value_model_.eval(state_matrix);
    vector_view values = matrix_view(value_matrix).flatten();
    std::size_t curr = 0;
    vector updated_values({values.size()});
    for (const auto &traj : experience) {
      for (const auto &transition : traj) {
        updated_values[curr] =
            transition.reward + this->gamma_ * values[curr + 1];
        ++curr;
      }
      updated_values[curr] = values[curr];
      ++curr;
    }
    value_optimizer_.step(state_matrix,
                          std::bind_front(square_loss_grad, updated_values));
  }

  // policy_gradient.h:220-281: GAE over each trajectory (V(end) zeroed for
  // the frozen ones), the reference's O(T^2) sums
  vector calculate_advantage(const std::vector<td<A, S>> &experience,
                             matrix_view state_matrix) {
    matrix value_matrix = value_model_.eval(state_matrix);
    vector_view values = matrix_view(value_matrix).flatten();
    vector advantage({values.size()});
    vector deltas({values.size()});
    std::size_t curr = 0;
    for (const auto &traj : experience) {
      curr += traj.size();
      if (traj.frozen()) values[curr] = 0;
      ++curr;
    }
    curr = 0;
    for (const auto &traj : experience) {
      for (const auto &transition : traj) {
        deltas[curr] = transition.reward + this->gamma_ * values[curr + 1] -
                       values[curr];
        ++curr;
      }
      deltas[curr] = 0;
      ++curr;
    }
    curr = 0;
    for (const auto &traj : experience) {
      const std::size_t traj_end = curr + traj.size();
      for (std::size_t k = 0; k < traj.size(); ++k) {
        advantage[curr] = 0;
        float coefficient = 1;
        for (std::size_t i = curr; i < traj_end; ++i) {
          advantage[curr] += deltas[i] * coefficient;
          coefficient *= lambda_ * this->gamma_;
        }
        ++curr;
      }
      advantage[curr] = 0;
      ++curr;
    }
    return advantage;
  }

 protected:
  virtual learner_kind kind() const { return learner_kind::actor_critic; }
  virtual bool device_fused() const {
    return typeid(*this) == typeid(actor_critic_learner) &&
           detail::device_fusable<A, S>(desc());
  }
  learner_desc desc() const {
    auto *self = const_cast<actor_critic_learner *>(this);
    return {kind(), &self->policy_model_, &self->policy_optimizer_,
            &value_model_, &value_optimizer_, this->gamma_, lambda_,
            [self] { return self->device_fused(); }};
  }
  // Derived constructors re-attach with their own kind.
  void reattach() { detail::device_attach(this->replay_buffer_, desc()); }

  model &value_model_;
  optimizer &value_optimizer_;
  float lambda_ = 0.95;
};

// PPO-clip, k = 4 full-batch epochs (policy_gradient.h:290-308).
template <typename A, typename S>
class ppo_learner : public actor_critic_learner<A, S> {
 public:
  ppo_learner(replay_buffer<A, S> &rb, model &action_model,
              optimizer &action_optimizer, model &value_model,
              optimizer &value_optimizer, float gamma = 0.99)
      : actor_critic_learner<A, S>(rb, action_model, action_optimizer,
                                   value_model, value_optimizer, gamma) {
    this->reattach();
  }
  void optimize_action(matrix_view state_matrix, const std::vector<A> &actions,
                       vector_view advantage) override {
    constexpr std::size_t k = 4;
    for (std::size_t i = 0; i < k; ++i)
      this->policy_optimizer_.step(state_matrix, [&](matrix_view v) -> matrix {
        return surrogate_loss(actions, advantage, v);
      });
  }

 protected:
  learner_kind kind() const override { return learner_kind::ppo; }
  bool device_fused() const override {
    return typeid(*this) == typeid(ppo_learner) &&
           detail::device_fusable<A, S>(this->desc());
  }
};

// KL-regulated PPO (policy_gradient.h:310-335).
template <typename A, typename S>
class kl_ppo_learner : public actor_critic_learner<A, S> {
 public:
  kl_ppo_learner(replay_buffer<A, S> &rb, model &action_model,
                 optimizer &action_optimizer, model &value_model,
                 optimizer &value_optimizer, float gamma = 0.99)
      : actor_critic_learner<A, S>(rb, action_model, action_optimizer,
                                   value_model, value_optimizer, gamma) {
    this->reattach();
  }
  void optimize_action(matrix_view state_matrix, const std::vector<A> &actions,
                       vector_view advantage) override {
    constexpr std::size_t k = 4;
    for (std::size_t i = 0; i < k; ++i)
      this->policy_optimizer_.step(state_matrix, [&](matrix_view v) -> matrix {
        return kl_regulated_loss(actions, advantage, d_targ_, beta_, v);
      });
  }

 protected:
  learner_kind kind() const override { return learner_kind::kl_ppo; }
  bool device_fused() const override {
    return typeid(*this) == typeid(kl_ppo_learner) &&
           detail::device_fusable<A, S>(this->desc());
  }

 private:
  float beta_ = 1;
  float d_targ_ = 1e-9;
};

// Stochastic policy (policy_gradient.h:338-353).  Batched play
// (agent::play_steps on bp envs) samples inside the device rollout; a single
// react() on a host state evaluates the model on the device (model::eval ->
// xh_model_eval) and samples from the global engine as the reference does.
template <typename A, typename S>
class policy_gradient_policy : public policy<A, S> {
 public:
  policy_gradient_policy(model &m) : m_(m) {}
  model &device_model() const { return m_; }

 protected:
  A react(const S &state) const override {
    vector v = to_vector(state);
    matrix out = m_.eval(fold<2>(vector_view(v), {1, v.size()}));
    A action;
    action.from_vector(flatten(out));
    return action;
  }

 private:
  model &m_;
};

// Argmax policy (policy_gradient.h:356-373): episodes play on the device
// (agent::play_one_episode on bp envs); react() on a host state evaluates on
// the device and takes the argmax.
template <typename A, typename S>
class policy_gradient_deterministic_policy : public policy<A, S> {
 public:
  policy_gradient_deterministic_policy(model &m) : m_(m) {}
  model &device_model() const { return m_; }

 protected:
  A react(const S &state) const override {
    vector v = to_vector(state);
    matrix out = m_.eval(fold<2>(vector_view(v), {1, v.size()}));
    A action;
    action.from_vector_deterministic(flatten(out));
    return action;
  }

 private:
  model &m_;
};

}  // namespace xylo

#endif  // XYLO_HIP_COMPAT_POLICY_GRADIENT_H_
