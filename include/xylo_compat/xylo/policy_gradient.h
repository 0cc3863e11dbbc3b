// xylo/policy_gradient.h (xylo-hip drop-in layer): the learners and policies
// of policy_gradient.h:88-373 with the reference's constructors.  learn()
// hands the whole update (value step, TD targets, GAE, k surrogate epochs,
// SGD) to the device trainer through device_traits<A, S>; there is no host
// learner.
#ifndef XYLO_HIP_COMPAT_POLICY_GRADIENT_H_
#define XYLO_HIP_COMPAT_POLICY_GRADIENT_H_

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
}  // namespace detail

// REINFORCE (policy_gradient.h:88-147).
template <typename A, typename S>
class policy_gradient_learner : public learner<A, S> {
 public:
  policy_gradient_learner(replay_buffer<A, S> &rb, model &action_model,
                          optimizer &action_optimizer, float gamma = 1)
      : learner<A, S>(rb, action_model, action_optimizer, gamma) {
    detail::device_attach(rb, desc());
  }
  void learn() override { detail::device_learn(this->replay_buffer_, desc()); }

 private:
  learner_desc desc() {
    return {learner_kind::reinforce, &this->policy_model_,
            &this->policy_optimizer_, nullptr, nullptr, this->gamma_};
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
  void learn() override { detail::device_learn(this->replay_buffer_, desc()); }

 protected:
  virtual learner_kind kind() const { return learner_kind::actor_critic; }
  learner_desc desc() {
    return {kind(), &this->policy_model_, &this->policy_optimizer_,
            &value_model_, &value_optimizer_, this->gamma_, lambda_};
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

 protected:
  learner_kind kind() const override { return learner_kind::ppo; }
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

 protected:
  learner_kind kind() const override { return learner_kind::kl_ppo; }
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
