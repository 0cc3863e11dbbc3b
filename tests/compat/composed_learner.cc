// tests/compat/composed_learner.cc -- a learner assembled from the drop-in
// layer's public pieces, the way the reference's own learners are written
// (policy_gradient.h:159-185 learn -> :196-218 update_value_model -> :220-281
// calculate_advantage -> :297-307 ppo_learner::optimize_action with
// optimizer::step(state_matrix, surrogate_loss(...)), nn.h:594-605).  Built
// against include/xylo_compat only; every model / loss / optimizer piece runs
// on the device through include/xylo_hip.h.
//
//   composed_learner mode=subclass|pieces|fused N=8 T=8 iters=5 seed=42
//                    widths=128,64 out=PREFIX
//
// subclass: a learner class derived from xylo::ppo_learner that overrides
//           optimize_action (the reference's body);
// pieces:   a learner derived from xylo::actor_critic_learner whose learn()
//           builds the state matrix itself and calls the public
//           update_value_model / calculate_advantage, then four
//           optimizer::step(surrogate_loss) epochs;
// fused:    bp::ppo_learner (the device trainer's one-call learn), for A/B.
// The setup is ref_harness's learn mode (oracle/ref_harness.cc): engine
// seeded, per-bin policy conv(4,w1)-relu-conv(w1,w2)-relu-conv(w2,1)-softmax,
// value full(32,64)-relu-full(64,32)-relu-full(32,1), sgd 1e-4 / 1e-5, N
// agents stepped T steps each in order.  After iteration k the policy and
// value parameters go to PREFIX.it<k>.policy.bin / .value.bin (raw f32).
#include <apps/bin_packing/bin_packing.h>

#include <cstdio>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

using A = bp::action;
using S = bp::observation;

// the reference's ppo_learner::optimize_action, written by a caller
class my_ppo_learner : public xylo::ppo_learner<A, S> {
 public:
  using xylo::ppo_learner<A, S>::ppo_learner;
  void optimize_action(xylo::matrix_view state_matrix,
                       const std::vector<A> &actions,
                       xylo::vector_view advantage) override {
    for (int i = 0; i < 4; ++i)
      this->policy_optimizer_.step(
          state_matrix, [&](xylo::matrix_view v) -> xylo::matrix {
            return xylo::surrogate_loss(actions, advantage, v);
          });
  }
};

// learn() assembled from the public pieces
class pieces_learner : public xylo::actor_critic_learner<A, S> {
 public:
  using xylo::actor_critic_learner<A, S>::actor_critic_learner;
  void learn() override {
    std::vector<xylo::td<A, S>> experience = this->replay_buffer_.sample_td();
    const std::size_t rows = xylo::num_transitions(experience) + experience.size();
    xylo::matrix state_matrix({rows, S::length()});
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
    this->update_value_model(experience, state_matrix);
    xylo::vector advantage = this->calculate_advantage(experience, state_matrix);
    for (int i = 0; i < 4; ++i)
      this->policy_optimizer_.step(
          state_matrix, [&](xylo::matrix_view v) -> xylo::matrix {
            return xylo::surrogate_loss(actions, advantage, v);
          });
  }
};

static void write(const std::string &path, xylo::vector v) {
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char *>(v.data()), v.size() * sizeof(float));
}

int main(int argc, char **argv) {
  std::map<std::string, std::string> a;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto p = s.find('=');
    if (p != std::string::npos) a[s.substr(0, p)] = s.substr(p + 1);
  }
  auto num = [&](const char *k, long d) {
    return a.count(k) ? std::stol(a[k]) : d;
  };
  const std::string mode = a.count("mode") ? a["mode"] : "subclass";
  const int N = int(num("N", 8)), T = int(num("T", 8)), iters = int(num("iters", 5));
  std::vector<int> widths;
  {
    std::stringstream ss(a.count("widths") ? a["widths"] : "128,64");
    std::string tok;
    while (std::getline(ss, tok, ',')) widths.push_back(std::stoi(tok));
  }
  xylo::default_generator().seed(std::uint32_t(num("seed", 42)));

  xylo::model pol, val;
  int prev = 4;
  for (int w : widths) {
    pol.add_layer(std::make_unique<xylo::convolution1d_1_layer>(prev, w));
    pol.add_layer(std::make_unique<xylo::relu_activation>());
    prev = w;
  }
  pol.add_layer(std::make_unique<xylo::convolution1d_1_layer>(prev, 1));
  pol.add_layer(std::make_unique<xylo::softmax_layer>());
  prev = int(S::length());
  for (int w : {64, 32}) {
    val.add_layer(std::make_unique<xylo::full_layer>(prev, w));
    val.add_layer(std::make_unique<xylo::relu_activation>());
    prev = w;
  }
  val.add_layer(std::make_unique<xylo::full_layer>(prev, 1));
  xylo::sgd_optimizer opt_pi(pol, 1e-4f), opt_v(val, 1e-5f);

  std::vector<bp::environment> envs;
  envs.reserve(N);
  for (int i = 0; i < N; ++i) envs.emplace_back();
  xylo::replay_buffer<A, S> rb;
  xylo::policy_gradient_policy<A, S> policy(pol);
  std::vector<bp::agent> agents;
  agents.reserve(N);
  for (int i = 0; i < N; ++i) agents.emplace_back(policy, envs[i], rb);

  std::unique_ptr<xylo::learner<A, S>> learner;
  if (mode == "subclass")
    learner = std::make_unique<my_ppo_learner>(rb, pol, opt_pi, val, opt_v);
  else if (mode == "pieces")
    learner = std::make_unique<pieces_learner>(rb, pol, opt_pi, val, opt_v);
  else
    learner = std::make_unique<bp::ppo_learner>(rb, pol, opt_pi, val, opt_v);

  const std::string out = a.count("out") ? a["out"] : "composed";
  for (int it = 0; it < iters; ++it) {
    for (auto &agt : agents) agt.play_steps(T);
    learner->step();
    rb.forget();
    write(out + ".it" + std::to_string(it) + ".policy.bin", pol.parameters());
    write(out + ".it" + std::to_string(it) + ".value.bin", val.parameters());
  }
  std::printf("composed_learner mode=%s N=%d T=%d iters=%d ok\n", mode.c_str(),
              N, T, iters);
  return 0;
}
