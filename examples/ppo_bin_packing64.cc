// PPO on 2-D bin packing with 64 bins (BASELINE config 3 per GPU), written
// against the reference's own API (xylo:: / bp::, as in
// apps/bin_packing/ppo_training.cc) and compiled with the xylo-hip drop-in
// headers: the 32768 workers' play_steps() become one batched device rollout
// and learner.step() one device update.
//
//   build/compat/ppo_bin_packing64 [iterations=200] [workers=32768]
#define XYLO_BP_NUM_BINS 64

#include <chrono>
#include <cstdlib>

#include <xeno/sys/thread.h>
#include <xylo/nn.h>
#include <xylo/rl.h>

#include <apps/bin_packing/bin_packing.h>

int main(int argc, char **argv) {
  const int iterations = argc > 1 ? std::atoi(argv[1]) : 200;
  const int num_workers = argc > 2 ? std::atoi(argv[2]) : 32768;
  constexpr int steps_per_worker = 4;

  xylo::model action_model;
  action_model.add_layer(std::make_unique<xylo::convolution1d_1_layer>(4, 128));
  action_model.add_layer(std::make_unique<xylo::relu_activation>());
  action_model.add_layer(std::make_unique<xylo::convolution1d_1_layer>(128, 128));
  action_model.add_layer(std::make_unique<xylo::relu_activation>());
  action_model.add_layer(std::make_unique<xylo::convolution1d_1_layer>(128, 1));
  action_model.add_layer(std::make_unique<xylo::softmax_layer>());
  xylo::sgd_optimizer action_optimizer(action_model, 1e-4);

  xylo::model value_model;
  value_model.add_layer(std::make_unique<xylo::full_layer>(4 * bp::num_bins, 64));
  value_model.add_layer(std::make_unique<xylo::relu_activation>());
  value_model.add_layer(std::make_unique<xylo::full_layer>(64, 32));
  value_model.add_layer(std::make_unique<xylo::relu_activation>());
  value_model.add_layer(std::make_unique<xylo::full_layer>(32, 1));
  xylo::sgd_optimizer value_optimizer(value_model, 1e-5);

  xylo::replay_buffer<bp::action, bp::observation> replay_buffer;
  std::vector<bp::environment> envs;
  std::vector<bp::agent> agents;
  envs.reserve(num_workers);
  agents.reserve(num_workers);
  xylo::policy_gradient_policy<bp::action, bp::observation> policy(action_model);
  for (int i = 0; i < num_workers; ++i) {
    envs.emplace_back();
    agents.emplace_back(policy, envs[i], replay_buffer);
  }
  bp::ppo_learner learner(replay_buffer, action_model, action_optimizer,
                          value_model, value_optimizer, 0.99);

  auto t0 = std::chrono::steady_clock::now();
  for (int steps = 1; steps <= iterations; ++steps) {
    for (auto &agent : agents) agent.play_steps(steps_per_worker);
    learner.step();
    replay_buffer.forget();

    if (steps % 50 == 0) {
      xylo::vector p = action_model.parameters();  // waits for the device
      const double s = std::chrono::duration<double>(
                           std::chrono::steady_clock::now() - t0)
                           .count();
      lg() << "iteration " << steps << " env-steps/s "
           << double(steps) * num_workers * steps_per_worker / s;
      xylo::policy_gradient_deterministic_policy<bp::action, bp::observation>
          eval_policy(action_model);
      bp::environment env;
      xylo::replay_buffer<bp::action, bp::observation> rb;
      bp::agent agent(eval_policy, env, rb);
      for (int i = 0; i < 100; ++i) agent.play_one_episode();
      lg() << "round " << steps << " "
           << xylo::total_rewards<bp::action, bp::observation>(rb.sample_td()) /
                  100.0;
      rb.forget();
      t0 = std::chrono::steady_clock::now() -
           std::chrono::duration_cast<std::chrono::steady_clock::duration>(
               std::chrono::duration<double>(s));
    }
  }
  return 0;
}
