// The weight writer of the drop-in layer, xylo::save_parameters
// (include/xylo_compat/xylo/nn.h), round-tripped through the reference's own
// loading path: model::set_parameters on an xeno::sys::mmap<float> of the
// file (apps/bin_packing/deep_agent.cc:21-23, xylo/nn.h:490-508).
//
//   save_weights copy <in> <out>   deep_agent's network: <in> mapped and set,
//                                  saved to <out>, <out> mapped into a fresh
//                                  model; prints "equal <n>" when every
//                                  parameter came back bit for bit
//   save_weights train <out>       ppo_training.cc's networks on the device
//                                  (8 workers x 4 steps, two learner.step()),
//                                  then save_parameters of the trained policy
//                                  (pulled from the device); prints
//                                  "params <n> <sum as %.17g>" of parameters()
#include <cstdio>
#include <cstring>
#include <string>

#include <xeno/sys/file_descriptor.h>
#include <xylo/nn.h>
#include <xylo/rl.h>

#include <apps/bin_packing/bin_packing.h>

namespace {

void deep_agent_net(xylo::model &m) {
  m.add_layer(std::make_unique<xylo::convolution1d_1_layer>(4, 128));
  m.add_layer(std::make_unique<xylo::relu_activation>());
  m.add_layer(std::make_unique<xylo::convolution1d_1_layer>(128, 64));
  m.add_layer(std::make_unique<xylo::relu_activation>());
  m.add_layer(std::make_unique<xylo::convolution1d_1_layer>(64, 1));
}

int copy(const char *in, const char *out) {
  xylo::model a;
  deep_agent_net(a);
  xeno::sys::mmap f = xeno::sys::mmap<float>(in);
  a.set_parameters(xylo::borrow_vector(f.span()));
  xylo::save_parameters(a, out);

  xylo::model b;
  deep_agent_net(b);
  xeno::sys::mmap g = xeno::sys::mmap<float>(out);
  b.set_parameters(xylo::borrow_vector(g.span()));
  const xylo::vector pa = a.parameters(), pb = b.parameters();
  if (pa.size() != pb.size() || g.span().size() != pa.size()) {
    std::printf("size mismatch %zu %zu %zu\n", pa.size(), pb.size(),
                g.span().size());
    return 1;
  }
  if (std::memcmp(pa.data(), pb.data(), pa.size() * sizeof(float)) != 0) {
    std::printf("parameters differ\n");
    return 1;
  }
  std::printf("equal %zu\n", pa.size());
  return 0;
}

int train(const char *out) {
  constexpr int num_workers = 8, steps_per_worker = 4;
  xylo::model action_model;
  action_model.add_layer(std::make_unique<xylo::convolution1d_1_layer>(4, 128));
  action_model.add_layer(std::make_unique<xylo::relu_activation>());
  action_model.add_layer(std::make_unique<xylo::convolution1d_1_layer>(128, 64));
  action_model.add_layer(std::make_unique<xylo::relu_activation>());
  action_model.add_layer(std::make_unique<xylo::convolution1d_1_layer>(64, 1));
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
  for (int it = 0; it < 2; ++it) {
    for (auto &agent : agents) agent.play_steps(steps_per_worker);
    learner.step();
    replay_buffer.forget();
  }
  xylo::save_parameters(action_model, out);  // pulls the device copy
  const xylo::vector p = action_model.parameters();
  double sum = 0;
  for (float v : p) sum += v;
  std::printf("params %zu %.17g\n", p.size(), sum);
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc == 4 && std::string(argv[1]) == "copy") return copy(argv[2], argv[3]);
  if (argc == 3 && std::string(argv[1]) == "train") return train(argv[2]);
  std::fprintf(stderr, "usage: save_weights copy <in> <out> | train <out>\n");
  return 2;
}
