// Test program: the model + env prologue of ppo_training.cc (argv[1] = "ppo")
// or ac_training.cc ("ac") built with the drop-in headers, seeded by
// XYLO_SEED; writes the initial parameters (raw float32, policy then value)
// to argv[2] and "x_models x_envs item0 item1 ..." to stdout.  Host only: no
// device call is made.
#include <cstdio>
#include <fstream>
#include <string>

#include <xylo/nn.h>
#include <xylo/rl.h>

#include <apps/bin_packing/bin_packing.h>

int main(int argc, char **argv) {
  const bool ac = argc > 1 && std::string(argv[1]) == "ac";
  const int h1 = ac ? 64 : 128, h2 = ac ? 32 : 64, workers = ac ? 16 : 8;
  xylo::model action_model;
  action_model.add_layer(std::make_unique<xylo::convolution1d_1_layer>(4, h1));
  action_model.add_layer(std::make_unique<xylo::relu_activation>());
  action_model.add_layer(std::make_unique<xylo::convolution1d_1_layer>(h1, h2));
  action_model.add_layer(std::make_unique<xylo::relu_activation>());
  action_model.add_layer(std::make_unique<xylo::convolution1d_1_layer>(h2, 1));
  if (ac)
    action_model.add_layer(std::make_unique<xylo::softmax_cross_entropy_layer>());
  else
    action_model.add_layer(std::make_unique<xylo::softmax_layer>());
  xylo::model value_model;
  value_model.add_layer(std::make_unique<xylo::full_layer>(4 * bp::num_bins, 64));
  value_model.add_layer(std::make_unique<xylo::relu_activation>());
  value_model.add_layer(std::make_unique<xylo::full_layer>(64, 32));
  value_model.add_layer(std::make_unique<xylo::relu_activation>());
  value_model.add_layer(std::make_unique<xylo::full_layer>(32, 1));
  const auto x_models = bp::device::engine_state(xylo::default_generator());
  std::vector<bp::environment> envs;
  envs.reserve(workers);
  for (int i = 0; i < workers; ++i) envs.emplace_back();
  std::ofstream f(argv[2], std::ios::binary);
  for (xylo::model *m : {&action_model, &value_model}) {
    xylo::vector p = m->parameters();
    f.write(reinterpret_cast<const char *>(p.data()), p.size() * sizeof(float));
  }
  std::printf("%u %u", x_models, bp::device::engine_state(xylo::default_generator()));
  for (auto &e : envs) {
    bp::observation o = e.view(0);
    std::printf(" %d %d", o.item.first, o.item.second);
  }
  std::printf("\n");
  return 0;
}
