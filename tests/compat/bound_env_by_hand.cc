// Test program, built twice: against the real reference headers (the golden
// run, tests/golden/make_compat_golden.py) and against include/xylo_compat
// (the device run, tests/test_gpu_compat.py).  It trains 8 agents for two
// windows (their envs then live on the device in the drop-in build), then
// drives those envs BY HAND through the reference API -- environment::apply /
// reset / view (bin_packing.h:53-70), a host random_policy agent stepping one
// of them (rl.h:305-349), a stochastic policy's react on a host env
// (policy_gradient.h:343-350 -> model::eval) and model::eval itself
// (nn.h:473-479) -- and prints every state, the engine position and the
// probabilities.  lr = 0 keeps the parameters at their seeded init, so the
// sampled actions of both builds agree.
#include <cstdio>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include <apps/bin_packing/bin_packing.h>

static void dump(const char *tag, const bp::observation &o) {
  std::printf("%s item %d %d bins", tag, o.item.first, o.item.second);
  for (const auto &b : o.bins) std::printf(" %d,%d", b.first, b.second);
  std::printf("\n");
}

static unsigned long engine() {
  std::ostringstream os;
  os << xylo::default_generator();
  return std::stoul(os.str());
}

int main() {
  xylo::default_generator().seed(11);
  xylo::model actor;
  actor.add_layer(std::make_unique<xylo::convolution1d_1_layer>(4, 128));
  actor.add_layer(std::make_unique<xylo::relu_activation>());
  actor.add_layer(std::make_unique<xylo::convolution1d_1_layer>(128, 64));
  actor.add_layer(std::make_unique<xylo::relu_activation>());
  actor.add_layer(std::make_unique<xylo::convolution1d_1_layer>(64, 1));
  actor.add_layer(std::make_unique<xylo::softmax_layer>());
  xylo::model value;
  value.add_layer(std::make_unique<xylo::full_layer>(4 * bp::num_bins, 64));
  value.add_layer(std::make_unique<xylo::relu_activation>());
  value.add_layer(std::make_unique<xylo::full_layer>(64, 32));
  value.add_layer(std::make_unique<xylo::relu_activation>());
  value.add_layer(std::make_unique<xylo::full_layer>(32, 1));
  xylo::sgd_optimizer aopt(actor, 0.0f), vopt(value, 0.0f);
  xylo::replay_buffer<bp::action, bp::observation> rb;
  bp::ppo_learner learner(rb, actor, aopt, value, vopt);
  xylo::policy_gradient_policy<bp::action, bp::observation> pol(actor);

  const int W = 8;  // the device trainer packs 64 / num_bins envs per group
  std::vector<std::unique_ptr<bp::environment>> envs;
  std::vector<std::unique_ptr<bp::agent>> agents;
  for (int i = 0; i < W; ++i) envs.push_back(std::make_unique<bp::environment>());
  for (int i = 0; i < W; ++i)
    agents.push_back(std::make_unique<bp::agent>(pol, *envs[i], rb));
  for (int round = 0; round < 2; ++round) {
    for (auto &a : agents) a->play_steps(4);
    learner.step();
    rb.forget();
    std::printf("round %d engine %lu\n", round, engine());
  }
  for (int i = 0; i < W; ++i) dump("trained", envs[i]->view(0));

  // by hand on the trained envs
  bp::action x;
  x.choice = 3;
  envs[0]->apply(x, 0);
  x.choice = 3;
  envs[0]->apply(x, 0);
  envs[1]->reset(0);
  dump("env0", envs[0]->view(0));
  dump("env1", envs[1]->view(0));
  std::printf("engine %lu\n", engine());

  // a host random_policy agent on a trained env (its own replay buffer)
  xylo::random_policy<bp::num_bins, bp::observation> rp;
  xylo::replay_buffer<bp::action, bp::observation> rb2;
  bp::agent ra(rp, *envs[2], rb2);
  for (int s = 0; s < 6; ++s) ra.step();
  dump("env2", envs[2]->view(0));
  std::printf("engine %lu\n", engine());

  // the stochastic policy's react on a host env (model::eval + sampling)
  bp::environment henv;
  xylo::replay_buffer<bp::action, bp::observation> rb3;
  bp::agent ha(pol, henv, rb3);
  for (int s = 0; s < 5; ++s) ha.step();
  dump("henv", henv.view(0));
  std::printf("engine %lu\n", engine());

  // model::eval on one observation
  xylo::vector v = xylo::to_vector(envs[3]->view(0));
  xylo::matrix p = actor.eval(xylo::fold<2>(v, {1, v.size()}));
  std::printf("probs");
  for (std::size_t j = 0; j < bp::num_bins; ++j) std::printf(" %.5f", p[0][j]);
  std::printf("\n");
  return 0;
}
