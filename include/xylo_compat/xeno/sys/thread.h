// xeno/sys/thread.h (xylo-hip drop-in layer).
//
// The reference runs each worker's agent.play_steps() on its own pthread
// (xeno/sys/thread.h:14-48, ppo_training.cc:47-62), racing on the one global
// engine.  Here a worker's closure runs inline at run(): with device policies
// play_steps() only enqueues its env into the device batch, so there is no
// host work to overlap, and the run is deterministic (reference order: worker
// 0, worker 1, ...).
#ifndef XYLO_HIP_COMPAT_XENO_SYS_THREAD_H_
#define XYLO_HIP_COMPAT_XENO_SYS_THREAD_H_

#include <functional>
#include <stdexcept>
#include <string>
#include <string_view>

namespace xeno {
namespace sys {

class thread {
 public:
  explicit thread(std::string_view name = "") : name_(name) {}
  thread(const thread &) = delete;
  void operator=(const thread &) = delete;

  template <typename F, typename... Args> void run(F &&f, Args &&...args) {
    if (joinable()) throw std::runtime_error("launching on joinable thread");
    running_ = true;
    std::invoke(std::forward<F>(f), std::forward<Args>(args)...);
  }

  void set_name(std::string_view s) { name_ = s; }
  std::string_view get_name() { return name_; }
  bool joinable() { return running_; }
  void join() { running_ = false; }
  void cancel() {}

 private:
  std::string name_;
  bool running_ = false;
};

class thread_pool {
 public:
  explicit thread_pool(std::size_t) {}
};

}  // namespace sys
}  // namespace xeno

#endif  // XYLO_HIP_COMPAT_XENO_SYS_THREAD_H_
