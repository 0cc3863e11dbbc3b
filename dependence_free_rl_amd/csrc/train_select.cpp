// train_select.cpp -- which policy train kernel an epoch launches (host code).
//
// Product kernels (libxylo_hip.so), f16 pairs + the exact bf16 split
// (DESIGN.md §3.0a-d):
//   64 bins, 2-D, [128,128] (configs 3 / 4)  policy_train_spec8_kernel
//                                  (KL-PPO: policy_train_spec8_kl_kernel;
//                                  XH_TRAIN_KERNEL=split8wh: the earlier
//                                  policy_train_split8wh_kernel)
//   128 bins, 3-D, [128,128] (config 5)      policy_train_split8x_kernel
//                                  (KL-PPO: policy_train_split8x_kl_kernel)
//   32 bins, 1-D, [64,64] (config 2)         policy_train_split4h_kernel
//                                  (KL-PPO: policy_train_split4h_kl_kernel;
//                                  XH_TRAIN_KERNEL=spec4: the wave-specialised
//                                  policy_train_spec4_kernel)
// and the f32-MFMA kernels of policy_kernels.hip for every other shape (KL-PPO
// included), and under XH_TRAIN_KERNEL=f32 (the accuracy reference of the split
// kernels' tests).
//
// The superseded config-3 / config-5 forms (split4w, split8w, split8wp,
// split4p, split8wg, split128) are built only into the variant library
// (`make variants` -> build/variants/libxylo_hip.so, loaded through
// XH_LIB_PATH for A/B runs, never by the product path): this file is compiled
// there with XH_VARIANT_KERNELS=1.  In the product library an override that
// names one of them fails the epoch with hipErrorNotSupported.
#include <cstdlib>
#include <cstring>

#include "xh_kernels.h"

#ifndef XH_VARIANT_KERNELS
#define XH_VARIANT_KERNELS 0
#endif

namespace xh {

#if XH_VARIANT_KERNELS
hipError_t launch_policy_train_split4w(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s);
#endif

// Diagnostic override, read per launch and reported by xh_trainer_kernel_info.
bool train_split_enabled() {
  const char *e = std::getenv("XH_TRAIN_KERNEL");
  return !(e && e[0] == 'f');
}
static const char *train_override() {
  const char *e = std::getenv("XH_TRAIN_KERNEL");
  return e && *e ? e : nullptr;
}
#if XH_VARIANT_KERNELS
static bool train_kernel_is(const char *name) {
  const char *e = train_override();
  return e && std::strcmp(e, name) == 0;
}
#endif

// the wave-specialised config-2 kernel (policy_spec4_kernels.hip, round 6) is
// opt-in: XH_TRAIN_KERNEL=spec4.  Parity-green, but 2-3% slower than
// policy_train_split4h_kernel on paired boxes (0.068 against 0.0663 ms per
// epoch: its matrix waves' phase B bounds the group)
static bool spec4_selected() {
  const char *ov = train_override();
  return ov && std::strcmp(ov, "spec4") == 0;
}
bool train_spec4_default(int B, int D, int H1, int H2, int kl) {
  return !kl && spec4_selected() && B == kSplit4hBins && D == 1 && H1 == 64 && H2 == 64;
}

bool policy_train_split_supported(const PolicyTrainArgs &a, int H1, int H2) {
  const bool algo = a.algo == kPPO || a.algo == kAC;
  // KL-PPO: the KL builds of the 64-bin 2-D, 128-bin 3-D and 32-bin 1-D
  // [64,64] kernels (two rows per group there, any row count)
  if (a.algo == kKLPPO)
    return (H1 == 128 && H2 == 128 &&
            ((a.env.B == 64 && a.env.D == 2) ||
             (a.env.B == kSplit128Bins && a.env.D == kSplit128Dims))) ||
           (H1 == 64 && H2 == 64 && a.env.B == kSplit4hBins && a.env.D == 1);
  if (algo && H1 == 64 && H2 == 64 && a.env.B == kSplit4hBins && a.env.D == 1)
    return (a.b.T * a.b.N) % 2 == 0;  // 64-row groups of two envs
  return algo && H1 == 128 && H2 == 128 &&
         ((a.env.B == 64 && a.env.D == 2) ||
          (a.env.B == kSplit128Bins && a.env.D == kSplit128Dims));
}

hipError_t launch_policy_train_split(const PolicyTrainArgs &a, int grid,
                                     hipStream_t s, KernelInfo *info) {
  KernelInfo dummy;
  if (!info) info = &dummy;
  info->math = kMathSplitTrainF16;
  const char *ov = train_override();
  if (a.env.B == kSplit4hBins) {
    // policy_train_split4h_kernel (and its KL-PPO build); the
    // wave-specialised form under XH_TRAIN_KERNEL=spec4 (A/B runs)
    if (spec4_selected() && a.algo != kKLPPO) {
      info->name = "policy_train_spec4_kernel";
      return launch_policy_train_spec4(a, grid, s);
    }
    info->name = a.algo == kKLPPO ? "policy_train_split4h_kl_kernel"
                                  : "policy_train_split4h_kernel";
    return launch_policy_train_split4h(a, grid, s);
  }
  if (a.env.B == kSplit128Bins) {
    if (!ov) {
      info->name = a.algo == kKLPPO ? "policy_train_split8x_kl_kernel"
                                    : "policy_train_split8x_kernel";
      return launch_policy_train_split8x(a, grid, s);
    }
#if XH_VARIANT_KERNELS
    if (train_kernel_is("split128")) {
      info->name = "policy_train_split128_kernel";
      return launch_policy_train_split128(a, grid, s);
    }
#endif
  } else {
    // the wave-specialised kernel (PPO / actor-critic) and its KL-PPO build;
    // the override XH_TRAIN_KERNEL=split8wh (A/B runs, the test of the two
    // against each other) runs policy_train_split8wh_kernel / its KL build
    if (!ov) {
      info->name = a.algo == kKLPPO ? "policy_train_spec8_kl_kernel"
                                    : "policy_train_spec8_kernel";
      return a.algo == kKLPPO ? launch_policy_train_spec8_kl(a, grid, s)
                              : launch_policy_train_spec8(a, grid, s);
    }
    if (!ov || std::strcmp(ov, "split8wh") == 0) {
      info->name = a.algo == kKLPPO ? "policy_train_split8wh_kl_kernel"
                                    : "policy_train_split8wh_kernel";
      return launch_policy_train_split8wh(a, grid, s);
    }
#if XH_VARIANT_KERNELS
    if (train_kernel_is("split8wg")) {
      info->name = "policy_train_split8wg_kernel";
      return launch_policy_train_split8wg(a, grid, s);
    }
    info->math = kMathSplitTrain;  // the all-bf16 forms
    if (train_kernel_is("split8w")) {
      info->name = "policy_train_split8w_kernel";
      return launch_policy_train_split8w(a, grid, s);
    }
    if (train_kernel_is("split8wp")) {
      info->name = "policy_train_split8wp_kernel";
      return launch_policy_train_split8wp(a, grid, s);
    }
    if (train_kernel_is("split4p")) {
      info->name = "policy_train_split4p_kernel";
      return launch_policy_train_split4p(a, grid, s);
    }
    if (train_kernel_is("split4w")) {
      info->name = "policy_train_split_kernel";
      return launch_policy_train_split4w(a, grid, s);
    }
#endif
  }
  info->name = nullptr;
  return hipErrorNotSupported;  // an override this library was built without
}

}  // namespace xh
