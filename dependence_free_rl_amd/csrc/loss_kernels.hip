// loss_kernels.hip -- the discrete-action loss gradients of a batch, the
// `loss_grad` the reference's learners hand to optimizer::step
// (nn.h:594-605):
//   policy_loss       (policy_gradient.h:24-34)  softmax_gradient_log per row
//   surrogate_loss    (policy_gradient.h:36-46)  clipped_gradient per row
//   kl_regulated_loss (policy_gradient.h:55-85)  softmax_gradient_log
//                                                + beta (p - q) (the gradient
//                                                part; the beta adaptation is
//                                                the caller's, on the host)
//   and discrete_action::gradient_log (rl.h:33-42) for completeness.
// One thread per (row, column), the reference's expressions in its operation
// order (fp contraction off): per element the same roundings as its host loop.
#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {

__global__ void action_loss_kernel(int kind, int rows, int range,
                                   const int32_t *__restrict__ choice,
                                   const float *__restrict__ distrib,
                                   const float *__restrict__ adv,
                                   const float *__restrict__ probs, float param,
                                   float *__restrict__ out) {
#pragma clang fp contract(off)
  const long n = (long)rows * range;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / range), c = (int)(i - (long)r * range);
    const int ch = choice[r];
    const float a = adv[r];
    const float *p = probs + (size_t)r * range;
    float v = 0.0f;
    if (kind == kLossSoftmaxGradientLog || kind == kLossKlRegulated) {
      // output = input * advantage; output[choice] -= advantage (rl.h:44-52)
      v = p[c] * a;
      if (c == ch) v = v - a;
      if (kind == kLossKlRegulated) {
        // regulation = (orig - truth) * beta, result += regulation (:69-73)
        const float reg = (p[c] - distrib[(size_t)r * range + c]) * param;
        v = v + reg;
      }
    } else if (c == ch) {
      const float q = distrib[(size_t)r * range + ch];
      if (kind == kLossClipped) {  // rl.h:54-74, epsilon = param (0.2)
        const float ratio = p[ch] / q;
        float clipped = ratio;
        if (ratio > 1.0f + param)
          clipped = 1.0f + param;
        else if (ratio < 1.0f - param)
          clipped = 1.0f - param;
        // std::min(clipped * advantage, ratio * advantage) * -1
        const float x = clipped * a, y = ratio * a;
        const float imp = (y < x ? y : x) * -1.0f;
        v = imp / p[ch];
      } else {  // gradient_log, rl.h:33-42
        const float log_grad = 1.0f / p[ch];
        const float weighted = log_grad * a * -1.0f;
        v = p[ch] / q * weighted;
      }
    }
    out[i] = v;
  }
}

hipError_t launch_action_loss(int kind, int rows, int range,
                              const int32_t *choice, const float *distrib,
                              const float *adv, const float *probs, float param,
                              float *out, hipStream_t s) {
  const long n = (long)rows * range;
  long b = (n + 255) / 256;
  b = b < 1 ? 1 : (b > 4096 ? 4096 : b);
  hipLaunchKernelGGL(action_loss_kernel, dim3((unsigned)b), dim3(256), 0, s,
                     kind, rows, range, choice, distrib, adv, probs, param, out);
  return hipGetLastError();
}

}  // namespace xh
