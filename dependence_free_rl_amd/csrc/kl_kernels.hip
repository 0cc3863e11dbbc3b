// kl_kernels.hip -- the small device-side steps of kl_ppo_learner
// (policy_gradient.h:41-85, 310-335) around the KL train epoch:
//   end_list_kernel   which transitions ended an episode (their terminal end
//                     rows join the state matrix), and how many trajectories
//                     are still open (their end rows are the slot-T states);
//   kl_reduce_kernel  sum of the per-workgroup KL partials (fixed order);
//   kl_beta_kernel    d = mean KL over all rows; beta halves below
//                     d_targ / 1.5, doubles above 1.5 d_targ, clamped to
//                     [1e-25, 0.1]; the next epoch uses the new beta.
#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {

// One 1024-thread workgroup.  Entries t*N + e in env-major order (e
// ascending, then t), so the list -- and every sum over it -- is the same
// from run to run.
__global__ __launch_bounds__(1024) void end_list_kernel(EndListArgs a) {
  __shared__ int scan[1024];
  __shared__ int open_part[1024];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int chunk = (a.N + nt - 1) / nt;
  const int e0 = tid * chunk, e1 = min(a.N, e0 + chunk);
  int cnt = 0, open = 0;
  for (int e = e0; e < e1; ++e) {
    for (int t = 0; t < a.T; ++t) cnt += a.done[(size_t)t * a.N + e] != 0;
    open += a.done[(size_t)(a.T - 1) * a.N + e] == 0;
  }
  scan[tid] = cnt;
  open_part[tid] = open;
  __syncthreads();
  // Hillis-Steele inclusive scan
  for (int off = 1; off < nt; off <<= 1) {
    const int v = tid >= off ? scan[tid - off] : 0;
    __syncthreads();
    scan[tid] += v;
    __syncthreads();
  }
  int pos = scan[tid] - cnt;
  for (int e = e0; e < e1; ++e)
    for (int t = 0; t < a.T; ++t)
      if (a.done[(size_t)t * a.N + e]) a.end_list[pos++] = t * a.N + e;
  if (tid == nt - 1) *a.n_end = scan[tid];
  // open count: ordered tree sum
  for (int off = nt / 2; off > 0; off >>= 1) {
    if (tid < off) open_part[tid] += open_part[tid + off];
    __syncthreads();
  }
  if (tid == 0) *a.n_open = open_part[0];
}

hipError_t launch_end_list(const EndListArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(end_list_kernel, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

// kl_sum[0] = sum of the partials, kl_sum[1] = rows of the state matrix
// (T*N transitions + n_end terminal end rows + n_open open end rows).
__global__ __launch_bounds__(256) void kl_reduce_kernel(
    const double *kl_part, int nparts, const int *n_end, const int *n_open,
    double rows_main, double *kl_sum) {
  __shared__ double part[256];
  double v = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) v += kl_part[i];
  part[threadIdx.x] = v;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) part[threadIdx.x] += part[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    kl_sum[0] = part[0];
    kl_sum[1] = rows_main + (double)*n_end + (double)*n_open;
  }
}

hipError_t launch_kl_reduce(const double *kl_part, int nparts, const int *n_end,
                            const int *n_open, double rows_main,
                            double *kl_sum, hipStream_t s) {
  hipLaunchKernelGGL(kl_reduce_kernel, dim3(1), dim3(256), 0, s, kl_part,
                     nparts, n_end, n_open, rows_main, kl_sum);
  return hipGetLastError();
}

__global__ void kl_beta_kernel(const double *kl_sum, float *beta, float d_targ,
                               float *log) {
  const float d = (float)(kl_sum[0] / kl_sum[1]);
  const float b0 = *beta;
  float b = b0;
  if (fabsf(d) < d_targ / 1.5f)
    b /= 2;
  else if (fabsf(d) > d_targ * 1.5f)
    b *= 2;
  b = fmaxf(b, 1e-25f);
  b = fminf(b, 0.1f);
  *beta = b;
  if (log) {
    log[0] = b0;
    log[1] = d;
    log[2] = b;
  }
}

hipError_t launch_kl_beta_update(const double *kl_sum, float *beta,
                                 float d_targ, float *log, hipStream_t s) {
  hipLaunchKernelGGL(kl_beta_kernel, dim3(1), dim3(1), 0, s, kl_sum, beta,
                     d_targ, log);
  return hipGetLastError();
}

}  // namespace xh
