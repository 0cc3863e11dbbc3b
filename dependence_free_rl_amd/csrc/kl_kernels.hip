// kl_kernels.hip -- the small device-side steps of kl_ppo_learner
// (policy_gradient.h:41-85, 310-335) around the KL train epoch:
//   end_*_kernel      which transitions ended an episode (their terminal end
//                     rows join the state matrix), and how many trajectories
//                     are still open (their end rows are the slot-T states);
//   kl_reduce_kernel  sum of the per-workgroup KL partials (fixed order);
//   kl_beta_kernel    d = mean KL over all rows; beta halves below
//                     d_targ / 1.5, doubles above 1.5 d_targ, clamped to
//                     [1e-25, 0.1]; the next epoch uses the new beta.
#include "xh_device.h"
#include "xh_kernels.h"

namespace xh {

// Entries t*N + e in env-major order (e ascending, then t), so the list --
// and every sum over it -- is the same from run to run.  Three parallel
// passes (envs on threads, coalesced done reads): per-block counts and local
// exclusive scans, one workgroup scanning the block totals, then each env
// writes its entries.
constexpr int kELB = 256;  // envs per block
__device__ __forceinline__ int env_done_count(const EndListArgs &a, int e) {
  int c = 0;
  if (e < a.N)
    for (int t = 0; t < a.T; ++t) c += a.done[(size_t)t * a.N + e] != 0;
  return c;
}
// block-local exclusive scan of v over kELB threads; *total = block sum
__device__ __forceinline__ int block_excl_scan(int v, int *total) {
  __shared__ int sc[kELB];
  const int tid = threadIdx.x;
  __syncthreads();  // a previous call's reads are done
  sc[tid] = v;
  __syncthreads();
  for (int off = 1; off < kELB; off <<= 1) {
    const int u = tid >= off ? sc[tid - off] : 0;
    __syncthreads();
    sc[tid] += u;
    __syncthreads();
  }
  *total = sc[kELB - 1];
  return sc[tid] - v;
}
__global__ __launch_bounds__(kELB) void end_count_kernel(EndListArgs a,
                                                         int *blk) {
  const int e = blockIdx.x * kELB + threadIdx.x;
  int total;
  (void)block_excl_scan(env_done_count(a, e), &total);
  const int open = e < a.N && a.done[(size_t)(a.T - 1) * a.N + e] == 0;
  int open_total;
  (void)block_excl_scan(open, &open_total);
  if (threadIdx.x == 0) {
    blk[2 * blockIdx.x] = total;
    blk[2 * blockIdx.x + 1] = open_total;
  }
}
// one workgroup: exclusive scan of the block totals (in place), n_end,
// n_open, rows_out
__global__ __launch_bounds__(1024) void end_base_kernel(EndListArgs a, int *blk,
                                                        int nblk) {
  __shared__ int sc[1024];
  __shared__ int carry, ocarry;
  if (threadIdx.x == 0) carry = ocarry = 0;
  __syncthreads();
  for (int b0 = 0; b0 < nblk; b0 += 1024) {
    const int b = b0 + threadIdx.x;
    const int v = b < nblk ? blk[2 * b] : 0;
    const int o = b < nblk ? blk[2 * b + 1] : 0;
    sc[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int u = threadIdx.x >= off ? sc[threadIdx.x - off] : 0;
      __syncthreads();
      sc[threadIdx.x] += u;
      __syncthreads();
    }
    if (b < nblk) blk[2 * b] = carry + sc[threadIdx.x] - v;
    const int chunk = sc[1023];
    __syncthreads();
    sc[threadIdx.x] = o;  // open counts: ordered tree sum
    __syncthreads();
    for (int off = 512; off > 0; off >>= 1) {
      if (threadIdx.x < off) sc[threadIdx.x] += sc[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      carry += chunk;
      ocarry += sc[0];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *a.n_end = carry;
    *a.n_open = ocarry;
    if (a.rows_out) *a.rows_out = a.rows_base + carry;
  }
}
__global__ __launch_bounds__(kELB) void end_write_kernel(EndListArgs a,
                                                         const int *blk) {
  const int e = blockIdx.x * kELB + threadIdx.x;
  const int c = env_done_count(a, e);
  int total;
  int pos = blk[2 * blockIdx.x] + block_excl_scan(c, &total);
  if (e < a.N)
    for (int t = 0; t < a.T; ++t)
      if (a.done[(size_t)t * a.N + e]) a.end_list[pos++] = t * a.N + e;
}

// The same list in one launch of one workgroup for N <= 1024 C, N % 4 == 0
// (used up to C = 8):
// thread i owns envs [i C, (i+1) C), reads their done bytes as 32-bit words
// (independent loads), keeps one count per env in registers; the exclusive
// scan of the thread totals is a wave scan (shuffles) plus the sixteen wave
// totals from LDS behind one barrier (integer sums: any order is exact); then
// each thread writes its envs' entries (t outer, so each env's entries stay
// in t order at their env-major positions).
template <int C>
__global__ __launch_bounds__(1024) void end_list_kernel(EndListArgs a) {
  static_assert(C % 4 == 0, "whole words");
  __shared__ int wsum[16], wopen[16];
  const int tid = threadIdx.x, e0 = tid * C, wv = tid >> 6, ln = tid & 63;
  int cnt[C];
#pragma unroll
  for (int i = 0; i < C; ++i) cnt[i] = 0;
  int open = 0;
  auto word = [&](int t, int w) -> unsigned {
    return e0 + 4 * w < a.N
               ? reinterpret_cast<const unsigned *>(a.done + (size_t)t * a.N + e0)[w]
               : 0u;
  };
  for (int t = 0; t < a.T; ++t)
#pragma unroll
    for (int w = 0; w < C / 4; ++w) {
      const unsigned v = word(t, w);
#pragma unroll
      for (int b = 0; b < 4; ++b) cnt[4 * w + b] += ((v >> (8 * b)) & 0xffu) != 0;
    }
#pragma unroll
  for (int w = 0; w < C / 4; ++w) {
    const unsigned v = word(a.T - 1, w);
#pragma unroll
    for (int b = 0; b < 4; ++b)
      open += e0 + 4 * w + b < a.N && ((v >> (8 * b)) & 0xffu) == 0;
  }
  int total = 0;
#pragma unroll
  for (int i = 0; i < C; ++i) total += cnt[i];
  int incl = total;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int u = __shfl_up(incl, d, 64);
    if (ln >= d) incl += u;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) open += __shfl_xor(open, d, 64);
  if (ln == 63) wsum[wv] = incl;
  if (ln == 0) wopen[wv] = open;
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) base += i < wv ? wsum[i] : 0;
  int pos[C];
  {
    int p = base + incl - total;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      pos[i] = p;
      p += cnt[i];
    }
  }
  for (int t = 0; t < a.T; ++t)
#pragma unroll
    for (int w = 0; w < C / 4; ++w) {
      const unsigned v = word(t, w);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((v >> (8 * b)) & 0xffu) a.end_list[pos[4 * w + b]++] = t * a.N + e0 + 4 * w + b;
    }
  if (tid == 0) {
    int ne = 0, no = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      ne += wsum[i];
      no += wopen[i];
    }
    *a.n_end = ne;
    *a.n_open = no;
    if (a.rows_out) *a.rows_out = a.rows_base + ne;
  }
}

int end_list_scratch_ints(int N) { return 2 * ((N + kELB - 1) / kELB); }

hipError_t launch_end_list(const EndListArgs &a, int *scratch,
                               hipStream_t s) {
  // one workgroup up to 8192 envs (config 2: 6 us against 14 us + two
  // launch gaps); the parallel three passes beyond (measured at 32768 envs:
  // 36 us in one workgroup, 14 us in three passes)
  if (a.N % 4 == 0 && a.N <= 1024 * 8) {
    if (a.N <= 1024 * 4)
      hipLaunchKernelGGL(end_list_kernel<4>, dim3(1), dim3(1024), 0, s, a);
    else
      hipLaunchKernelGGL(end_list_kernel<8>, dim3(1), dim3(1024), 0, s, a);
    return hipGetLastError();
  }
  const int nblk = (a.N + kELB - 1) / kELB;
  hipLaunchKernelGGL(end_count_kernel, dim3(nblk), dim3(kELB), 0, s, a, scratch);
  hipLaunchKernelGGL(end_base_kernel, dim3(1), dim3(1024), 0, s, a, scratch,
                     nblk);
  hipLaunchKernelGGL(end_write_kernel, dim3(nblk), dim3(kELB), 0, s, a, scratch);
  return hipGetLastError();
}

__global__ void scatter_list_kernel(const int *list, const int *n,
                                    const float *src, float *dst) {
  const int cnt = *n;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt;
       j += gridDim.x * blockDim.x)
    dst[list[j]] = src[j];
}

hipError_t launch_scatter_list(const int *list, const int *n, const float *src,
                               float *dst, int max_n, hipStream_t s) {
  int blocks = (max_n + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
  hipLaunchKernelGGL(scatter_list_kernel, dim3(blocks), dim3(256), 0, s, list,
                     n, src, dst);
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
