// xh_kernels.h -- kernel argument blocks and launch entry points shared by the
// host runtime (xylo_hip.cpp) and the HIP kernel files.  No torch types.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xh {

enum Algo { kPPO = 0, kAC = 1, kKLPPO = 2 };
enum Heuristic { kHeurRandom = 0, kHeurFirstfit = 1, kHeurBestfit = 2,
                 kHeurMinwaste = 3 };

// Flat parameter offsets of the per-bin policy, in the reference layout
// model::parameters() (nn.h:499-508): conv1d_1(F0->H1), relu,
// conv1d_1(H1->H2), relu, conv1d_1(H2->1), head.  Each dense layer stores
// [A(out x in) row-major, b(out)].
struct PolicyLayout {
  int F0, H1, H2;
  __host__ __device__ int oW1() const { return 0; }
  __host__ __device__ int ob1() const { return H1 * F0; }
  __host__ __device__ int oW2() const { return ob1() + H1; }
  __host__ __device__ int ob2() const { return oW2() + H2 * H1; }
  __host__ __device__ int ow3() const { return ob2() + H2; }
  __host__ __device__ int ob3() const { return ow3() + H2; }
  __host__ __device__ int size() const { return ob3() + 1; }
};

// Value net: full(Fin->V1), relu, full(V1->V2), relu, full(V2->1)
// (ppo_training.cc:19-26).
struct ValueLayout {
  int Fin, V1, V2;
  __host__ __device__ int oW1() const { return 0; }
  __host__ __device__ int ob1() const { return V1 * Fin; }
  __host__ __device__ int oW2() const { return ob1() + V1; }
  __host__ __device__ int ob2() const { return oW2() + V2 * V1; }
  __host__ __device__ int ow3() const { return ob2() + V2; }
  __host__ __device__ int ob3() const { return ow3() + V2; }
  __host__ __device__ int size() const { return ob3() + 1; }
};

// Environment description (bin_packing.h:46-85, generalised to D dims).
struct EnvDesc {
  int B, D;
  int item_a[3], item_b[3];
  double p_a;
};

// Per-iteration trajectory storage (device).  Slot t of `bins`/`items` is the
// state S_t before step t; slot T is the state after the last step (the next
// iteration's S_0).  Terminal states E_t are recomputed from S_t + action.
struct Batch {
  int N, T;
  int8_t *bins;     // [T+1][N][B*D]
  int8_t *items;    // [T+1][N][4]
  int32_t *action;  // [T][N]
  float *pold;      // [T][N]   distrib[choice] at sampling time (rl.h:29)
  uint8_t *done;    // [T][N]
  uint32_t *rng;    // [N]      per-env minstd_rand0 state (reference order)
};

struct RolloutArgs {
  EnvDesc env;
  Batch b;
  int t;              // step index within the iteration
  uint32_t jump_mul;  // a^(4T(Nglobal-1)) mod m, applied after step T-1
  const float *params;
  const int32_t *forced;  // optional [T][N] actions (teacher forcing)
  float *logits_out;      // optional [N][B] (debug / parity)
  float *probs_out;       // optional [N][B]
  float *qold_out;        // KL-PPO: [T][N][B] the sampled distribution
  int wide;  // slot t holds a bin below -capacity (the f16-pair rollouts
             // bound |bins / capacity| by 1) or an item outside the item
             // table (they fold the item into per-entry biases): the f32
             // kernels run that slot
  int src_slot;  // > 0 (with t == 0): slot 0 := slot src_slot first
                 // (replay_buffer::forget keeping the open trajectories), done
                 // by the register-stepping kernels as they fetch, else by
                 // copies before the launch; 0 / -1: slot 0 as it is
  int nsteps;  // slots t .. t + nsteps - 1 (0 = 1); logits_out / probs_out
               // receive the last one's.  launch_rollout_step runs them in
               // one launch where the kernel steps in registers
               // (rollout_split_kernel), else one launch per slot
};

struct PolicyTrainArgs {
  EnvDesc env;
  Batch b;
  int algo;
  float clip_eps;
  const float *params;
  const float *adv;  // [T][N]
  float *slab;       // [gridDim.x][slab_stride]
  int slab_stride;
  int wide;          // a slot of the batch holds a bin below -capacity: the
                     // f32-MFMA kernels run (RolloutArgs::wide)
  int ablate;        // diagnostic build only (XH_ABLATE, make diag): bit0 skip
                     // dW2, bit1 skip dH1/dW1, bit2 skip layer-2 fwd, bit3
                     // skip softmax/loss; folded away in the product build
  // KL-PPO (kl_regulated_loss): every row of the learner's state matrix,
  // i.e. the T*N transitions, the open trajectories' end rows (slot T) and
  // the terminal end rows E_t listed in end_list.
  const float *qold;     // [T][N][B] old distributions
  const float *beta;     // device scalar (adapted between epochs)
  const int *end_list;   // [n_end] t*N + env of terminal transitions
  const int *n_end;      // device scalar
  double *kl_part;       // [gridDim.x] sum over rows of KL(q || p)
  // diagnostic build only (XH_PHASE_TRACE): per-wave cycle stamps at the
  // 8-wave train kernel's phase boundaries, [4 blocks][32 groups][8 waves][8]
  long long *trace;
};
constexpr int kTraceBlocks = 4, kTraceGroups = 32, kTraceSlots = 8;

// End-row bookkeeping: the ended transitions (KL-PPO end rows, the value
// step's terminal views).
struct EndListArgs {
  const uint8_t *done;   // [T][N]
  int N, T;
  int *end_list;         // [T*N] env-major, t ascending
  int *n_end;            // scalar
  int *n_open;           // scalar: envs whose last step is not terminal
  int *rows_out;         // optional: *rows_out = rows_base + n_end
  int rows_base;
};
// end_list / n_end / n_open (scratch: end_list_scratch_ints(N) ints).
int end_list_scratch_ints(int N);
// dst[list[j]] = src[j] for j < *n (terminal-view values to transition rows)
hipError_t launch_scatter_list(const int *list, const int *n, const float *src,
                               float *dst, int max_n, hipStream_t s);

// TD targets and GAE around the value net (the net itself runs on the Dense
// GEMMs, MlpArgs).
struct ValueArgs {
  EnvDesc env;
  Batch b;
  float *v_state;        // [T+1][N]   V(S_t)
  float *v_term;         // [T][N]     V(E_t) (terminal view of step t)
  float *row_g;          // [T*N] dL/dV = V - target (targets kernel), or null
};

// Deterministic (argmax) evaluation, policy_gradient_deterministic_policy
// (policy_gradient.h:356-373) as used by deep_agent.cc and the drivers'
// every-100-iterations evaluation: `episodes` whole episodes per env, env e
// on its own minstd stream starting at jump(x0, e * stream_stride).
struct EvalArgs {
  EnvDesc env;
  const float *params;
  int n_envs;
  int episodes;
  int argmax_probs;  // 1: argmax over softmax output, 0: over raw logits
  uint32_t x0;
  uint64_t stream_stride;
  long max_steps;     // safety bound per env
  const int *init_items;  // [n_envs][D] device, or nullptr: construct
  double *total;      // [n_envs] summed rewards
  long *steps;        // [n_envs] env steps taken
  int *final_items;   // [n_envs][D]
  uint32_t *rng_out;  // [n_envs]
  int *trace;         // env 0's actions [trace_cap] or nullptr
  long trace_cap;
};

// Heuristic agents (heuristic_kernels.hip): same stream / output convention
// as EvalArgs.
struct HeuristicArgs {
  EnvDesc env;
  int n_envs;
  int episodes;
  uint32_t x0;
  uint64_t stream_stride;
  long max_steps;
  const int *init_items;
  double *total;
  long *steps;
  int *final_items;
  uint32_t *rng_out;
  int *trace;
  long trace_cap;
};
// Full MLP (full_layer / relu chain, nn.h:60-110, 350-377) over a batch of
// rows whose input is the observation of (slot, env) states
// (dense_kernels.hip).  Layer l maps w[l] -> w[l+1]; relu after every layer
// but the last.  act[l] / grad[l]: [max_rows][w[l+1]] outputs and
// dL/d(pre-activation) of layer l.
struct MlpArgs {
  EnvDesc env;
  const int8_t *bins, *items;  // Batch state layout
  const int *list;             // row -> slot * N + env (nullptr: env = row)
  int N, slot;                 // slot used when list == nullptr
  const int32_t *action;       // non-null: rows >= term_from are the terminal
  int term_from;               //   views E_t of transition row - term_from
  const int *term_list;        //   (or of transition term_list[row - term_from])
  const int *rows;             // device row count (nullptr: max_rows)
  int max_rows;
  // optional [w[1]][B*D + D] scratch: layer 0 on the reduced observation
  // (bins, then the item once -- its B copies' weights pre-summed)
  float *w0red;
  int nlayers;
  int w[4];
  const float *params;  // flat model::parameters() layout
  float *act[3];
  float *grad[3];
  // optional with term_list: the output of row term_from + j also goes to
  // v_term[term_list[j]] for j < *term_n (the terminal views' values onto
  // their transition rows)
  float *v_term;
  const int *term_n;
  // the bf16 value-net kernels (value_net_kernels.hip): scratch for W0's
  // three-part fragments (vnet_frag_bytes), and the rows whose activations
  // the forward stores for the backward (0: all, -1: none)
  void *w0frag;
  int act_rows;
  // 1: w0frag already holds the fragments of these parameters (the trainer
  // knows they did not change since the last forward prepared them): the
  // forward skips its preparation launch
  int w0frag_ready;
};
hipError_t mlp_forward(const MlpArgs &a, hipStream_t s);
// Weight gradients of every layer into slab[split] (flat layout), data
// gradients down to layer 1 (layer 0 gets no backward, nn.h:516-526).
hipError_t mlp_backward(const MlpArgs &a, float *slab, int stride, int splits,
                        hipStream_t s);
// update_value_model's backward (policy_gradient.h:196-218) over the
// a.max_rows transition rows: TD targets and dL/dV = V - target
// (value_targets_kernel, into targets and a.grad[last]), then mlp_backward.
// The Fin -> 64 -> 32 -> 1 value net runs fused (two launches, the same
// bits) unless XH_VALUE_KERNEL=gemm.
hipError_t value_backward(const MlpArgs &a, const ValueArgs &va, float gamma,
                          float *targets, float *slab, int stride, int splits,
                          hipStream_t s);
// The kernels mlp_forward / value_backward run for a value net:
//   "vnet_bf16"  value_net_kernels.hip (Fin -> 64 -> 32 -> 1, B*D % 16 == 0,
//                B*D + D < 416, w0frag set): the default
//   "mlp3_fused" the f32 fused kernels (the same shape; XH_VALUE_KERNEL=mlp3)
//   "gemm"       layer by layer (any shape; XH_VALUE_KERNEL=gemm)
const char *value_kernel_name(const MlpArgs &a);
// true: the value kernels write layer 0's gradient on the reduced
// observation (bin 0's item columns only: slab_reduce needs SlabAlias)
bool value_reduced_slab(const MlpArgs &a);
bool vnet_shape_ok(const MlpArgs &a);
size_t vnet_frag_bytes(const EnvDesc &e);
hipError_t vnet_forward(const MlpArgs &a, hipStream_t s);
hipError_t vnet_backward(const MlpArgs &a, const ValueArgs &va, float gamma,
                         float *targets, float *slab, int stride, int splits,
                         hipStream_t s);

// model::eval of a described layer chain (dense_kernels.hip, xh_model_eval).
enum LayerKind { kLayerFull = 0, kLayerConv1d = 1, kLayerRelu = 2,
                 kLayerSoftmax = 3, kLayerSoftmaxXent = 4 };
struct ModelLayer {
  int kind, in, out;
};
hipError_t model_forward(const ModelLayer *layers, int nl, const float *params,
                         const float *x, int rows, int cols, float *a, float *b,
                         const float **out, int *out_cols, hipStream_t s);
// One layer of the reference's layer interface (nn.h:20-33) on device
// buffers: forward (y: rows x output width), backward (out: rows x cols, the
// data gradient), gradient (grad: the layer's flat parameter gradient, via
// layer_gradient_splits(...) slabs of `stride` floats; activations: none).
hipError_t layer_forward(const ModelLayer &L, const float *W, const float *x,
                         int rows, int cols, float *y, hipStream_t s);
hipError_t layer_backward(const ModelLayer &L, const float *W, const float *x,
                          int rows, int cols, const float *bp, float *out,
                          hipStream_t s);
int layer_gradient_splits(const ModelLayer &L, int rows, int cols);
hipError_t layer_gradient(const ModelLayer &L, const float *x, int rows,
                          int cols, const float *bp, float *slab, int stride,
                          float *grad, hipStream_t s);
// The discrete-action loss gradients of a batch (rl.h:33-74 row by row;
// policy_gradient.h:24-85): out [rows][range].
enum LossKind { kLossGradientLog = 0, kLossSoftmaxGradientLog = 1,
                kLossClipped = 2, kLossKlRegulated = 3 };
hipError_t launch_action_loss(int kind, int rows, int range,
                              const int32_t *choice, const float *distrib,
                              const float *adv, const float *probs, float param,
                              float *out, hipStream_t s);

// REINFORCE (pg_kernels.hip).  Batch.T = the per-iteration step bound.
struct PgStepArgs {
  EnvDesc env;
  Batch b;
  int t, episodes;
  const float *logits;    // [N][B] of slot t
  const int32_t *forced;  // [T][N] or nullptr
  int *ep_done, *len, *active;
};
struct PgLearnArgs {
  int N, B, episodes;
  float gamma;
  const int *len;
  int *row_off, *list, *nrows;
  const uint8_t *done;
  const int32_t *action;
  float *rtg;       // [rows]
  double *ep_part;  // [N]
  double *stats;    // [2]: sum of slot-0 returns, trajectories
  const float *logits;
  float *dlogits;
  float *adv_grid;  // [T][N] advantages for introspection
};
hipError_t launch_pg_env_init(const EnvDesc &env, Batch b, uint32_t x0,
                              int env_offset, uint64_t stride, hipStream_t s);
hipError_t launch_pg_seed(Batch b, uint32_t x, int env_offset, uint64_t stride,
                          hipStream_t s);
hipError_t launch_pg_begin(int N, int *active, int *ep_done, int *len,
                           hipStream_t s);
hipError_t launch_pg_step(const PgStepArgs &a, hipStream_t s);
hipError_t launch_pg_rows(const PgLearnArgs &a, hipStream_t s);
hipError_t launch_pg_adv(const PgLearnArgs &a, hipStream_t s);
hipError_t launch_pg_loss(const PgLearnArgs &a, int max_rows, hipStream_t s);

// Vectorised environment for callers with their own policy (xh_venv_*,
// venv_kernels.hip): bins int8 [N][B*D], items int8 [N][4], rng u32 [N].
enum VenvOp { kVenvStep = 0, kVenvReset = 1, kVenvObserve = 2 };
struct VenvArgs {
  EnvDesc env;
  int N;
  int8_t *bins, *items;
  uint32_t *rng;
  const int32_t *action;  // [N] chosen bins
  const uint8_t *mask;    // [N] or nullptr (all envs)
  float *reward;          // [N] (step)
  uint8_t *done;          // [N] game_over after the apply
  float *obs;             // [N][B][2D] or nullptr
  int *err;               // device flag: an action was out of range
  int mode;               // 0 environment::apply, 1 agent::step minus react
  uint32_t skip_mul;      // a^policy_draws (step)
  uint32_t jump_mul;      // a^(k (Nglobal - 1)) after a step (reference order)
};
bool venv_shape_supported(int B, int D);
hipError_t launch_venv(const VenvArgs &a, int op, hipStream_t s);
hipError_t launch_venv_init(const VenvArgs &a, uint32_t x0, int env_offset,
                            int n_global, int k, hipStream_t s);

// 1 when the kernels were built with the phase-ablation switches
// (make diag, -DXH_DIAG_ABLATE=1), 0 in the product library.
int diag_build();

bool heuristic_shape_supported(int B, int D);
hipError_t launch_heuristic(const HeuristicArgs &a, int kind, hipStream_t s);

// Launchers (return hipError_t of the launch). `variant` selects the
// <B,D,H1,H2> instantiation; returns hipErrorInvalidValue when unsupported.
bool policy_shape_supported(int B, int D, int H1, int H2);
hipError_t launch_env_init(const EnvDesc &env, Batch b, uint32_t x0,
                           int env_offset, int n_global, hipStream_t s);
hipError_t launch_env_seed(Batch b, uint32_t x, int env_offset,
                           hipStream_t s);
hipError_t launch_end_list(const EndListArgs &a, int *scratch, hipStream_t s);
// beta <- adapt(beta, mean KL) (policy_gradient.h:68-80); kl_sum[0] = the
// (all-reduced) KL sum, rows[0] the (all-reduced) row count.
hipError_t launch_kl_reduce(const double *kl_part, int nparts, const int *n_end,
                            const int *n_open, double rows_main,
                            double *kl_sum, hipStream_t s);
hipError_t launch_kl_beta_update(const double *kl_sum, float *beta,
                                 float d_targ, float *log, hipStream_t s);
// What a launch entry point ran, recorded by the trainer for
// xh_trainer_kernel_info: the kernel's name and its arithmetic.
enum Math {
  kMathF32Mfma = 0,       // f32-input MFMA (v_mfma_f32_32x32x2_f32) / f32 VALU
  kMathSplitTrain = 1,    // bf16 MFMA on 3-part splits: layer 2 six products per
                          // f32 product, dW2 / dH1 three (rank-1 backward)
  kMathSplitRollout = 2,  // layer 2 on f16 pairs: three f16 products per f32
                          // product (the other layers f32 MFMA)
  kMathSplitTrainF16 = 3  // layer 2 three f16 MFMAs per f32 product (scaled f16
                          // pairs), dH1 two, dW2 three bf16 (8 per 3 products)
};
struct KernelInfo {
  const char *name = nullptr;
  int math = kMathF32Mfma;
};
hipError_t launch_rollout_step(const RolloutArgs &a, int H1, int H2, int grid,
                               hipStream_t s, KernelInfo *info = nullptr);
hipError_t launch_policy_train(const PolicyTrainArgs &a, int H1, int H2,
                               int grid, hipStream_t s,
                               KernelInfo *info = nullptr);
// The f32-accurate split train kernels for the 64-bin 2-D and 128-bin 3-D
// [128,128] shapes and the 32-bin 1-D [64,64] one (dispatch in
// train_select.cpp); XH_TRAIN_KERNEL=f32 selects the f32-MFMA ones.  The
// launchers of the superseded forms (split128 / 8w / 8wp / 4p / 8wg) are
// linked only into the variant library (`make variants`).
constexpr int kSplit128Bins = 128, kSplit128Dims = 3;
constexpr int kSplit4hBins = 32;
bool train_split_enabled();
bool policy_train_split_supported(const PolicyTrainArgs &a, int H1, int H2);
hipError_t launch_policy_train_split(const PolicyTrainArgs &a, int grid,
                                     hipStream_t s, KernelInfo *info);
hipError_t launch_policy_train_split128(const PolicyTrainArgs &a, int grid,
                                        hipStream_t s);
hipError_t launch_policy_train_split8w(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s);
hipError_t launch_policy_train_split8wp(const PolicyTrainArgs &a, int grid,
                                        hipStream_t s);
hipError_t launch_policy_train_split4p(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s);
hipError_t launch_policy_train_split8wh(const PolicyTrainArgs &a, int grid,
                                        hipStream_t s);
// its KL-PPO build (policy_split8wh_kl_kernels.o; called by
// launch_policy_train_split8wh)
hipError_t launch_policy_train_split8wh_kl(const PolicyTrainArgs &a, int grid,
                                           hipStream_t s);
// the wave-specialised config-3 / config-4 epoch (policy_spec8_kernels.hip)
hipError_t launch_policy_train_spec8(const PolicyTrainArgs &a, int grid, hipStream_t s);
// its KL-PPO build (policy_spec8_kl_kernels.o)
hipError_t launch_policy_train_spec8_kl(const PolicyTrainArgs &a, int grid, hipStream_t s);
// the wave-specialised config-2 epoch (policy_spec4_kernels.hip, opt-in by
// XH_TRAIN_KERNEL=spec4; one 8-wave workgroup per CU: train_spec4_default
// says when the grid is one per CU)
hipError_t launch_policy_train_spec4(const PolicyTrainArgs &a, int grid, hipStream_t s);
bool train_spec4_default(int B, int D, int H1, int H2, int kl);
hipError_t launch_policy_train_split8wg(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s);
hipError_t launch_policy_train_split4h(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s);
// its KL-PPO build (policy_split4h_kl_kernels.o; called by
// launch_policy_train_split4h)
hipError_t launch_policy_train_split4h_kl(const PolicyTrainArgs &a, int grid,
                                          hipStream_t s);
hipError_t launch_policy_train_split8x(const PolicyTrainArgs &a, int grid,
                                       hipStream_t s);
// its KL-PPO build (policy_split8x_kl_kernels.o; called by
// launch_policy_train_split8x)
hipError_t launch_policy_train_split8x_kl(const PolicyTrainArgs &a, int grid,
                                          hipStream_t s);
int policy_train_grid(int B, int D, int H1, int H2, int kl);
hipError_t launch_eval_argmax(const EvalArgs &a, int H1, int H2,
                              hipStream_t s);
int rollout_grid(int B, int D, int H1, int H2);

bool value_shape_supported(int V1, int V2);
hipError_t launch_value_targets(const ValueArgs &a, float gamma, float *targets,
                                hipStream_t s);
// GAE; part != nullptr also writes per-block (sum, sum of squares) of the
// advantages for the opt-in normalisation ([gae_grid(N)][2] doubles).
int gae_grid(int N);
hipError_t launch_gae(const ValueArgs &a, float gamma, float lambda, float *adv,
                      double *part, hipStream_t s);
hipError_t launch_adv_stats(const double *part, int nparts, double *stats,
                            hipStream_t s);
hipError_t launch_adv_normalize(float *adv, long n, const double *stats,
                                double count, hipStream_t s);
// Slab entries the value net's reduced layer 0 leaves unwritten: the item
// columns of bins b > 0 of its first [rows][in] block, whose sums equal bin
// 0's (EpSlabRed).  B = 0: none.
struct SlabAlias {
  int rows, in, B, D;
};
hipError_t launch_slab_reduce(const float *slab, int nslab, int stride, int n,
                              float *out, hipStream_t s,
                              SlabAlias al = SlabAlias{0, 0, 0, 0});
hipError_t launch_sgd(float *params, const float *grad, int n, float lr,
                      float wd, hipStream_t s);
// momentum_optimizer (kind 1) / adam_optimizer (kind 2), nn.h:630-698: state
// m (velocity / first moment) and v (second moment); c1, c2 = adam's bias
// corrections 1 - beta^t computed on the host as the reference does.
struct OptStep {
  int kind;  // XH_OPT_SGD / XH_OPT_MOMENTUM / XH_OPT_ADAM
  float lr, beta1, beta2, c1, c2;
  float wd;  // sgd weight decay
};
hipError_t launch_opt(float *params, const float *grad, float *m, float *v,
                      int n, OptStep o, hipStream_t s);
// Single-rank fusion of launch_slab_reduce and the optimizer step: the same
// fixed-order slab sum (written to out) and the same per-element update.
hipError_t launch_slab_reduce_opt(const float *slab, int nslab, int stride,
                                  int n, float *out, float *params, float *m,
                                  float *v, OptStep o, hipStream_t s,
                                  SlabAlias al = SlabAlias{0, 0, 0, 0});


// xylo/tensor.{h,cc} arithmetic on device arrays (tensor_kernels.hip; the
// drop-in tensor type's device tensors and large host operations).
enum TensorMapOp {
  kTensorAdd = 0, kTensorMinus = 1, kTensorMultiply = 2, kTensorDivide = 3,
  kTensorAddS = 4, kTensorMinusS = 5, kTensorMultiplyS = 6, kTensorDivideS = 7,
  kTensorAbs = 8, kTensorSin = 9, kTensorExp = 10, kTensorLog = 11,
  kTensorSqrt = 12, kTensorFill = 13, kTensorRMinusS = 14, kTensorRDivideS = 15
};
enum TensorReduceOp {
  kTensorSum = 0, kTensorDot = 1, kTensorSqDev = 2, kTensorMax = 3,
  kTensorArgmax = 4
};
// out[i] = op(a[i], b[i], s) for i < n (b: the binary ops; s: the scalar ops
// and fill)
hipError_t launch_tensor_map(int op, const float *a, const float *b, float s,
                             float *out, long n, hipStream_t st);
// workgroup partials of a reduction over n elements; scratch holds
// tensor_reduce_parts(n) + 1 records of 16 bytes, the result (double value,
// int64 index) in the last
int tensor_reduce_parts(long n);
hipError_t launch_tensor_reduce(int op, const float *a, const float *b, float s,
                                long n, void *scratch, hipStream_t st);
hipError_t launch_tensor_transpose(const float *in, float *out, int rows,
                                   int cols, hipStream_t st);
// C[m][n] = sum_k A[m][k] B(n, k): b_nk = B is [N][K] (matmul_transposed,
// tensor.cc:218-227), else B is [K][N] (matmul, :228-230); the Dense f32-MFMA
// GEMM (dense_kernels.hip)
hipError_t launch_tensor_gemm(bool b_nk, const float *A, const float *B,
                              float *C, int M, int N, int K, hipStream_t st);

}  // namespace xh
