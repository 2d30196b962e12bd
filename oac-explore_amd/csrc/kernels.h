// Kernel argument structs and launch helpers shared by the plan builders.
#pragma once
#include <cstring>
#include <vector>
#include "oac_common.h"

namespace oac {

// ----------------------------------------------------------- Philox4x32-10
__host__ __device__ __forceinline__ void philox4x32_10(unsigned (&c)[4], unsigned k0, unsigned k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c[0];
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c[2];
    const unsigned hi0 = (unsigned)(p0 >> 32), lo0 = (unsigned)p0;
    const unsigned hi1 = (unsigned)(p1 >> 32), lo1 = (unsigned)p1;
    const unsigned n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

// One standard normal for element `idx` of draw `stream` at step `counter`
// (Box-Muller on two 24-bit uniforms in (0,1)).
__device__ __forceinline__ float philox_normal(unsigned long long seed, unsigned long long counter,
                                               unsigned stream, unsigned idx) {
  unsigned c[4] = {idx >> 1, stream, (unsigned)counter, (unsigned)(counter >> 32)};
  philox4x32_10(c, (unsigned)seed, (unsigned)(seed >> 32));
  const float u1 = ((float)(c[0] >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float u2 = ((float)(c[1] >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float r = sqrtf(-2.f * logf(u1));
  const float th = 6.283185307179586f * u2;
  return (idx & 1) ? r * sinf(th) : r * cosf(th);
}

// ------------------------------------------------------------- row kernels
struct PolicySampleSeg {
  const float* head;   // [B, 2*Da] = mean | ls_raw
  const float* eps;    // [B, Da]
  float* act;          // [B, Da]
  float* stdv;         // [B, Da]
  float* u;            // [B, Da] z - mean
  float* logp;         // [B]
  float* act_row;      // optional strided copy of the action (critic input)
  long ld_act_row;
};

// fused policy head + sample + critics' action columns (head.hip)
struct HeadSeg {
  const float* h2;        // [B, H] policy hidden layer 2
  const float* wh; const float* bh;   // this segment's stacked heads [2*Da, H], [2*Da]
                                      // (null: HeadArgs.wh / bh)
  const float* eps;       // [B, Da] (unused with HeadArgs.det)
  float* head; float* act; float* stdv; float* u; float* logp;   // per-row outputs
  int n_nets;             // critics fed with this batch's actions (0..2)
  const float* wa[2];     // W0[:, Do:] of each critic (row n at wa + n*ld_wa)
  const float* pre[2];    // [B, H] saved obs projection (+ bias) of each critic
  float* h1[2];           // [B, H] relu(pre + a . wa^T)
};
struct HeadArgs {
  HeadSeg seg[3];
  const float* wh; const float* bh;   // stacked heads [2*Da, H], [2*Da]
  int det;                            // deterministic policies: a = tanh(mean) (policies.py:286-288);
                                      // stdv / u / logp / eps unused
  long ld_wa;
  int B, H, Da;
  int col_chunks;                     // workgroups per 32-row block
  long long* stage_clock;             // tools/micro builds only (-DOAC_STAGE_CLOCK)
  // non-null: segment 0's row blocks also write sum_rows (logp + te) of their
  // 16 rows (rows in order) to logp_part[row block] (data-parallel alpha)
  float* logp_part; float target_entropy;
};
hipError_t launch_policy_head(const HeadArgs& a, int nseg, hipStream_t s);

struct PolicySampleArgs {
  PolicySampleSeg seg[2];
  int B, act_dim;
};

enum { QV_Q1 = 0, QV_Q2, QV_QN1, QV_QN2, QV_TQ1, QV_TQ2, QV_COUNT };
struct CriticTargetArgs {
  // Q_i(obs, actions), Q_i(obs, a~), target Q_i(next_obs, a')  (QV_* order).
  // n_part > 0: q[k] is an output, assembled as part_bias[k] + sum_t
  // part[k][t*B + r] (per-tile partial dots of the last hidden layer)
  float* q[QV_COUNT];
  const float* part[QV_COUNT]; const float* part_bias[QV_COUNT]; int n_part;
  const float* logp2;
  const float* batch; long ld_batch; int off_rew, off_term;
  AlphaState* alpha;                    // null -> alpha = 0 (no entropy tuning)
  const StepState* state;
  const float* logp1;                   // for the alpha gradient
  float target_entropy;
  double lr, beta1, beta2, adam_eps;    // alpha optimiser (policy_lr)
  int world_size;                       // > 1: use alpha->sum (all-reduced), or with
  const float* logp_part; int n_logp_part;   // logp_part: the sum of these (all-reduced) partials
  float reward_scale, discount;
  int B;
  float* y; float* dq1; float* dq2; float* gq1; float* gq2; float* sqe1; float* sqe2;
  float* qnew;
  // large batch (wl_h2[0] set): the critics' last-layer dW in split-K slab
  // form, slab s = the sum over rows [256 s, 256 s + 256) -- the rows of
  // block s -- of dq_i[m] h2_i[m, :] (and of dq_i[m] for the bias), computed
  // here (grid.y = wl_H / 32 column groups) instead of as 64-row GEMM tiles
  const float* wl_h2[2]; float* wl_g[2]; float* wl_gb[2]; long wl_slab_stride; int wl_H;
};

struct PolicyHeadBwdArgs {
  const float* da1; const float* da2;
  const float* act; const float* stdv; const float* u; const float* eps;
  const float* head;    // [B, 2Da] (ls_raw for the clamp mask)
  const AlphaState* alpha;
  int B, act_dim;
  float* dhead;         // [B, 2Da]
};


struct ExplFusedArgs {                  // expl_split.hip: the exploration action
  const float* obs; long ld_obs;        // [N, ld_obs] observation rows
  const float* pol; const float* q[2];  // parameter blocks (oac_sac_layout offsets below)
  long p_fc0_w, p_fc0_b, p_fc1_w, p_fc1_b, p_head_w, p_head_b;
  long q_fc0_w, q_fc0_b, q_fc1_w, q_fc1_b, q_last_w, q_last_b;
  int Do, Da, H, n;
  int nq, K;                            // nq = 2, K = 1: twin critics (Q_UB = mean + beta |Q1-Q2|/2);
                                        // nq = 1, K > 1: one critic with K heads (share_layers:
                                        // Q_UB = mean_k + beta std_k, optimistic_exploration.py:48-58)
  const float* eps;                     // [N, Da] or null -> Philox (counter expl_counter)
  float* out;                           // [3][N][Da]: action | mu_E | std
  float* grad;                          // [N, Da] dQ_UB/dmu_T or null
  StepState* state; unsigned* ticket;   // ticket: zeroed device word (re-armed by the kernel)
  unsigned long long seed;
  float beta_UB, sqrt_2delta;
  int ub_index;                         // K heads: >= 0 -> Q_UB = sorted head ub_index
                                        // (trainer.predict, particle_trainer_oac.py:147-167)
  unsigned* done; unsigned done_seq;    // expl_split.hip: completion word (host-polled) or null;
                                        // bit 31 of the word set: a hand-off of the call timed out
  unsigned* fail;                       // zeroed device word: a group's timed-out hand-off (re-armed
                                        // by the kernel that reports it)
  // non-null with n == 1 (oac_expl_action_now): the outputs as [3][Da] tagged
  // 8-byte granules {value bits, done_seq | failed << 31} in host memory, in
  // place of the drained outputs + completion word (no wait for the stores)
  unsigned long long* tags;
};
// expl_split.hip: one observation per group of expl_split_group(rows) <=
// kExplGroup workgroups; a launch carries at most kExplRows observations
constexpr int kExplGroup = 32;
constexpr int kExplRows = 256;
int expl_split_group(int n_rows);
int expl_split_threads();
size_t expl_split_lds_bytes(int Do, int Da, int H);
long expl_split_scratch_floats(int H);
hipError_t launch_expl_split(const ExplFusedArgs& a, int row0, int n_rows, float* scratch,
                             hipStream_t s);
// the single-observation call with the observation inside the kernel
// arguments (the argument segment is written with the launch: no read of the
// host-coherent row from the kernel), Do <= kExplObsArg
constexpr int kExplObsArg = 512;
struct ExplObsArg { float v[kExplObsArg]; };
hipError_t launch_expl_split_obs(const ExplFusedArgs& a, const ExplObsArg& obs, float* scratch,
                                 hipStream_t s);

// row-wise network evaluation off the gradient step (mlp_eval.hip)
struct MlpEvalArgs {
  const float* x0; long ld_x0; int d0;   // input = [x0 | x1] per row
  const float* x1; long ld_x1; int d1;
  const float* net[2]; int n_nets;       // parameter blocks
  long w0, b0, w1, b1, wl, bl;           // layer offsets inside a block
  int H, Q, N;                           // hidden width, outputs, rows
  float* out; long ld_out;               // critic: [N, n_nets*Q]
  float* jac;                            // critic: [N, n_nets*Q, d0+d1] d out / d input, or null
  // policy outputs ([N, Q/2] each; log_prob [N] or null); eps null = deterministic
  const float* p_eps;
  float* p_action; float* p_mean; float* p_log_std; float* p_log_prob; float* p_std; float* p_pre_tanh;
};

// ------------------------------------------------------------ replay/adam
struct GatherArgs {
  const float* replay; long row_stride;   // [N, row_stride]
  const int* idx;                         // ring [ring_slots * B] or [B]
  int ring_slots;                         // 0: use idx[0:B] directly
  float* out;                             // [n_steps][B, row_stride]
  int B;
  int n_steps;                            // consecutive steps gathered (0 = 1): step j uses
                                          // ring slot / Philox counter batch_counter + j
  long out_stride, eps_stride;            // floats between the steps' batches / eps
  // eps generation (Philox) -- skipped when eps1 == null
  float* eps1; float* eps2; int n_eps;
  unsigned long long seed;
  const StepState* state;
};


// replay insert / ReplayBufferCount (replay_count.hip)
struct ReplayInsertArgs {
  float* storage; long row_stride, capacity, top;
  int n;                                   // transitions
  const double* obs; const double* act; const double* rew; const double* next_obs;
  const unsigned char* term;
  int obs_dim, act_dim, off_obs, off_act, off_rew, off_term, off_next_obs;
};
hipError_t launch_replay_insert(const ReplayInsertArgs& a, hipStream_t s);
struct CountsStepArgs {
  int* counts; int* tags; int* epoch;   // ReplayBufferCount device state
  const int* idx; int ring_slots; const StepState* state; int B;
  float* out;                           // [B] the step's batch counts
};
hipError_t launch_counts_step(const CountsStepArgs& a, hipStream_t s);
hipError_t launch_counts_update(int* counts, int* tags, const int* idx, int B, int epoch,
                                float* counts_out, hipStream_t s);
long prio_scratch_doubles(long size);
hipError_t launch_priority_sample(const int* counts, long size, const double* u, int B,
                                  double* scratch, int* idx_out, hipStream_t s);

// ParticleTrainer (share_layers) per-sample kernels, particle_trainer_oac.py
// A critic's K-output last layer evaluated inside a row kernel instead of a
// separate GEMM launch (det_plan.hip): out[r, k] = b[k] + sum_j h[r, j] W[k, j]
// for the kernel's 16-row block (h null: the outputs were stored by a GEMM)
struct RowHead {
  const float* h; const float* w; const float* b;   // h [B, H], W [K, H], b [K]
  float* out;                                        // [B, K] (workspace view, diagnostics)
  int H;
};

struct ParticleTargetArgs {
  const float* q; const float* tq;      // [B, K] critic / target critic outputs
  RowHead th;                           // th.h set: tq computed here (into th.out)
  RowHead qh;                           // qh.h set: q computed here (into qh.out)
  // dh2 set (needs qh.h): the critic backward into its last hidden layer,
  // dh2[r, n] = [h2[r, n] > 0] sum_k dq[r, k] W_last[k, n] (h2 = qh.h,
  // W_last = qh.w, n < qh.H): the rank-K dX launch it replaces
  float* dh2;
  const float* batch; long ld_batch; int off_rew, off_term;
  float reward_scale, discount;
  int B, K;
  float* dq;                            // [B, K] dL/dq (sort backward scatter)
  float* sqe;                           // [B, K] (sorted_q - y)^2 per sorted slot
  float* y;                             // [B, K] quantile targets (sorted slots)
  const float* counts;                  // [B] batch counts (counts=True) or null
  // particle_trainer.py (OAC_KIND_PARTICLE_UB) only; 1 / -1 / 0 keep the
  // particle_trainer_oac.py behaviour
  float loss_scale;                     // 1/K: qf_loss /= num_particles (:269)
  float soft_prob;                      // std_soft_update_prob (:222-231), < 0: off
  float rescale_spread;                 // rescale_targets_around_mean (:254-262), <= 0: off
};
struct ParticleMinArgs {
  const float* qn; int B, K;            // [B, K] Q(obs, a~) with the post-step critic
  RowHead hn;                           // hn.h set: qn computed here (into hn.out)
  float* gq;                            // [B, K] -1/B at the argmin head
  float* qmin;                          // [B]
  // dh2 set (needs hn.h): the -min Q backward into the last hidden layer,
  // dh2[r, n] = [h2[r, n] > 0] (-1/B) W_last[argmin_r, n] (the one nonzero
  // term of gq . W_last) with h2 = hn.h, W_last = hn.w, n < hn.H
  float* dh2;
  // alpha update (same as CriticTargetArgs)
  AlphaState* alpha; const StepState* state; const float* logp; float target_entropy;
  double lr, beta1, beta2, adam_eps; int world_size;
  const float* logp_part; int n_logp_part;   // world_size > 1: all-reduced partials (else alpha->sum)
};
hipError_t launch_particle_targets(const ParticleTargetArgs& a, hipStream_t s);
hipError_t launch_particle_min(const ParticleMinArgs& a, hipStream_t s);

// g-oac GaussianTrainer, share_layers=True (trainer/gaussian_trainer.py:177-437):
// the critic has two outputs, column 0 = Q mean, column 1 = log std (the
// FlattenMlp positive=[False, True] exp, networks.py:69-75, is applied here).

struct GaussTargetArgs {
  const float* q; const float* tq;      // [B, 2] Q(obs, a), Q_target(next_obs, a') raw outputs
  RowHead th;                           // th.h set: tq computed here (into th.out)
  RowHead qh;                           // qh.h set: q computed here (into qh.out)
  // dh2 set (needs qh.h): the critic backward into its last hidden layer,
  // dh2[r, n] = [h2[r, n] > 0] sum_k dq[r, k] W_last[k, n] (h2 = qh.h,
  // W_last = qh.w, n < qh.H): the rank-K dX launch it replaces
  float* dh2;
  const float* batch; long ld_batch; int off_rew, off_term;
  float reward_scale, discount, std_init;
  float soft_prob;                      // std_soft_update_prob, < 0: off
  const float* counts;                  // [B] batch counts (counts=True) or null
  int B;
  float* dq;                            // [B, 2] dL/d(raw outputs) of q_loss + std_loss
  float* y;                             // [B, 2] q_target | std_target
  float* sqe;                           // [B, 2] squared errors
};
hipError_t launch_gauss_targets(const GaussTargetArgs& a, hipStream_t s);

struct GaussSeedArgs {
  const float* qn;                      // [B, 2] post-step Q(obs, tanh(mean_pi(obs)))
  const float* qt;                      // [B, 2] post-step Q(obs, tanh(mean_target_pi(obs))) (unread)
  RowHead hn;                           // hn.h set: qn computed here
  float std_bound; int B;
  float* g; float* gt;                  // [B, 2] seeds of -mean(upper bound), -mean(q)
  float* ub;                            // [B] upper bound q + std_bound * std
};
hipError_t launch_gauss_seed(const GaussSeedArgs& a, hipStream_t s);

struct ParticleUbSeedArgs {            // particle_trainer.py:317-330, :339-348
  const float* qn;                      // [B, K] post-step Q(obs, tanh(mean_pi(obs)))
  const float* qt;                      // [B, K] post-step Q(obs, tanh(mean_target_pi(obs))) (unread)
  RowHead hn;                           // hn.h set: qn computed here
  int B, K, delta_index;
  float* g;                             // [B, K] -1/B at the delta_index-th sorted head
  float* gt;                            // [B, K] -1/(B K) on every head (mean over particles)
  float* ub;                            // [B] upper bound sorted_k[delta_index]
};
hipError_t launch_particle_ub_seed(const ParticleUbSeedArgs& a, hipStream_t s);

struct DetHeadBwdArgs {                 // d tanh(mean): dmean = da (1 - a^2), d log std = 0
  const float* da[2]; const float* act[2]; float* dhead[2];
  int nseg, B, act_dim;
};
hipError_t launch_det_head_backward(const DetHeadBwdArgs& a, hipStream_t s);

struct LogpSumArgs { const float* logp; int B; float target_entropy; AlphaState* alpha; };
hipError_t launch_logp_sum(const LogpSumArgs& a, hipStream_t s);

// Launch records in device memory.  A plan's launches pass the same GemmBatch
// step after step; read by value from the kernel arguments, every workgroup's
// first dependent load (its task record) goes to memory the host wrote for
// that launch, where a record the GPU read before is served by its caches
// (tools/micro/kernarg_micro: 304-byte record, chains of 11 launches of 256
// workgroups, 3.37 -> 2.93 us per launch).  The cache keeps each distinct
// batch a plan launches at a position of its step in a device slot, uploaded
// once (stream-ordered, before its first launch) and never rewritten, so a
// captured graph may keep the pointer; a batch the cache cannot hold (slots
// or variants per position exhausted) is passed by value as before.
struct BatchCache {
  static constexpr int kSlots = 512;       // 1.4 MB of device memory
  static constexpr int kPerPosition = 16;  // distinct batches per launch position
  static constexpr int kPositions = 64;    // launch positions per step (a step has <= 20)
  char* dev = nullptr;
  char* host = nullptr;   // pinned mirror: the uploads' sources, never rewritten
  int used = 0;
  bool failed = false;
  std::vector<std::vector<int>> at;   // launch position -> slots of the batches seen there
  long long hits = 0, misses = 0;
  // device copy of b (bytewise identical), or null (pass b by value)
  const GemmBatch* get(const GemmBatch& b, int pos, hipStream_t s);
  ~BatchCache();
};

inline const GemmBatch* BatchCache::get(const GemmBatch& b, int pos, hipStream_t s) {
  // a position past kPositions means the caller never reset its launch index
  // (it must be the launch's index within ONE step): no record, by value
  if (failed || pos < 0 || pos >= kPositions) return nullptr;
  constexpr size_t sz = sizeof(GemmBatch);
  if (!dev) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;   // (no allocation under capture)
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    if (hipMalloc(&dev, kSlots * sz) != hipSuccess) { dev = nullptr; failed = true; return nullptr; }
    if (hipHostMalloc(&host, kSlots * sz, 0) != hipSuccess) {
      (void)hipFree(dev); dev = nullptr; host = nullptr; failed = true; return nullptr;
    }
  }
  if ((int)at.size() <= pos) at.resize(pos + 1);
  for (int slot : at[pos])
    if (std::memcmp(host + slot * sz, &b, sz) == 0) {
      ++hits;
      return reinterpret_cast<const GemmBatch*>(dev + slot * sz);
    }
  ++misses;
  if (used >= kSlots || (int)at[pos].size() >= kPerPosition) return nullptr;
  // no upload into a stream capture (the copy would become a graph node of
  // its own): a captured launch of a batch not seen before takes it by value
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  const int slot = used;
  std::memcpy(host + slot * sz, &b, sz);
  if (hipMemcpyAsync(dev + slot * sz, host + slot * sz, sz, hipMemcpyHostToDevice, s) != hipSuccess) {
    failed = true;
    return nullptr;
  }
  ++used;
  at[pos].push_back(slot);
  return reinterpret_cast<const GemmBatch*>(dev + slot * sz);
}

inline BatchCache::~BatchCache() {
  if (dev) (void)hipFree(dev);
  if (host) (void)hipHostFree(host);
}


// launchers (defined in the .hip files)
void gemm_batch_finalize(GemmBatch& b, int cfg);
hipError_t gemm_batch_launch(const GemmBatch& b, int cfg, hipStream_t s, BatchCache* bc = nullptr,
                             int pos = -1);
int gemm_tile_m(int cfg);
int gemm_tile_n(int cfg);

hipError_t launch_policy_sample(const PolicySampleArgs& a, int nseg, hipStream_t s);
hipError_t launch_critic_targets(const CriticTargetArgs& a, hipStream_t s);
hipError_t launch_policy_head_backward(const PolicyHeadBwdArgs& a, hipStream_t s);
hipError_t launch_gather(const GatherArgs& a, hipStream_t s);
hipError_t launch_adam(const AdamArgs& a, hipStream_t s);
hipError_t launch_mt_randint(unsigned* mt_state, unsigned long long size, int count, int* out,
                             hipStream_t s);

}  // namespace oac
