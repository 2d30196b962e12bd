/* liboac_amd -- MI355X (gfx950) native OAC/SAC gradient-step hot path.
 *
 * Plain C ABI: no C++ or torch types cross this boundary.  All device memory
 * is owned by the caller (PyTorch allocates it); the library never frees a
 * caller pointer.  Every call returns 0 on success or nonzero on failure, in
 * which case oac_last_error() describes it.  Work is stream-ordered on the
 * hipStream_t passed as `stream` (void*), with no host synchronisation.
 * One handle per device; a handle is used from one host thread at a time
 * (the reference trainer is single-threaded, launcher_util.py:90).
 *
 * Reference interfaces replaced (paths under /root/reference):
 *   oac_sac_step          SACTrainer.train / train_from_torch
 *                         (trainer/trainer.py:99-103, 126-280) incl. the
 *                         ReplayBuffer.random_batch gather (replay_buffer.py:106-115)
 *                         and np_to_pytorch_batch (utils/core.py:56-61)
 *   oac_sac_step_phase    the same step split at the data-parallel exchange points
 *   oac_sac_set_allreduce the data-parallel step with its exchanges (no reference
 *   oac_rccl_*            counterpart: main.py:575-578 runs replicas)
 *   oac_particle_*        ParticleTrainer.train_from_torch, share_layers=True
 *                         (trainer/particle_trainer_oac.py:169-363)
 *   OAC_KIND_GAUSS        GaussianTrainer.train_from_torch (g-oac), share_layers=True
 *                         (trainer/gaussian_trainer.py:177-437)
 *   OAC_KIND_PARTICLE_UB  ParticleTrainer.train_from_torch, share_layers=True
 *                         (trainer/particle_trainer.py:175-432; the p-oac recipes)
 *   oac_expl_action       get_optimistic_exploration_action (stochastic branch)
 *                         (optimistic_exploration.py:7-11, 14-109)
 *   oac_replay_sample_indices   np.random.randint(0, size, B) (replay_buffer.py:107)
 *   oac_replay_gather     the fancy-index gather of replay_buffer.py:108-114
 *   oac_adam_polyak       torch optim.Adam.step (trainer/trainer.py:75-91) +
 *                         soft_update_from_to (utils/pytorch_util.py:5-9)
 */
#ifndef OAC_AMD_H
#define OAC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OAC_ABI_VERSION 3

/* ---------------------------------------------------------------- config */
enum oac_kind {
  OAC_KIND_SAC = 0,          /* SACTrainer (OAC / SAC)                         */
  OAC_KIND_PARTICLE = 1,     /* particle_trainer_oac.ParticleTrainer (p-oac + OAC exploration) */
  OAC_KIND_GAUSS = 2,        /* gaussian_trainer.GaussianTrainer (g-oac)       */
  OAC_KIND_PARTICLE_UB = 3   /* particle_trainer.ParticleTrainer (p-oac recipes: deterministic
                                policy, upper-bound quantile loss, target_policy) */
};

typedef struct oac_sac_config {
  int kind;              /* OAC_KIND_SAC (twin critics, q_out=1); OAC_KIND_PARTICLE and
                            OAC_KIND_PARTICLE_UB (one critic, q_out = K particles);
                            OAC_KIND_GAUSS (one critic, q_out=2: mean | log std) */
  int obs_dim, act_dim;
  int hidden;            /* width of both hidden layers (reference: [M]*N, N=2) */
  int q_out;             /* 1 for SAC/OAC; K heads for the shared-layer particle critic */
  int batch;             /* per-rank batch size */
  float discount, reward_scale, tau;
  double policy_lr, qf_lr, beta1, beta2, adam_eps;
  int auto_alpha;        /* use_automatic_entropy_tuning */
  float target_entropy;
  int target_update_period;
  int row_stride;        /* floats per replay row (multiple of 4) */
  int off_obs, off_act, off_rew, off_term, off_next_obs; /* row layout; off_act == off_obs+obs_dim */
  uint64_t seed;         /* Philox key for the policy noise */
  int gemm_cfg;          /* -1 auto (2 at batch >= 1024, else 0), 0 small tiles + split-K,
                            1 LDS-tiled large tiles, 2 large-batch per-launch choice */
  int world_size;        /* data-parallel ranks (alpha / gradient averaging) */
  /* OAC_KIND_GAUSS (gaussian_trainer.py:65-72, main.py:219-233, 549-554) */
  float std_bound;       /* standard_bound = norm.ppf(delta) */
  float std_init;        /* (q_max - q_min) / sqrt(12): upper clamp of the std target */
  int std_soft_update;   /* GAUSS, PARTICLE_UB: std_soft_update with probability std_soft_prob */
  float std_soft_prob;   /* std_soft_update_prob */
  /* OAC_KIND_GAUSS / OAC_KIND_PARTICLE_UB */
  int mean_update;       /* next actions from target_policy instead of policy */
  /* OAC_KIND_PARTICLE_UB (particle_trainer.py:61-69, 255-264) */
  int delta_index;       /* sorted particle the policy maximises */
  float rescale_spread;  /* rescale_targets_around_mean: q_max - q_min; <= 0: off */
  /* PARTICLE, PARTICLE_UB, GAUSS: train_bias=False (networks.py:59-60: the critic's
   * last_fc.bias has requires_grad=False, so it is never updated) */
  int freeze_q_bias;
} oac_sac_config;

/* Flat parameter arena layout (float offsets; every tensor 16-byte aligned).
 * The policy block holds fc0.weight, fc0.bias, fc1.weight, fc1.bias and the
 * two heads stacked as one [2*act_dim, hidden] matrix (rows 0..Da-1 =
 * last_fc.weight, rows Da..2Da-1 = last_fc_log_std.weight) and their biases
 * likewise.  Each critic block holds fc0.weight, fc0.bias, fc1.weight,
 * fc1.bias, last_fc.weight, last_fc.bias.  Arenas: params/grads/adam_m/adam_v
 * = [policy | critic 1 | critic 2] (one critic for PARTICLE; [policy |
 * target_policy | critic] for GAUSS and PARTICLE_UB); targets = [target critic 1 | target
 * critic 2]. */
typedef struct oac_sac_layout {
  int64_t pol_fc0_w, pol_fc0_b, pol_fc1_w, pol_fc1_b, pol_head_w, pol_head_b, pol_size;
  int64_t q_fc0_w, q_fc0_b, q_fc1_w, q_fc1_b, q_last_w, q_last_b, q_size;
  int64_t q1_base, q2_base;   /* critic blocks in the params arena (q2_base < 0: none) */
  int64_t n_critics;
  int64_t params_total, targets_total;
  int64_t workspace_floats;
  int64_t tpol_base;     /* GAUSS, PARTICLE_UB: target_policy block (params = [policy |
                            target_policy | critic], one Adam group over both policies); else -1 */
} oac_sac_layout;

typedef struct oac_sac_buffers {
  float* params; float* grads; float* adam_m; float* adam_v; float* targets;
  void* alpha_state;     /* 16 floats: log_alpha, exp_avg, exp_avg_sq, alpha, alpha_loss, grad,
                            sum (data-parallel all-reduce slot), -, next_* (in-step scratch) */
  void* step_state;      /* 64-byte device step counters (zeroed by the caller) */
  float* workspace;      /* layout.workspace_floats */
  const float* replay;   /* [replay_rows, row_stride] fp32 */
  int64_t replay_rows;
  const int32_t* idx_ring; /* [ring_slots * batch] sampled indices */
  int ring_slots;
  /* ReplayBufferCount state for the ring path of counts=True trainers (may be
   * NULL): per-row sample counts and dedupe tags [replay_rows], and a device
   * epoch counter (one value per draw).  With OAC_STEP_GATHER | OAC_STEP_COUNTS
   * each step reads its batch counts and bumps the drawn rows on the device
   * (replay_buffer.py:186-197), so the counts recipes run from the ring. */
  int32_t* counts; int32_t* count_tags; int32_t* count_epoch;
  /* GAUSS / PARTICLE_UB with use_target_policy and no mean_update
   * (particle_trainer.py:150-154, 196-199; gaussian_trainer.py:154-158,
   * 196-199): a policy-shaped block (layout pol_* offsets) whose actions on
   * next_obs replace the policy's in the TD target; NULL = the policy */
  const float* next_policy;
} oac_sac_buffers;

typedef struct oac_sac oac_sac;

/* named workspace buffers (for parity checks and diagnostics) */
enum oac_ws_buffer {
  OAC_WS_BATCH = 0, OAC_WS_EPS1, OAC_WS_EPS2,
  OAC_WS_HEAD1, OAC_WS_HEAD2,          /* policy heads [B, 2Da] = mean | raw log_std */
  OAC_WS_ACT1, OAC_WS_ACT2, OAC_WS_LOGP1, OAC_WS_LOGP2,
  OAC_WS_Q1, OAC_WS_Q2, OAC_WS_QN1, OAC_WS_QN2, OAC_WS_TQ1, OAC_WS_TQ2,
  OAC_WS_Y, OAC_WS_SQE1, OAC_WS_SQE2, OAC_WS_QNEW,
  OAC_WS_COUNTS,                       /* [B] batch counts (ReplayBufferCount) for OAC_STEP_COUNTS */
  OAC_WS_HEAD3, OAC_WS_ACT3,           /* GAUSS, PARTICLE_UB: target_policy(obs) head and action */
  OAC_WS_LOGP_PART,                    /* [ceil(B/16)] sum of (logp1 + target_entropy) per 16-row
                                          block: the data-parallel alpha exchange (world_size > 1)
                                          all-reduces this vector, the targets kernel sums it */
  OAC_WS_H2Q1, OAC_WS_H2Q2,            /* SAC: the critics' second hidden layer on (obs, a) [B, H]
                                          after the ReLU -- the masks their backward used (parity
                                          checks; 0 rows for the other kinds) */
  OAC_WS_H1P, OAC_WS_H2P,              /* SAC / P-OAC: the policy's hidden layers on obs [B, H]
                                          after the ReLU -- the masks the policy backward used
                                          (parity checks; 0 rows for the other kinds) */
  OAC_WS_COUNT_PUBLIC
};

/* step flags */
#define OAC_STEP_GATHER       1  /* gather the batch from the replay via idx_ring */
#define OAC_STEP_DEVICE_EPS   2  /* draw eps1/eps2 with Philox (else caller wrote them) */
#define OAC_STEP_USE_GRAPH    4  /* replay the captured hipGraph of the step */
#define OAC_STEP_COUNTS       8  /* particle / gaussian trainer with counts=True: the batch
                                    counts the caller wrote into OAC_WS_COUNTS shape the
                                    quantile targets (particle_trainer_oac.py:220-224,
                                    particle_trainer.py:236-241) or the std target
                                    (gaussian_trainer.py:238-242) */

int oac_sac_query_layout(const oac_sac_config* cfg, oac_sac_layout* out);
int oac_sac_create(const oac_sac_config* cfg, const oac_sac_buffers* bufs, oac_sac** out);
int oac_sac_destroy(oac_sac* h);
int oac_sac_step(oac_sac* h, int flags, void* stream);

/* n_steps consecutive steps (each its own minibatch from the device index
 * ring, exactly as n calls of oac_sac_step); with OAC_STEP_USE_GRAPH they are
 * captured into one graph, so the per-launch host/graph cost is paid once per
 * n steps.  Used by rl_algorithm-style loops that run num_trains_per_train_loop
 * steps back to back (rl_algorithm.py: trainer.train per step). */
int oac_sac_step_n(oac_sac* h, int flags, int n_steps, void* stream);
/* Drop-in stepping with host-drawn indices -- rl_algorithm.py:160-167 calls
 * replay_buffer.random_batch(B) (np.random.randint on numpy's global stream,
 * replay_buffer.py:107) and then trainer.train(batch) once per step.
 * set_host_ring registers a pinned host staging ring [ring_slots][batch] int32
 * (ring_slots = the handle's idx_ring slots, a multiple of 16).  step_host_idx
 * copies the step's B int64 indices (host memory, each in [0, replay_rows))
 * into staging slot bc % ring_slots, enqueues the H2D copy into the idx_ring
 * slot the step's gather reads, and enqueues the step's launches (issued
 * directly: a one-step graph launch cost more than the launches it holds;
 * OAC_DROPIN_GRAPH=1 enqueues the captured one-step graph instead) --
 * all on `stream`, with no host synchronisation (a staging slot is rewritten
 * only after the copy that last read it has completed).  bc = the device
 * step_state batch counter at this step (the caller mirrors it).
 * pinned_ring = NULL: the handle allocates its own host-coherent ring
 * (oac_sac_host_ring returns it) and, at small batch (the batch-256 kernel
 * set), reads the step's indices straight from it inside the step's first
 * launch -- no H2D copy and no gather launch. */
int oac_sac_set_host_ring(oac_sac* h, int32_t* pinned_ring);
int32_t* oac_sac_host_ring(oac_sac* h);
int oac_sac_step_host_idx(oac_sac* h, const int64_t* idx, int64_t bc, int flags, void* stream);
/* the staging + H2D copy of step_host_idx alone (the data-parallel step then
 * runs its phases and all-reduces on the same stream) */
int oac_sac_stage_host_idx(oac_sac* h, const int64_t* idx, int64_t bc, void* stream);
/* the data-parallel drop-in step as one call (rl_algorithm.py:160-167 at
 * world_size > 1): the caller captures one step -- the phases below and its
 * collectives -- into a graph on its own collective library and hands the
 * instantiated graph (hipGraphExec_t) to the handle; oac_sac_step_host_idx
 * then stages the indices and launches that graph on `stream`, exactly as the
 * single-process step launches its own.  `flags` = the step flags the graph's
 * phases were captured with (OAC_STEP_GATHER implied, OAC_STEP_USE_GRAPH
 * ignored); while a graph is attached, oac_sac_step_host_idx must be called
 * with the same flags or it fails without launching.  NULL detaches it (the
 * caller still owns the graph and destroys it after the last step that
 * launched it). */
int oac_sac_set_step_graph(oac_sac* h, void* graph_exec, int flags);
/* data-parallel split (config.world_size > 1): phase 0 = forward through the
 * policy sample and the local sum(logp + target_entropy) as per-16-row
 * partials into the workspace buffer OAC_WS_LOGP_PART (ceil(B / 16) floats):
 * with auto-alpha on and world_size > 1 that vector is what the caller
 * all-reduces (SUM) before phase 1 (the targets kernel adds its entries);
 * 1 = alpha update from the caller's all-reduced partials through the critic
 * gradients (reduced into the grads arena); 2 = critic Adam + Polyak (after
 * the caller's critic-grad all-reduce, averaged) through the policy gradient
 * (grads arena); 3 = policy Adam + step advance (after the policy-grad
 * all-reduce).  oac_sac_step (world_size 1) runs the same sequence with the
 * split-K reduction fused into the Adam passes.  SAC kind only: phase 4 = the
 * part of phase 1 that needs no alpha (the critics on the fresh actions) and
 * phase 5 = the rest of phase 1, so 0, [alpha all-reduce || 4], 5, 2, 3 is
 * the same step with the first exchange overlapped. */
int oac_sac_step_phase(oac_sac* h, int phase, int flags, void* stream);

/* ------------------------------------------------ data-parallel exchanges */
/* The data-parallel step with its exchanges issued by the library itself
 * (SURVEY 8b "oac_allreduce_hook(...) (or an RCCL comm passed in)", 8e: the
 * alpha partials OAC_WS_LOGP_PART, the critic gradients [q1_base, q1_base +
 * n_critics * q_size) and the policy gradients [0, q1_base) of the grads arena
 * -- three in-place SUM all-reduces per step, at the points of the torch-1.4
 * order of trainer/trainer.py:139-210 where a whole-batch quantity is needed).
 * fn(ctx, buf, n, stream) must enqueue an in-place fp32 SUM of buf[0:n] over
 * the ranks on `stream` (stream-ordered) and return 0.  With a hook attached
 * and config.world_size > 1 (or OAC_DP_FORCE), every step entry
 * (oac_sac_step, _step_n, _step_host_idx) runs phase 0, [alpha], 1, [critic
 * grads], 2, [policy grads], 3 with the exchanges in between, as direct
 * launches on `stream` (no graph); at world size 1 without OAC_DP_FORCE a sum
 * over one rank is the identity and the single-process step runs.  fn = NULL
 * detaches the hook.  Replaces the caller-side exchange loop over
 * oac_sac_step_phase (and a captured graph of it, oac_sac_set_step_graph). */
typedef int (*oac_allreduce_fn)(void* ctx, float* buf, int64_t n, void* stream);
#define OAC_DP_FORCE    1   /* issue the exchanges at world size 1 too (measurement, tests) */
#define OAC_DP_OVERLAP  2   /* SAC: the alpha exchange on the handle's side stream beside
                               phase 4 (the critics on the fresh actions), joined before phase 5 */
int oac_sac_set_allreduce(oac_sac* h, oac_allreduce_fn fn, void* ctx, int flags);
/* RCCL implementation of the hook.  librccl is loaded at run time from
 * librccl_path (the librccl.so the process already uses, e.g. torch's);
 * unique_id: rank 0 fills 128 bytes that every rank passes to create
 * (collective: all ranks call create together).  oac_rccl_allreduce is an
 * oac_allreduce_fn with ctx = the oac_rccl handle. */
typedef struct oac_rccl oac_rccl;
int oac_rccl_unique_id(const char* librccl_path, void* id128);
int oac_rccl_create(const char* librccl_path, const void* id128, int rank, int world,
                    oac_rccl** out);
int oac_rccl_destroy(oac_rccl* c);
int oac_rccl_allreduce(void* rccl, float* buf, int64_t n, void* stream);

/* which branches of the launch plan the steps issued since the last reset
 * took (bitmask of OAC_TRACE_*; reset != 0 clears it after reading) */
#define OAC_TRACE_DIRECT        1    /* small batch: layer 0 reads rows through the index slot */
#define OAC_TRACE_DIRECT_BIG    2    /* large batch: the LDS-DMA layer 0 reads rows through the slot */
#define OAC_TRACE_BATCH_COPY    4    /* large batch: the batch copy in the fresh-action critic launch */
#define OAC_TRACE_QDOT          8    /* width-1 critic heads as layer-1 epilogue partials */
#define OAC_TRACE_WL_TARGETS    16   /* the critics' last-layer dW slabs in the targets kernel */
#define OAC_TRACE_SPLIT_PHASE1  32   /* phase 1 issued as 4 + 5 (the overlapped alpha exchange) */
#define OAC_TRACE_FUSED         64   /* the single-process fused-Adam step */
#define OAC_TRACE_EXCHANGE      128  /* data-parallel exchanges issued through the hook */
#define OAC_TRACE_LA_ADAM       256  /* large batch: policy layer-0 Adam by last arrival (no launch) */
#define OAC_TRACE_HEAD_DH2      512  /* the head's dX in the dL/da launch, head dW with policy layer 1 */
int oac_sac_trace(oac_sac* h, int reset);

int oac_sac_workspace_view(oac_sac* h, int which, int64_t* offset, int64_t* rows, int64_t* cols);
/* number of kernel launches of one step (for the launch/graph accounting) */
int oac_sac_launch_count(oac_sac* h);
/* the device launch-record cache (no reference counterpart; diagnostics):
   out[0] records uploaded, out[1] launch positions seen, out[2] hits, out[3]
   misses.  Positions are launch indices within one step, so both stay
   bounded however many steps run (<= 512 records, <= 64 positions). */
int oac_sac_cache_stats(oac_sac* h, int64_t* out);
/* bench instrumentation: with timing enabled, steps run as direct launches
 * bracketed by hipEvents; read_timing returns (and resets) the summed device
 * milliseconds and launch counts per kernel kind: 0 grouped GEMM, 1 row
 * kernels, 2 fused Adam, 3 gather. */
int oac_sac_set_timing(oac_sac* h, int enable);
int oac_sac_read_timing(oac_sac* h, double* ms_by_kind, int64_t* count_by_kind, int nkinds);
/* the same timing per launch, in issue order (before read_timing resets it):
 * returns the number of launches written (<= max_n), -1 on error */
int oac_sac_read_launch_times(oac_sac* h, double* ms, int* kinds, int max_n);

/* ---------------------------------------------------------------- replay */
/* numpy legacy seeding (init_genrand) of a 625-word MT19937 state, on the host */
int oac_mt_seed_host(uint32_t seed, uint32_t* state625);
/* device: out[0:count] = np.random.randint(0, size, count), advancing the
 * device MT19937 state (625 words) bit-exactly like numpy's legacy RandomState */
int oac_replay_sample_indices(uint32_t* mt_state_dev, uint64_t size, int count, int32_t* out,
                              void* stream);
/* device: out[r, :] = replay[idx[r], :] for r < B (row_stride % 4 == 0) */
int oac_replay_gather(const float* replay, int64_t row_stride, const int32_t* idx, int B,
                      float* out, void* stream);

/* device insert (ReplayBuffer.add_path / add_sample, replay_buffer.py:50-104):
 * n transitions in the reference's host dtypes -- obs / act / next_obs
 * float64 [n, dim], rew float64 [n], term uint8 [n] -- rounded to fp32 and
 * packed into the ring rows (top + i) % capacity of the row layout
 * [obs | act | rew | term | next_obs | pad] (offsets in floats) */
int oac_replay_insert(float* storage, int64_t row_stride, int64_t capacity, int64_t top, int n,
                      const double* obs, const double* act, const double* rew,
                      const double* next_obs, const uint8_t* term, int obs_dim, int act_dim,
                      int off_obs, int off_act, int off_rew, int off_term, int off_next_obs,
                      void* stream);
/* ReplayBufferCount.random_batch bookkeeping (replay_buffer.py:186-197):
 * counts_out[i] = counts[idx[i]] (float, before the update; may be NULL), then
 * counts[j] += 1 once per distinct j of idx (numpy fancy-index `+=`).  tags:
 * int32 [capacity] owned by the caller, epoch: a value this buffer never
 * passed before (dedupe tags are never cleared) */
int oac_replay_counts_update(int32_t* counts, int32_t* tags, const int32_t* idx, int B,
                             int32_t epoch, float* counts_out, void* stream);
/* priority sampling (replay_buffer.py:180-184, np.random.choice(p = 1/(c+1),
 * normalised)): idx_out[i] = the inverse-cdf index of the caller's uniform
 * u[i] (numpy random_sample draws) over counts[0:size]; scratch: device fp64
 * [oac_replay_priority_scratch_doubles(size)], size <= 4,194,304 */
int64_t oac_replay_priority_scratch_doubles(int64_t size);
int oac_replay_priority_sample(const int32_t* counts, int64_t size, const double* u, int B,
                               double* scratch, int32_t* idx_out, void* stream);

/* ------------------------------------------------------------------ Adam */
/* advance 0: Adam step t = n_steps+1, snapshot t (step_state), Polyak when
 * n_steps % period == 0; advance 1: t from the snapshot, then n_steps += 1. */
int oac_adam_polyak(float* p, const float* g, float* m, float* v, int64_t n, float* target,
                    float tau, int target_update_period, double lr, double beta1, double beta2,
                    double eps, void* step_state, int advance, void* stream);

/* -------------------------------------------------------- OAC exploration */
typedef struct oac_expl oac_expl;
/* policy / q1 / q2 point at their blocks in a params arena laid out as
 * oac_sac_layout describes; workspace: oac_expl_workspace_floats() floats. */
int64_t oac_expl_workspace_floats(int obs_dim, int act_dim, int hidden);
int oac_expl_create(int obs_dim, int act_dim, int hidden, const float* policy, const float* q1,
                    const float* q2, float* workspace, void* step_state, uint64_t seed,
                    oac_expl** out);
int oac_expl_destroy(oac_expl* h);
/* vectorised rollouts: one handle for n_obs observations; the
 * obs slot is then [n_obs, obs_dim + act_dim] (row stride obs_dim + act_dim,
 * the caller writes the first obs_dim floats of each row), eps [n_obs,
 * act_dim], outputs [n_obs, act_dim]; each row is computed exactly as a
 * single-observation call.  oac_expl_create = oac_expl_create_batch(1, ...) */
int64_t oac_expl_workspace_floats_batch(int n_obs, int obs_dim, int act_dim, int hidden);
int oac_expl_create_batch(int n_obs, int obs_dim, int act_dim, int hidden, const float* policy,
                          const float* q1, const float* q2, float* workspace, void* step_state,
                          uint64_t seed, oac_expl** out);
/* one critic with K heads (share_layers, K in [2, 16]): Q_UB = mean_k Q_k + beta_UB std_k Q_k
 * (unbiased std; optimistic_exploration.py:48-58, the except branch taken when qfs has
 * one shared-layer critic); q points at its block in a K-head critic layout */
int oac_expl_create_shared(int n_obs, int obs_dim, int act_dim, int hidden, int K,
                           const float* policy, const float* q, float* workspace,
                           void* step_state, uint64_t seed, oac_expl** out);
/* ob: device [obs_dim] fp32 (already in the workspace slot returned by
 * oac_expl_obs_slot, or any device pointer); eps: device [act_dim] or NULL
 * (Philox).  Writes action[act_dim]; optional mu_E / std / grad outputs. */
float* oac_expl_obs_slot(oac_expl* h);
int oac_expl_action(oac_expl* h, const float* eps, float beta_UB, float delta, float* action,
                    float* mu_E, float* std_out, float* grad_out, void* stream);
/* the handle's device result block [3][n_obs][act_dim]: action | mu_E | std
 * (valid after the call's work on `stream` completes) */
const float* oac_expl_outputs(oac_expl* h);
/* optional pinned host staging: host_obs [n_obs, obs_dim + act_dim] (the
 * first obs_dim floats of each row are the observation) is uploaded and the
 * result block downloaded into host_out [3][n_obs][act_dim] inside the call's
 * graph, so a call is one graph replay + one stream synchronisation (NULLs
 * switch it off) */
int oac_expl_set_host_io(oac_expl* h, const float* host_obs, float* host_out);
/* Latency path (the per-env-step call of optimistic_exploration.py:14-109 from
 * path_collector.py:176-257): the handle's own host-coherent buffers -- obs
 * [n_obs, obs_dim + act_dim] (write the first obs_dim floats of each row) and
 * results [3][n_obs][act_dim] (action | mu_E | std) -- are read and written by
 * the kernel itself; oac_expl_action_now launches on `stream` (behind the
 * work already queued there) and returns once the results are in *out. */
int oac_expl_host_staging(oac_expl* h, float** obs, float** out);
int oac_expl_action_now(oac_expl* h, const float* eps, float beta_UB, float delta, void* stream);
/* --trainer_UB with particle_trainer_oac.ParticleTrainer (optimistic_exploration.py:38-39
 * -> trainer.predict(upper_bound=True), particle_trainer_oac.py:147-167): with a K-head
 * handle, index in [0, K) makes Q_UB = sort_k(Q_k)[index] (the trainer's delta_index;
 * beta_UB unused); -1 restores the mean + beta_UB std bound */
int oac_expl_set_ub_index(oac_expl* h, int index);

/* ----------------------------------------------------- network evaluation */
/* Row-wise forward of the trainer's networks outside the gradient step, one
 * workgroup per (row, network).  offsets = {fc0.weight, fc0.bias, fc1.weight,
 * fc1.bias, last_fc.weight, last_fc.bias} inside each parameter block
 * (oac_sac_layout q_* or pol_* fields; the policy's last_fc is the stacked
 * [2*act_dim, hidden] head).
 * oac_critic_eval: FlattenMlp(obs, act) (networks.py:154-161) of n_nets (1 or 2)
 * critic blocks -> q [n, n_nets*q_out]; jac (optional) [n, n_nets*q_out,
 * obs_dim+act_dim] = d q / d [obs | act], for SACTrainer.predict /
 * ParticleTrainer.predict whose Q_UB the exploration differentiates
 * (trainer/trainer.py:105-123, particle_trainer_oac.py:147-167,
 * optimistic_exploration.py:39,64). */
int oac_critic_eval(const float* const* nets, int n_nets, const int64_t* offsets, int obs_dim,
                    int act_dim, int hidden, int q_out, const float* obs, int64_t ld_obs,
                    const float* act, int64_t ld_act, int n, float* q, float* jac, void* stream);
/* TanhGaussianPolicy.forward (trainer/policies.py:260-316) of n rows: eps
 * [n, act_dim] standard normals (stochastic) or NULL (deterministic: tanh(mean));
 * outputs [n, act_dim] action, mean, log_std (clamped), std, pre_tanh (z), and
 * log_prob [n] (summed over the action dims; may be NULL) */
int oac_policy_eval(const float* net, const int64_t* offsets, int obs_dim, int act_dim, int hidden,
                    const float* obs, int64_t ld_obs, int n, const float* eps, float* action,
                    float* mean, float* log_std, float* log_prob, float* std_out, float* pre_tanh,
                    void* stream);

/* ---------------------------------------------------------------- errors */
const char* oac_last_error(void);
int oac_abi_version(void);

/* Kernel / schedule choices that are not the default, for A/B measurements
   and the alternative-kernel parity tests (no reference counterpart).  The
   library reads no environment variable: a process sets a choice with
   oac_tuning_set (0 = the default) before it creates the plans that use it.
   Returns 1 for an unknown key. */
enum oac_tuning_key {
  OAC_TUNE_BWDP_CFG = 0,     /* large-batch backward tile config: 9-15, 17 (default: 12, 64x64 2-stage) */
  OAC_TUNE_FWD_TILE_M,       /* large-batch forward tile rows: 64 / 128 (default: per launch) */
  OAC_TUNE_FWD_TILE_N,       /* large-batch forward tile columns: 64 / 128 */
  OAC_TUNE_FWD_NB,           /* large-batch forward LDS ring depth: 2 / 3 */
  OAC_TUNE_SPLIT_ADAM,       /* 1: side-workgroup Adam (default), -1: one Adam launch per group */
  OAC_TUNE_DH2_TARGETS,      /* 1: P-OAC rank-K dX in the targets kernel (default), -1: own GEMM */
  OAC_TUNE_HEAD_CC,          /* policy-head column chunks per row block (default: by batch) */
  OAC_TUNE_SPLITS_Q1,        /* forced split-K counts of the dW products (0: sized by the plan) */
  OAC_TUNE_SPLITS_Q0,
  OAC_TUNE_SPLITS_PH,
  OAC_TUNE_SPLITS_P1,
  OAC_TUNE_SPLITS_P0,
  OAC_TUNE_DEBUG_CFG,        /* 1: print each GEMM launch's config and tasks to stderr */
  OAC_TUNE_RING_DIRECT,      /* -1: the device-ring small-batch path through a gather launch per
                                8 steps instead of each step's layer-0 launch reading its rows
                                through the device index ring (the drop-in path's form) */
  OAC_TUNE_RING_PREFETCH,    /* 1: on that gather-launch path, the next step's critic-side
                                forward inside the policy backward (instead of the deferred
                                layer-0 Adam) */
  OAC_TUNE_LA_ADAM,          /* 1: the large-batch SAC step's policy layer-0 Adam by the last
                                arrival of each dW tile (no Adam launch) */
  OAC_TUNE_HEAD_DH2,         /* -1: the small-batch SAC step's policy-head dX in the head-dW
                                launch instead of in the dL/da launch's epilogue (the default,
                                which merges the head dW into the policy layer-1 backward
                                launch); 2: the epilogue form at large batch too */
  OAC_TUNE_COUNT
};
int oac_tuning_set(int key, int value);

#ifdef __cplusplus
}
#endif
#endif /* OAC_AMD_H */
