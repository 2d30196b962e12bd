// The plan object behind an oac_sac handle (SAC twin-critic and particle
// K-head trainers share it; each kind has its own workspace layout and
// launch sequence).
#pragma once
#include "../../include/oac_amd.h"
#include <cstring>
#include "plan_common.h"

namespace oac {

constexpr int kMaxWs = 128;
// batch / eps slots: one gather launch fills the minibatches of up to
// kXSlots consecutive steps (slot i % kXSlots is step i's batch)
constexpr int kXSlots = 8;
// split-K weight-gradient slabs shaped like the critic / policy arena ranges
constexpr int WS_TICKETS = kMaxWs - 3;   // last-arrival Adam tickets (GemmBatch::la_ticket), zeroed
constexpr int WS_GSLAB_Q = kMaxWs - 2;
constexpr int WS_GSLAB_P = kMaxWs - 1;

struct SacPlan : PlanBase {
  oac_sac_config c;
  oac_sac_layout L;
  oac_sac_buffers b;
  WsBuf ws[kMaxWs];
  Split sp_q0, sp_q1, sp_ql, sp_p0, sp_p1, sp_ph;
  int S_q = 1, S_p = 1;   // slab counts per group (max over the group's dW tasks)
  int slot = 0;           // batch / eps slot of the step being issued
  bool ring_direct = false;
  bool la_now = false;        // run_step: the policy layer-0 Adam by last arrival (no Adam launch)   // device-ring step: layer 0 reads its rows through the index ring
  // the step being issued gathers directly at large batch (phase0 sets it;
  // phase1's fresh-action critic launch then carries the batch copy)
  bool direct_big = false;
  const int* direct_ring = nullptr;   // its index ring (device or host-coherent)
  // data-parallel exchanges issued by the library (oac_sac_set_allreduce):
  // the hook, its flags, and the side stream + fork / join events of the
  // overlapped alpha exchange (created on first use, owned by the plan)
  oac_allreduce_fn ar_fn = nullptr;
  void* ar_ctx = nullptr;
  int ar_flags = 0;
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int trace = 0;   // OAC_TRACE_* bits of the branches issued since the last read
  // the drop-in step's staged indices (B <= kInlineRows), passed to the
  // direct layer-0 launch in its kernel arguments; valid after a staging call
  int inline_rows[kInlineRows];
  bool inline_ok = false;

  float* W(int id) const { return b.workspace + ws[id].off; }
  float* X() const { return W(OAC_WS_BATCH) + (long)slot * c.batch * c.row_stride; }
  float* E1() const { return W(OAC_WS_EPS1) + (long)slot * c.batch * c.act_dim; }
  float* E2() const { return W(OAC_WS_EPS2) + (long)slot * c.batch * c.act_dim; }
  float* P(int64_t off) const { return b.params + off; }
  float* T(int64_t off) const { return b.targets + off; }
  StepState* state() const { return reinterpret_cast<StepState*>(b.step_state); }
  AlphaState* alpha() const { return reinterpret_cast<AlphaState*>(b.alpha_state); }
};


// gradient destinations: the grads arena (no split) or the group's slabs
inline float* grad_q(SacPlan& p) {
  return p.S_q > 1 ? p.W(WS_GSLAB_Q) : p.b.grads + p.L.q1_base;
}
inline float* grad_p(SacPlan& p) { return p.S_p > 1 ? p.W(WS_GSLAB_P) : p.b.grads; }
inline long q_group(const SacPlan& p) { return (long)(p.L.n_critics * p.L.q_size); }
// the policy Adam group: everything in front of the critic block (the policy,
// plus the target_policy for GAUSS)
inline long p_group(const SacPlan& p) { return (long)p.L.q1_base; }

// critic update: reduce slabs, Adam (t = n_steps + 1), Polyak, snapshot t
inline AdamArgs critic_adam(SacPlan& p, int reduce_only, AlphaState* commit) {
  const oac_sac_config& c = p.c;
  AdamArgs a;
  std::memset(&a, 0, sizeof(a));
  a.p = p.b.params + p.L.q1_base; a.g = p.b.grads + p.L.q1_base;
  a.m = p.b.adam_m + p.L.q1_base; a.v = p.b.adam_v + p.L.q1_base; a.n = q_group(p);
  a.gslab = reduce_only < 0 ? a.g : grad_q(p);
  a.S = reduce_only < 0 ? 1 : p.S_q;
  a.slab_stride = q_group(p);
  // one critic: its layer 1 (and the last layer when split no wider) reads only
  // its own slabs (configs[4]: 16 of the group's 32)
  if (a.S > 1 && p.L.n_critics == 1 && p.sp_q1.S < a.S) {
    a.S2 = p.sp_q1.S; a.s2_lo = p.L.q_fc1_w;
    a.s2_hi = p.sp_ql.S <= p.sp_q1.S ? p.L.q_size : p.L.q_last_w;
  }
  a.target = p.b.targets; a.tau = c.tau; a.period = c.target_update_period;
  a.lr = c.qf_lr; a.beta1 = c.beta1; a.beta2 = c.beta2; a.eps = c.adam_eps;
  a.state = p.state(); a.advance = 0; a.alpha = commit;
  a.gscale = reduce_only < 0 ? 1.f / (float)c.world_size : 1.f;
  a.reduce_only = reduce_only > 0;
  return a;
}

// policy update: reduce slabs, Adam (t = snapshot + 1), advance the step
// reduce_only: 1 = reduce slabs into the grads arena only; -1 = the update from
// the (all-reduced) grads arena with gscale = 1/world; 0 = both in one pass.
inline AdamArgs policy_adam(SacPlan& p, int reduce_only, AlphaState* commit) {
  const oac_sac_config& c = p.c;
  AdamArgs a;
  std::memset(&a, 0, sizeof(a));
  a.p = p.b.params; a.g = p.b.grads; a.m = p.b.adam_m; a.v = p.b.adam_v; a.n = p_group(p);
  a.gslab = reduce_only < 0 ? a.g : grad_p(p);
  a.S = reduce_only < 0 ? 1 : p.S_p;
  a.slab_stride = p_group(p);
  if (a.S > 1 && p.sp_p1.S < a.S) {   // policy layer 1 (and the heads when split no wider)
    a.S2 = p.sp_p1.S; a.s2_lo = p.L.pol_fc1_w;
    a.s2_hi = p.sp_ph.S <= p.sp_p1.S ? p.L.pol_size : p.L.pol_head_w;
  }
  a.lr = c.policy_lr; a.beta1 = c.beta1; a.beta2 = c.beta2; a.eps = c.adam_eps;
  a.state = p.state(); a.advance = 1; a.alpha = commit;
  a.gscale = reduce_only < 0 ? 1.f / (float)c.world_size : 1.f;
  a.reduce_only = reduce_only > 0;
  return a;
}

// Fold a group's Adam into the launch that produces its last gradients (the
// layer-0 weight gradients): possible on the single-process path with the
// small-batch kernel and no split-K (a data-parallel step all-reduces first).
inline bool can_fuse_adam(const SacPlan& p) {
  return p.cfg == 0 && p.S_q == 1 && p.S_p == 1 && p.c.world_size == 1;
}

// attach `a` to batch `gb`: EPI_GRAD tiles update their own elements, tail
// blocks the given flat ranges (offsets from the group base a.p)
inline void fuse_adam(GemmBatch& gb, const AdamArgs& a, int nseg, const long* off, const long* n) {
  gb.fuse_adam = 1;
  gb.adam = a;
  gb.nseg = nseg;
  for (int i = 0; i < nseg; ++i) { gb.seg_off[i] = off[i]; gb.seg_n[i] = n[i]; }
}

// internal step flag (not in oac_amd.h): this step's indices are in the host
// ring slot (PlanBase::idx_host), read there by the gather / counts launch
constexpr int kStepHostIdx = 1 << 12;
inline const int* gather_idx(const SacPlan& p, int flags) {
  return ((flags & kStepHostIdx) && p.host_ring) ? p.host_ring : p.b.idx_ring;
}

// Large-batch single-process step (split-K slabs, no fused epilogue Adam):
// each group's Adam runs as side workgroups of a later GEMM launch that reads
// none of the updated parameters (GemmBatch::side_adam) instead of its own
// launch -- the critic's layer 1 + last layer beside its layer-0 dW, the
// critic's layer 0 beside the -min Q dX to layer 1, the policy's layer 1 +
// heads beside its layer-0 dW; only the policy's layer 0 keeps a launch.
// OAC_TUNE_SPLIT_ADAM = -1: one Adam launch per group (A/B runs).
inline bool split_adam_on(const SacPlan& p) {
  const bool v = tuning(OAC_TUNE_SPLIT_ADAM) >= 0;
  return v && p.cfg != 0 && p.c.world_size == 1 && !can_fuse_adam(p);
}
// With the split Adam: the policy layer 0's own Adam by the last arrival of
// each of its dW tiles (GemmBatch::la_adam) instead of the step's last launch.
// OAC_TUNE_LA_ADAM = 1 (A/B runs).
inline bool la_adam_on(const SacPlan& p) {
  return tuning(OAC_TUNE_LA_ADAM) > 0 && p.cfg == kCfgLargeBatch && p.c.world_size == 1;
}
// Attach the ranges [off[i], off[i] + n[i]) of `a` to batch gb as side
// workgroups when gb runs on gemm_bwdp; otherwise launch them now, one Adam
// launch per range (before gb: every caller's ranges are already final).
int side_adam(SacPlan& p, GemmBatch& gb, const AdamArgs& a, int nseg, const long* off,
              const long* n, bool book, hipStream_t s);

// a large-batch SAC step can gather directly (sac_plan phase0): every layer-0
// product on the LDS-DMA forward kernel, reading its rows from the replay
// through the index slot; eps and the batch copy from side workgroups of
// later forward launches.  (The same for the P-OAC step measured neutral at
// configs[4]: 18 -> 17 launches, 185.3 -> 184.3 us of launches, 203.9 us per
// step either way -- its short-K layer 0 took the index round trips, +3.2 us;
// not kept.)
inline bool big_direct_ok(const SacPlan& p) {
  // gemm_fwd's rank-Da continuation reads [obs | act] as one span of the row
  return (p.c.kind == OAC_KIND_SAC || p.c.kind == OAC_KIND_PARTICLE) && p.cfg == kCfgLargeBatch &&
         p.c.hidden >= 64 &&
         p.c.row_stride % 4 == 0 && p.c.row_stride / 4 <= 256 &&
         p.c.off_act == p.c.off_obs + p.c.obs_dim;
}

// particle trainer (particle_plan.hip)
void particle_layout_workspace(SacPlan& p);
int particle_run_step(SacPlan& p, int flags, hipStream_t s);
int particle_step_phase(SacPlan& p, int phase, int flags, hipStream_t s);
void particle_plan_splits(SacPlan& p);

// deterministic-policy trainers with a target_policy: g-oac GaussianTrainer and
// the p-oac ParticleTrainer of particle_trainer.py (det_plan.hip)
inline bool has_target_policy(int kind) {
  return kind == OAC_KIND_GAUSS || kind == OAC_KIND_PARTICLE_UB;
}
void det_layout_workspace(SacPlan& p);
int det_run_step(SacPlan& p, int flags, hipStream_t s);
int det_step_phase(SacPlan& p, int phase, int flags, hipStream_t s);

}  // namespace oac
