// P-OAC particle trainer step on MI355X (BASELINE configs[4]):
// ParticleTrainer.train_from_torch with share_layers=True
// (/root/reference/trainer/particle_trainer_oac.py:169-363) -- one critic with
// K outputs (quantile "particles"), per-sample sort over K, quantile TD
// targets without entropy, sum of K MSEs, then (after the critic Adam) the
// policy forward, alpha update and the policy loss on the min head of the
// POST-step critic, Polyak.  Reference order:
//   Q(obs,a) [185-191] -> sort [192] -> pi(next_obs; eps1) [193-195]
//   -> TQ(next_obs,a') sorted [198-202] -> y = scale*r + (1-d)*gamma*TQ_sorted [207]
//   -> Adam(Q, grad sum_i MSE(sorted_i, y_i)) [247-256]
//   -> pi(obs; eps2) [271-273] -> alpha [274-284]
//   -> min_K Q_new(obs, a~) [286-292] -> Adam(pi) [295-300] -> Polyak [320-324]
// The policy forward on obs uses the pre-step policy (it is only updated at
// the end), so it runs in the first forward stage with everything else.
#include <cstdlib>
#include <cstring>

#include "../../include/oac_amd.h"
#include "kernels.h"
#include "oac_common.h"
#include "plan_common.h"
#include "sac_plan.h"

namespace oac {

enum PWs {
  // public ids (OAC_WS_*) keep their meaning: HEAD1/ACT1/LOGP1 = policy(obs),
  // HEAD2/ACT2/LOGP2 = policy(next_obs), EPS1 = next_obs noise (drawn first,
  // line 193), EPS2 = obs noise (line 271), Q1 = Q(obs,a) [B,K],
  // QN1 = Q_new(obs,a~) [B,K], TQ1 = TQ(next_obs,a') [B,K], Y / SQE1 [B,K]
  // in sorted-slot order, QNEW = min_K Q_new [B].
  X_H1P = OAC_WS_COUNT_PUBLIC, X_H2P, X_H1P2, X_H2P2, X_P, X_H1Q, X_H2Q, X_PT, X_H1T, X_H2T,
  X_STD1, X_U1, X_STD2, X_U2, X_DQ, X_DH2Q, X_DH1Q, X_PN, X_H1N, X_H2N, X_GQ, X_DH2N, X_DH1N,
  X_DA, X_DHEAD, X_DH2P, X_DH1P,
  X_COUNT
};
static_assert(X_COUNT <= kMaxWs, "workspace ids");

void particle_layout_workspace(SacPlan& p) {
  const oac_sac_config& c = p.c;
  const int64_t B = c.batch, H = c.hidden, Da = c.act_dim, K = c.q_out;
  for (int i = 0; i < kMaxWs; ++i) p.ws[i] = {0, 0, 0};
  auto set = [&](int id, int64_t r, int64_t cl) { p.ws[id] = {0, r, cl}; };
  set(OAC_WS_BATCH, B, c.row_stride);
  set(OAC_WS_EPS1, B, Da); set(OAC_WS_EPS2, B, Da);
  set(OAC_WS_HEAD1, B, 2 * Da); set(OAC_WS_HEAD2, B, 2 * Da);
  set(OAC_WS_ACT1, B, Da); set(OAC_WS_ACT2, B, Da);
  set(OAC_WS_LOGP1, B, 1); set(OAC_WS_LOGP2, B, 1);
  for (int id : {OAC_WS_Q1, OAC_WS_QN1, OAC_WS_TQ1, OAC_WS_Y, OAC_WS_SQE1}) set(id, B, K);
  set(OAC_WS_QNEW, B, 1);
  set(OAC_WS_COUNTS, B, 1);
  set(OAC_WS_LOGP_PART, (B + 15) / 16, 1);
  for (int id = X_H1P; id <= X_H2T; ++id) set(id, B, H);
  for (int id : {X_STD1, X_U1, X_STD2, X_U2, X_DA}) set(id, B, Da);
  set(X_DQ, B, K); set(X_GQ, B, K);
  for (int id : {X_DH2Q, X_DH1Q, X_PN, X_H1N, X_H2N, X_DH2N, X_DH1N, X_DH2P, X_DH1P}) set(id, B, H);
  set(X_DHEAD, B, 2 * Da);
  if (p.S_q > 1) set(WS_GSLAB_Q, p.S_q, p.L.n_critics * p.L.q_size);
  if (p.S_p > 1) set(WS_GSLAB_P, p.S_p, p.L.pol_size);
  int64_t off = 0;
  for (int i = 0; i < kMaxWs; ++i) {
    p.ws[i].off = off;
    off = al64(off + p.ws[i].rows * p.ws[i].cols);
  }
  p.L.workspace_floats = off + 64;   // tail pad: GEMM k-contiguous loads may read 7 floats past a row
}

// ------------------------------------------------------------------ phases
// the critic's backward into its last hidden layer inside the targets kernel
// (rank-K dX of the K-output head; OAC_TUNE_DH2_TARGETS = -1 keeps its GEMM launch)
static bool dh2_in_targets(const SacPlan& p) {
  const bool v = tuning(OAC_TUNE_DH2_TARGETS) >= 0;
  return v && (p.c.hidden & 3) == 0;
}

static int pphase0(SacPlan& p, int flags, hipStream_t s) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int Dq = Do + Da;
  float* X = p.W(OAC_WS_BATCH);
  // direct gather at large batch (as the SAC step's, sac_plan.hip phase0): the
  // layer-0 launch's LDS-DMA tiles read their rows straight from the replay
  // through the step's index slot, side workgroups of that launch draw eps,
  // and the batch copy (first read by the targets kernel) rides in the target
  // critic's layer-1 launch -- no gather launch
  const bool direct_big = big_direct_ok(p) && (flags & OAC_STEP_GATHER) && p.b.ring_slots > 0;
  p.direct_big = direct_big;
  p.direct_ring = gather_idx(p, flags);
  const float* R0 = direct_big ? p.b.replay : X;
  const float* obs = R0 + c.off_obs;
  const float* nobs = R0 + c.off_next_obs;
  if (!direct_big && (flags & (OAC_STEP_GATHER | OAC_STEP_DEVICE_EPS))) {
    GatherArgs g;
    std::memset(&g, 0, sizeof(g));
    g.replay = p.b.replay; g.row_stride = RS; g.idx = gather_idx(p, flags); g.ring_slots = p.b.ring_slots;
    g.out = X; g.B = (flags & OAC_STEP_GATHER) ? B : 0;
    if (flags & OAC_STEP_DEVICE_EPS) {
      g.eps1 = p.W(OAC_WS_EPS1); g.eps2 = p.W(OAC_WS_EPS2); g.n_eps = B * Da;
    }
    g.seed = c.seed; g.state = p.state();
    TIMED(p, K_GATHER, s, OAC_HIP_CHECK(launch_gather(g, s)));
    p.launches++;
  }
  if ((flags & (OAC_STEP_GATHER | OAC_STEP_COUNTS)) == (OAC_STEP_GATHER | OAC_STEP_COUNTS) &&
      p.b.counts) {   // ring path of a counts=True trainer: this draw's counts on the device
    CountsStepArgs ca{p.b.counts, p.b.count_tags, p.b.count_epoch, gather_idx(p, flags), p.b.ring_slots,
                      p.state(), c.batch, p.W(OAC_WS_COUNTS)};
    TIMED(p, K_GATHER, s, OAC_HIP_CHECK(launch_counts_step(ca, s)));
    p.launches++;
  }
  const float* pol = p.b.params;
  const float* q = p.b.params + L.q1_base;
  const float* tq = p.b.targets;
  {
    GemmBatch gb{};
    add(gb, t_fwd(obs, RS, B, Do, pol + L.pol_fc0_w, Do, H, p.W(X_H1P), H, EPI_BIAS_RELU, pol + L.pol_fc0_b));
    gb.publish = p.state(); gb.pub_beta1 = c.beta1; gb.pub_beta2 = c.beta2;   // step's Adam constants
    add(gb, t_fwd(nobs, RS, B, Do, pol + L.pol_fc0_w, Do, H, p.W(X_H1P2), H, EPI_BIAS_RELU, pol + L.pol_fc0_b));
    GemmTask t = t_fwd(obs, RS, B, Do, q + L.q_fc0_w, Dq, H, p.W(X_P), H, EPI_BIAS_RANK_RELU, q + L.q_fc0_b);
    t.U = R0 + c.off_act; t.ldu = RS; t.V = q + L.q_fc0_w + Do; t.ldv = Dq; t.R = Da;
    t.C2 = p.W(X_H1Q); t.ldc2 = H;
    add(gb, t);
    add(gb, t_fwd(nobs, RS, B, Do, tq + L.q_fc0_w, Dq, H, p.W(X_PT), H, EPI_BIAS, tq + L.q_fc0_b));
    if (direct_big) {
      for (int i = 0; i < gb.ntasks; ++i) gb.t[i].a_rows = 1;
      RowGather& g = gb.rg;
      g.ring = p.direct_ring; g.slots = p.b.ring_slots; g.B = B; g.state = p.state();
      if (flags & OAC_STEP_DEVICE_EPS) {   // 512 tiles of 128 x 64: a free slot per CU
        g.eps1 = p.W(OAC_WS_EPS1); g.eps2 = p.W(OAC_WS_EPS2); g.n_eps = B * Da; g.seed = c.seed;
        g.blocks = 256;
      }
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    add(gb, t_fwd(p.W(X_H1P), H, B, H, pol + L.pol_fc1_w, H, H, p.W(X_H2P), H, EPI_BIAS_RELU, pol + L.pol_fc1_b));
    add(gb, t_fwd(p.W(X_H1P2), H, B, H, pol + L.pol_fc1_w, H, H, p.W(X_H2P2), H, EPI_BIAS_RELU, pol + L.pol_fc1_b));
    add(gb, t_fwd(p.W(X_H1Q), H, B, H, q + L.q_fc1_w, H, H, p.W(X_H2Q), H, EPI_BIAS_RELU, q + L.q_fc1_b));
    if (run_gemm(p, gb, s)) return 1;
  }
  {  // policy heads, tanh-Gaussian sample + log-prob (both batches), and the
     // target critic's action columns on a' (next_obs batch) in one launch
     // (head.hip); Q(obs, a)'s K-output last layer runs in the targets kernel
    HeadArgs a;
    std::memset(&a, 0, sizeof(a));
    a.wh = pol + L.pol_head_w; a.bh = pol + L.pol_head_b; a.ld_wa = Dq;
    a.B = B; a.H = H; a.Da = Da;
    a.col_chunks = B >= 1024 ? std::max(1, (H + 255) / 256) : std::max(1, (H + 63) / 64);
    HeadSeg& s0 = a.seg[0];   // policy(obs; eps2) (particle_trainer_oac.py:271-273)
    s0.h2 = p.W(X_H2P); s0.eps = p.W(OAC_WS_EPS2); s0.head = p.W(OAC_WS_HEAD1);
    s0.act = p.W(OAC_WS_ACT1); s0.stdv = p.W(X_STD1); s0.u = p.W(X_U1); s0.logp = p.W(OAC_WS_LOGP1);
    s0.n_nets = 0;
    HeadSeg& s1 = a.seg[1];   // policy(next_obs; eps1) -> TQ(next_obs, a') layer 0 (:193-202)
    s1.h2 = p.W(X_H2P2); s1.eps = p.W(OAC_WS_EPS1); s1.head = p.W(OAC_WS_HEAD2);
    s1.act = p.W(OAC_WS_ACT2); s1.stdv = p.W(X_STD2); s1.u = p.W(X_U2); s1.logp = p.W(OAC_WS_LOGP2);
    s1.n_nets = 1;
    s1.wa[0] = tq + L.q_fc0_w + Do; s1.pre[0] = p.W(X_PT); s1.h1[0] = p.W(X_H1T);
    if (c.world_size > 1 && c.auto_alpha) {   // the local alpha partials for the all-reduce
      a.logp_part = p.W(OAC_WS_LOGP_PART); a.target_entropy = c.target_entropy;
    }
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_policy_head(a, 2, s)));
    p.launches++;
  }
  return 0;
}

static int pphase1(SacPlan& p, int flags, hipStream_t s) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int K = c.q_out, Dq = Do + Da;
  float* X = p.W(OAC_WS_BATCH);
  const float* q = p.b.params + L.q1_base;
  const float* tq = p.b.targets;
  {  // target critic layer 1 (its layer 0 finished in the head launch)
    GemmBatch gb{};
    add(gb, t_fwd(p.W(X_H1T), H, B, H, tq + L.q_fc1_w, H, H, p.W(X_H2T), H, EPI_BIAS_RELU, tq + L.q_fc1_b));
    if (p.direct_big) {   // the direct-gather step's batch copy: 256 tiles, a free slot per CU
      RowGather& g = gb.rg;
      g.ring = p.direct_ring; g.slots = p.b.ring_slots; g.B = B; g.state = p.state();
      g.replay = p.b.replay; g.row_stride = RS; g.out = X;
      g.blocks = 256;
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  {  // the target critic's K-output last layer runs inside the targets kernel (row_heads)
    ParticleTargetArgs a;
    std::memset(&a, 0, sizeof(a));
    a.th = RowHead{p.W(X_H2T), tq + L.q_last_w, tq + L.q_last_b, p.W(OAC_WS_TQ1), H};
    a.qh = RowHead{p.W(X_H2Q), q + L.q_last_w, q + L.q_last_b, p.W(OAC_WS_Q1), H};
    if (dh2_in_targets(p)) a.dh2 = p.W(X_DH2Q);   // the rank-K dX launch, folded
    a.q = p.W(OAC_WS_Q1); a.tq = p.W(OAC_WS_TQ1); a.batch = X; a.ld_batch = RS;
    a.off_rew = c.off_rew; a.off_term = c.off_term; a.reward_scale = c.reward_scale;
    a.discount = c.discount; a.B = B; a.K = K;
    a.dq = p.W(X_DQ); a.sqe = p.W(OAC_WS_SQE1); a.y = p.W(OAC_WS_Y);
    a.counts = (flags & OAC_STEP_COUNTS) ? p.W(OAC_WS_COUNTS) : nullptr;
    a.loss_scale = 1.f; a.soft_prob = -1.f; a.rescale_spread = 0.f;   // particle_trainer_oac.py
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_particle_targets(a, s)));
    p.launches++;
  }
  // last layer: dW_last slab and dh2 = (dq . W_last) * [h2 > 0]; with dh2
  // from the targets kernel, dW_last rides in the layer-0 dW launch
  const bool fold = dh2_in_targets(p);
  GemmTask tl;
  {
    float* gq = grad_q(p);
    tl = t_dw(p.W(X_DQ), K, K, B, p.W(X_H2Q), H, H, gq + L.q_last_w, gq + L.q_last_b,
              q_group(p), p.sp_ql);
    // train_bias=False: no ones column, the frozen bias keeps a zero gradient
    // (Adam then leaves it, and its moments, exactly unchanged)
    if (c.freeze_q_bias) { tl.N = H; tl.b_ones = 0; tl.bias_grad = nullptr; }
  }
  if (!fold) {
    GemmBatch gb{};
    add(gb, tl);
    add(gb, t_dx(p.W(X_DQ), K, B, K, q + L.q_last_w, H, H, p.W(X_DH2Q), H, p.W(X_H2Q), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    float* gq = grad_q(p);
    add(gb, t_dw(p.W(X_DH2Q), H, H, B, p.W(X_H1Q), H, H, gq + L.q_fc1_w, gq + L.q_fc1_b,
                 q_group(p), p.sp_q1));
    add(gb, t_dx(p.W(X_DH2Q), H, B, H, q + L.q_fc1_w, H, H, p.W(X_DH1Q), H, p.W(X_H1Q), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    float* gq = grad_q(p);
    add(gb, t_dw(p.W(X_DH1Q), H, H, B, X + c.off_obs, RS, Dq, gq + L.q_fc0_w, gq + L.q_fc0_b,
                 q_group(p), p.sp_q0));
    // the last layer's dW (M = K rows) beside the layer-0 dW (B=4096: 7.9 us,
    // fewest workgroups of the backward launches; in the layer-1 launch it
    // added 5.8 us)
    if (fold) add(gb, tl);
    if (run_gemm(p, gb, s)) return 1;
  }
  return 0;
}

// critic Adam done; post-step critic forward on (obs, a~), alpha, policy grads
static int pphase2(SacPlan& p, hipStream_t s) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int K = c.q_out, Dq = Do + Da;
  float* X = p.W(OAC_WS_BATCH);
  const float* pol = p.b.params;
  const float* q = p.b.params + L.q1_base;
  {
    GemmBatch gb{};
    GemmTask t = t_fwd(X + c.off_obs, RS, B, Do, q + L.q_fc0_w, Dq, H, p.W(X_PN), H,
                       EPI_BIAS_RANK_RELU, q + L.q_fc0_b);
    t.U = p.W(OAC_WS_ACT1); t.ldu = Da; t.V = q + L.q_fc0_w + Do; t.ldv = Dq; t.R = Da;
    t.C2 = p.W(X_H1N); t.ldc2 = H;
    add(gb, t);
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    add(gb, t_fwd(p.W(X_H1N), H, B, H, q + L.q_fc1_w, H, H, p.W(X_H2N), H, EPI_BIAS_RELU, q + L.q_fc1_b));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    ParticleMinArgs a;
    std::memset(&a, 0, sizeof(a));
    a.qn = p.W(OAC_WS_QN1); a.B = B; a.K = K; a.gq = p.W(X_GQ); a.qmin = p.W(OAC_WS_QNEW);
    // the post-step critic's last layer on (obs, a~) runs in this kernel (row_heads)
    a.hn = RowHead{p.W(X_H2N), q + L.q_last_w, q + L.q_last_b, p.W(OAC_WS_QN1), H};
    if ((H & 3) == 0) a.dh2 = p.W(X_DH2N);   // the dX launch into the last hidden layer, folded
    a.alpha = c.auto_alpha ? p.alpha() : nullptr; a.state = p.state(); a.logp = p.W(OAC_WS_LOGP1);
    a.target_entropy = c.target_entropy; a.lr = c.policy_lr; a.beta1 = c.beta1; a.beta2 = c.beta2;
    a.adam_eps = c.adam_eps; a.world_size = c.world_size;
    if (c.world_size > 1) { a.logp_part = p.W(OAC_WS_LOGP_PART); a.n_logp_part = (B + 15) / 16; }
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_particle_min(a, s)));
    p.launches++;
  }
  if (H & 3) {   // (otherwise done by the min kernel)
    GemmBatch gb{};
    add(gb, t_dx(p.W(X_GQ), K, B, K, q + L.q_last_w, H, H, p.W(X_DH2N), H, p.W(X_H2N), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    add(gb, t_dx(p.W(X_DH2N), H, B, H, q + L.q_fc1_w, H, H, p.W(X_DH1N), H, p.W(X_H1N), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {  // dL/da through the critic's action columns + the tanh-Gaussian head
     // backward in the epilogue (EPI_HEAD_BWD, small kernel; one launch)
    GemmBatch gb{};
    GemmTask t = t_dx(p.W(X_DH1N), H, B, H, q + L.q_fc0_w + Do, Dq, Da, p.W(X_DHEAD), 2 * Da,
                      nullptr, 0);
    t.epi = EPI_HEAD_BWD;
    t.ex[0] = p.W(OAC_WS_ACT1); t.ex[1] = p.W(X_STD1); t.ex[2] = p.W(X_U1);
    t.ex[3] = p.W(OAC_WS_EPS2); t.ex[4] = p.W(OAC_WS_HEAD1);
    t.ex[5] = c.auto_alpha ? &p.alpha()->alpha : nullptr;
    add(gb, t);
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    float* gp = grad_p(p);
    add(gb, t_dw(p.W(X_DHEAD), 2 * Da, 2 * Da, B, p.W(X_H2P), H, H, gp + L.pol_head_w,
                 gp + L.pol_head_b, L.pol_size, p.sp_ph));
    add(gb, t_dx(p.W(X_DHEAD), 2 * Da, B, 2 * Da, pol + L.pol_head_w, H, H, p.W(X_DH2P), H, p.W(X_H2P), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    float* gp = grad_p(p);
    add(gb, t_dw(p.W(X_DH2P), H, H, B, p.W(X_H1P), H, H, gp + L.pol_fc1_w, gp + L.pol_fc1_b,
                 L.pol_size, p.sp_p1));
    add(gb, t_dx(p.W(X_DH2P), H, B, H, pol + L.pol_fc1_w, H, H, p.W(X_DH1P), H, p.W(X_H1P), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    float* gp = grad_p(p);
    add(gb, t_dw(p.W(X_DH1P), H, H, B, X + c.off_obs, RS, Do, gp + L.pol_fc0_w, gp + L.pol_fc0_b,
                 L.pol_size, p.sp_p0));
    if (run_gemm(p, gb, s)) return 1;
  }
  return 0;
}

int particle_run_step(SacPlan& p, int flags, hipStream_t s) {
  p.launches = 0;
  if (pphase0(p, flags, s)) return 1;
  // One Adam launch per group here.  (Side-workgroup Adam, as the SAC step
  // runs it, measured slower at configs[4] -- its layer-0 dW launches are short
  // (7.7 us; 111 obs dims): the side work lengthened each by ~2.6 us while the
  // remaining Adam launches shrank by 0.5 us, 4,336 -> 4,275 steps/s -- and
  // with the last layer's dW in the layer-0 dW launch the side blocks would
  // update that layer while its gradient is still being written; the switch
  // that kept it for A/B runs is gone.)
  if (pphase1(p, flags, s)) return 1;
  {
    AdamArgs a = critic_adam(p, 0, nullptr);   // alpha is updated after the critic step
    TIMED(p, K_ADAM, s, OAC_HIP_CHECK(launch_adam(a, s)));
    p.launches++;
  }
  if (pphase2(p, s)) return 1;
  {
    AdamArgs a = policy_adam(p, 0, p.c.auto_alpha ? p.alpha() : nullptr);
    TIMED(p, K_ADAM, s, OAC_HIP_CHECK(launch_adam(a, s)));
    p.launches++;
  }
  return 0;
}

int particle_step_phase(SacPlan& p, int phase, int flags, hipStream_t s) {
  switch (phase) {
    case 0: return pphase0(p, flags, s);
    case 1:
      if (pphase1(p, flags, s)) return 1;
      if (p.S_q > 1) {
        AdamArgs a = critic_adam(p, 1, nullptr);
        OAC_HIP_CHECK(launch_adam(a, s));
      }
      return 0;
    case 2: {
      AdamArgs a = critic_adam(p, -1, nullptr);
      OAC_HIP_CHECK(launch_adam(a, s));
      if (pphase2(p, s)) return 1;
      if (p.S_p > 1) {
        AdamArgs b = policy_adam(p, 1, nullptr);
        OAC_HIP_CHECK(launch_adam(b, s));
      }
      return 0;
    }
    case 3: {
      AdamArgs a = policy_adam(p, -1, p.c.auto_alpha ? p.alpha() : nullptr);
      OAC_HIP_CHECK(launch_adam(a, s));
      return 0;
    }
    default:
      set_error("bad phase %d", phase);
      return 1;
  }
}

}  // namespace oac
