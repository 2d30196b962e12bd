// Deterministic-policy trainers with a separately trained target_policy, on
// MI355X: one critic with K outputs, its target, the policy and the
// target_policy (params = [policy | target_policy | critic], one Adam group
// over both policies).  Two reference trainers share this launch sequence and
// differ only in their row kernels:
//
// * g-oac GaussianTrainer, share_layers=True (OAC_KIND_GAUSS, K = 2 outputs
//   Q | log std; /root/reference/trainer/gaussian_trainer.py) -- the
//   configuration of reproduce_g-oac*.sh (GaussianTrainer's default
//   deterministic=True is not overridden for g-oac, main.py:219-233):
//     Q(obs,a) [187] -> a' = tanh(mean_pi(next_obs)) [199-202]
//     -> QT(next_obs,a') [204] -> q / std targets (counts, soft update, clamp)
//        [207-237] -> Adam(Q, grad MSE(q) + MSE(std)) [227-237]
//     -> a~ = tanh(mean_pi(obs)) [315-318] -> ub = Q_new(a~)_0 + z*exp(Q_new(a~)_1)
//        [325-331] -> Adam(pi, -mean(ub)) [334-337]
//     -> a~_T = tanh(mean_piT(obs)) [342-344] -> Adam(piT, -mean(Q_new(a~_T)_0))
//        [346-354] -> Polyak Q -> QT [359-362]
// * p-oac ParticleTrainer, share_layers=True (OAC_KIND_PARTICLE_UB, K
//   particles; /root/reference/trainer/particle_trainer.py) -- what main.py
//   builds for --alg p-oac without --beta_UB (main.py:198-204, 364, 488-490),
//   i.e. every reproduce_p-oac*.sh recipe: sorted-particle TD targets (counts,
//   soft update, rescale) with the loss averaged over particles [190-270], the
//   policy maximising the delta_index-th sorted particle of Q_new [317-330],
//   the target policy the particle mean [339-348], Polyak [353-357].
//
// mean_update: next actions come from the target policy (both trainers).
// Both policy forwards on obs use pre-step policies and the post-step critic,
// freshly evaluated (no saved-activation quirk): the critic Adam completes
// before either policy loss is formed.  The two policy losses are independent
// (pi's step touches neither Q nor piT), so their backward passes share
// launches, and one Adam pass updates [policy | target_policy].
#include <cstring>

#include "../../include/oac_amd.h"
#include "kernels.h"
#include "oac_common.h"
#include "plan_common.h"
#include "sac_plan.h"

namespace oac {

enum GWs {
  // public ids: HEAD1/ACT1 = pi(obs), HEAD2/ACT2 = next-action policy
  // (pi or, mean_update, piT) on next_obs, HEAD3/ACT3 = target_policy(obs);
  // Q1 = Q(obs,a) [B,K] raw, TQ1 = QT(next_obs,a') [B,K], QN1 = Q_new(obs,a~),
  // QN2 = Q_new(obs,a~_T) [B,K]; Y / SQE1 [B,K] (GAUSS: q | std; PARTICLE_UB:
  // sorted slots), QNEW = upper bound [B].
  G_H1P = OAC_WS_COUNT_PUBLIC, G_H2P, G_H1P2, G_H2P2, G_H1TP, G_H2TP,
  G_P, G_H1Q, G_H2Q, G_PT, G_H1T, G_H2T,
  G_DQ, G_DH2Q, G_DH1Q,
  G_PN, G_H1N, G_H2N, G_PN3, G_H1N3, G_H2N3, G_GQ, G_GQ3, G_DH2N, G_DH1N, G_DH2N3, G_DH1N3,
  G_DA, G_DA3, G_DHEAD, G_DHEAD3, G_DH2P, G_DH1P, G_DH2TP, G_DH1TP,
  G_COUNT
};
static_assert(G_COUNT <= WS_GSLAB_Q, "workspace ids");

void det_layout_workspace(SacPlan& p) {
  const oac_sac_config& c = p.c;
  const int64_t B = c.batch, H = c.hidden, Da = c.act_dim, K = c.q_out;
  for (int i = 0; i < kMaxWs; ++i) p.ws[i] = {0, 0, 0};
  auto set = [&](int id, int64_t r, int64_t cl) { p.ws[id] = {0, r, cl}; };
  set(OAC_WS_BATCH, B, c.row_stride);
  for (int id : {OAC_WS_HEAD1, OAC_WS_HEAD2, OAC_WS_HEAD3}) set(id, B, 2 * Da);
  for (int id : {OAC_WS_ACT1, OAC_WS_ACT2, OAC_WS_ACT3}) set(id, B, Da);
  for (int id : {OAC_WS_Q1, OAC_WS_QN1, OAC_WS_QN2, OAC_WS_TQ1, OAC_WS_Y, OAC_WS_SQE1}) set(id, B, K);
  set(OAC_WS_QNEW, B, 1);
  set(OAC_WS_COUNTS, B, 1);
  set(OAC_WS_LOGP_PART, (B + 15) / 16, 1);
  for (int id = G_H1P; id <= G_H2T; ++id) set(id, B, H);
  for (int id : {G_DQ, G_GQ, G_GQ3}) set(id, B, K);
  for (int id : {G_DH2Q, G_DH1Q, G_PN, G_H1N, G_H2N, G_PN3, G_H1N3, G_H2N3, G_DH2N, G_DH1N,
                 G_DH2N3, G_DH1N3, G_DH2P, G_DH1P, G_DH2TP, G_DH1TP})
    set(id, B, H);
  for (int id : {G_DA, G_DA3}) set(id, B, Da);
  for (int id : {G_DHEAD, G_DHEAD3}) set(id, B, 2 * Da);
  if (p.S_q > 1) set(WS_GSLAB_Q, p.S_q, q_group(p));
  if (p.S_p > 1) set(WS_GSLAB_P, p.S_p, p_group(p));
  int64_t off = 0;
  for (int i = 0; i < kMaxWs; ++i) {
    p.ws[i].off = off;
    off = al64(off + p.ws[i].rows * p.ws[i].cols);
  }
  p.L.workspace_floats = off + 64;   // tail pad: GEMM k-contiguous loads may read 7 floats past a row
}

// ------------------------------------------------------------------ phases
// forward of everything the pre-step parameters determine
static int dphase0(SacPlan& p, int flags, hipStream_t s) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int Dq = Do + Da;
  float* X = p.W(OAC_WS_BATCH);
  const float* obs = X + c.off_obs;
  const float* nobs = X + c.off_next_obs;
  if (flags & OAC_STEP_GATHER) {
    GatherArgs g;
    std::memset(&g, 0, sizeof(g));
    g.replay = p.b.replay; g.row_stride = RS; g.idx = gather_idx(p, flags); g.ring_slots = p.b.ring_slots;
    g.out = X; g.B = B;
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
  const float* tpol = p.b.params + L.tpol_base;
  // the policy acting on next_obs: target_policy (mean_update), the
  // use_target_policy network, or the policy itself
  const float* npol = c.mean_update ? tpol : (p.b.next_policy ? p.b.next_policy : pol);
  const float* q = p.b.params + L.q1_base;
  const float* tq = p.b.targets;
  {
    GemmBatch gb{};
    add(gb, t_fwd(obs, RS, B, Do, pol + L.pol_fc0_w, Do, H, p.W(G_H1P), H, EPI_BIAS_RELU, pol + L.pol_fc0_b));
    gb.publish = p.state(); gb.pub_beta1 = c.beta1; gb.pub_beta2 = c.beta2;   // step's Adam constants
    add(gb, t_fwd(nobs, RS, B, Do, npol + L.pol_fc0_w, Do, H, p.W(G_H1P2), H, EPI_BIAS_RELU, npol + L.pol_fc0_b));
    add(gb, t_fwd(obs, RS, B, Do, tpol + L.pol_fc0_w, Do, H, p.W(G_H1TP), H, EPI_BIAS_RELU, tpol + L.pol_fc0_b));
    GemmTask t = t_fwd(obs, RS, B, Do, q + L.q_fc0_w, Dq, H, p.W(G_P), H, EPI_BIAS_RANK_RELU, q + L.q_fc0_b);
    t.U = X + c.off_act; t.ldu = RS; t.V = q + L.q_fc0_w + Do; t.ldv = Dq; t.R = Da;
    t.C2 = p.W(G_H1Q); t.ldc2 = H;
    add(gb, t);
    add(gb, t_fwd(nobs, RS, B, Do, tq + L.q_fc0_w, Dq, H, p.W(G_PT), H, EPI_BIAS, tq + L.q_fc0_b));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    add(gb, t_fwd(p.W(G_H1P), H, B, H, pol + L.pol_fc1_w, H, H, p.W(G_H2P), H, EPI_BIAS_RELU, pol + L.pol_fc1_b));
    add(gb, t_fwd(p.W(G_H1P2), H, B, H, npol + L.pol_fc1_w, H, H, p.W(G_H2P2), H, EPI_BIAS_RELU, npol + L.pol_fc1_b));
    add(gb, t_fwd(p.W(G_H1TP), H, B, H, tpol + L.pol_fc1_w, H, H, p.W(G_H2TP), H, EPI_BIAS_RELU, tpol + L.pol_fc1_b));
    add(gb, t_fwd(p.W(G_H1Q), H, B, H, q + L.q_fc1_w, H, H, p.W(G_H2Q), H, EPI_BIAS_RELU, q + L.q_fc1_b));
    if (run_gemm(p, gb, s)) return 1;
  }
  {  // the three heads, a = tanh(mean), and the target critic's action
     // columns on next_obs (h1 = relu(P + a'. W0[:, Do:]), one launch (head.hip)
    HeadArgs a;
    std::memset(&a, 0, sizeof(a));
    a.ld_wa = Dq; a.det = 1;
    a.B = B; a.H = H; a.Da = Da;
    a.col_chunks = std::max(1, (H + (B >= 1024 ? 127 : 63)) / (B >= 1024 ? 128 : 64));
    HeadSeg& s0 = a.seg[0];   // policy(obs) -> a~ (post-step critic, phase 2)
    s0.h2 = p.W(G_H2P); s0.wh = pol + L.pol_head_w; s0.bh = pol + L.pol_head_b;
    s0.head = p.W(OAC_WS_HEAD1); s0.act = p.W(OAC_WS_ACT1);
    HeadSeg& s1 = a.seg[1];   // next-action policy(next_obs) -> QT(next_obs, a')
    s1.h2 = p.W(G_H2P2); s1.wh = npol + L.pol_head_w; s1.bh = npol + L.pol_head_b;
    s1.head = p.W(OAC_WS_HEAD2); s1.act = p.W(OAC_WS_ACT2);
    s1.n_nets = 1; s1.wa[0] = tq + L.q_fc0_w + Do; s1.pre[0] = p.W(G_PT); s1.h1[0] = p.W(G_H1T);
    HeadSeg& s2 = a.seg[2];   // target_policy(obs) -> a~_T (phase 2)
    s2.h2 = p.W(G_H2TP); s2.wh = tpol + L.pol_head_w; s2.bh = tpol + L.pol_head_b;
    s2.head = p.W(OAC_WS_HEAD3); s2.act = p.W(OAC_WS_ACT3);
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_policy_head(a, 3, s)));
    p.launches++;
  }
  return 0;
}

// target critic, TD targets, critic gradients (into grad_q)
static int dphase1(SacPlan& p, int flags, hipStream_t s, bool fused) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int Dq = Do + Da, K = c.q_out;
  float* X = p.W(OAC_WS_BATCH);
  const float* q = p.b.params + L.q1_base;
  const float* tq = p.b.targets;
  {  // target critic layer 1, and the critic's outputs Q(obs, a)
    GemmBatch gb{};
    add(gb, t_fwd(p.W(G_H1T), H, B, H, tq + L.q_fc1_w, H, H, p.W(G_H2T), H, EPI_BIAS_RELU, tq + L.q_fc1_b));
    add(gb, t_fwd(p.W(G_H2Q), H, B, H, q + L.q_last_w, H, K, p.W(OAC_WS_Q1), K, EPI_BIAS, q + L.q_last_b));
    if (run_gemm(p, gb, s)) return 1;
  }
  // the target critic's K-output last layer runs inside the targets kernel
  // (row_heads, rows.hip): one launch fewer on the chain
  const RowHead th{p.W(G_H2T), tq + L.q_last_w, tq + L.q_last_b, p.W(OAC_WS_TQ1), H};
  const float* counts = (flags & OAC_STEP_COUNTS) ? p.W(OAC_WS_COUNTS) : nullptr;
  if (c.kind == OAC_KIND_GAUSS) {
    GaussTargetArgs a;
    std::memset(&a, 0, sizeof(a));
    a.q = p.W(OAC_WS_Q1); a.tq = p.W(OAC_WS_TQ1); a.batch = X; a.ld_batch = RS;
    a.off_rew = c.off_rew; a.off_term = c.off_term; a.reward_scale = c.reward_scale;
    a.discount = c.discount; a.std_init = c.std_init;
    a.soft_prob = c.std_soft_update ? c.std_soft_prob : -1.f;
    a.counts = counts; a.th = th;
    a.B = B; a.dq = p.W(G_DQ); a.y = p.W(OAC_WS_Y); a.sqe = p.W(OAC_WS_SQE1);
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_gauss_targets(a, s)));
    p.launches++;
  } else {
    ParticleTargetArgs a;
    std::memset(&a, 0, sizeof(a));
    a.q = p.W(OAC_WS_Q1); a.tq = p.W(OAC_WS_TQ1); a.batch = X; a.ld_batch = RS;
    a.off_rew = c.off_rew; a.off_term = c.off_term; a.reward_scale = c.reward_scale;
    a.discount = c.discount; a.B = B; a.K = K;
    a.dq = p.W(G_DQ); a.sqe = p.W(OAC_WS_SQE1); a.y = p.W(OAC_WS_Y); a.counts = counts; a.th = th;
    a.loss_scale = 1.f / (float)K;                       // qf_loss /= num_particles
    a.soft_prob = c.std_soft_update ? c.std_soft_prob : -1.f;
    a.rescale_spread = c.rescale_spread;
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_particle_targets(a, s)));
    p.launches++;
  }
  {
    GemmBatch gb{};
    float* gq = grad_q(p);
    GemmTask tl = t_dw(p.W(G_DQ), K, K, B, p.W(G_H2Q), H, H, gq + L.q_last_w, gq + L.q_last_b,
                 q_group(p), p.sp_ql);
    // train_bias=False: no ones column, the frozen bias keeps a zero gradient
    // (Adam then leaves it, and its moments, exactly unchanged)
    if (c.freeze_q_bias) { tl.N = H; tl.b_ones = 0; tl.bias_grad = nullptr; }
    add(gb, tl);
    add(gb, t_dx(p.W(G_DQ), K, B, K, q + L.q_last_w, H, H, p.W(G_DH2Q), H, p.W(G_H2Q), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    float* gq = grad_q(p);
    add(gb, t_dw(p.W(G_DH2Q), H, H, B, p.W(G_H1Q), H, H, gq + L.q_fc1_w, gq + L.q_fc1_b,
                 q_group(p), p.sp_q1));
    add(gb, t_dx(p.W(G_DH2Q), H, B, H, q + L.q_fc1_w, H, H, p.W(G_DH1Q), H, p.W(G_H1Q), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    float* gq = grad_q(p);
    add(gb, t_dw(p.W(G_DH1Q), H, H, B, X + c.off_obs, RS, Dq, gq + L.q_fc0_w, gq + L.q_fc0_b,
                 q_group(p), p.sp_q0));
    if (fused) {   // critic Adam + Polyak in the epilogue (other layers: tail blocks)
      const long off[1] = {(long)L.q_fc1_w};
      const long n[1] = {(long)(L.q_size - L.q_fc1_w)};
      fuse_adam(gb, critic_adam(p, 0, nullptr), 1, off, n);
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  return 0;
}

// critic Adam done: post-step critic on (obs, a~) and (obs, a~_T), the two
// policy losses' gradients (into grad_p: policy block, target_policy block)
static int dphase2(SacPlan& p, hipStream_t s, bool fused) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int Dq = Do + Da, K = c.q_out;
  float* X = p.W(OAC_WS_BATCH);
  const float* pol = p.b.params;
  const float* tpol = p.b.params + L.tpol_base;
  const float* q = p.b.params + L.q1_base;
  {
    GemmBatch gb{};
    for (int k = 0; k < 2; ++k) {
      GemmTask t = t_fwd(X + c.off_obs, RS, B, Do, q + L.q_fc0_w, Dq, H, p.W(k ? G_PN3 : G_PN), H,
                         EPI_BIAS_RANK_RELU, q + L.q_fc0_b);
      t.U = p.W(k ? OAC_WS_ACT3 : OAC_WS_ACT1); t.ldu = Da; t.V = q + L.q_fc0_w + Do; t.ldv = Dq;
      t.R = Da; t.C2 = p.W(k ? G_H1N3 : G_H1N); t.ldc2 = H;
      add(gb, t);
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    add(gb, t_fwd(p.W(G_H1N), H, B, H, q + L.q_fc1_w, H, H, p.W(G_H2N), H, EPI_BIAS_RELU, q + L.q_fc1_b));
    add(gb, t_fwd(p.W(G_H1N3), H, B, H, q + L.q_fc1_w, H, H, p.W(G_H2N3), H, EPI_BIAS_RELU, q + L.q_fc1_b));
    if (run_gemm(p, gb, s)) return 1;
  }
  // the post-step critic's last layer on (obs, a~) runs inside the seed
  // kernel (row_heads); on (obs, a~_T) it is not needed at all: the target
  // policy's seed is a constant, only the hidden activations (ReLU masks)
  // of that forward enter its backward
  const RowHead hn{p.W(G_H2N), q + L.q_last_w, q + L.q_last_b, p.W(OAC_WS_QN1), H};
  if (c.kind == OAC_KIND_GAUSS) {
    GaussSeedArgs a;
    std::memset(&a, 0, sizeof(a));
    a.qn = p.W(OAC_WS_QN1); a.qt = p.W(OAC_WS_QN2); a.hn = hn; a.std_bound = c.std_bound; a.B = B;
    a.g = p.W(G_GQ); a.gt = p.W(G_GQ3); a.ub = p.W(OAC_WS_QNEW);
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_gauss_seed(a, s)));
    p.launches++;
  } else {
    ParticleUbSeedArgs a;
    std::memset(&a, 0, sizeof(a));
    a.qn = p.W(OAC_WS_QN1); a.qt = p.W(OAC_WS_QN2); a.hn = hn; a.B = B; a.K = K;
    a.delta_index = c.delta_index;
    a.g = p.W(G_GQ); a.gt = p.W(G_GQ3); a.ub = p.W(OAC_WS_QNEW);
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_particle_ub_seed(a, s)));
    p.launches++;
  }
  {
    GemmBatch gb{};
    add(gb, t_dx(p.W(G_GQ), K, B, K, q + L.q_last_w, H, H, p.W(G_DH2N), H, p.W(G_H2N), H));
    add(gb, t_dx(p.W(G_GQ3), K, B, K, q + L.q_last_w, H, H, p.W(G_DH2N3), H, p.W(G_H2N3), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    add(gb, t_dx(p.W(G_DH2N), H, B, H, q + L.q_fc1_w, H, H, p.W(G_DH1N), H, p.W(G_H1N), H));
    add(gb, t_dx(p.W(G_DH2N3), H, B, H, q + L.q_fc1_w, H, H, p.W(G_DH1N3), H, p.W(G_H1N3), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    add(gb, t_dx(p.W(G_DH1N), H, B, H, q + L.q_fc0_w + Do, Dq, Da, p.W(G_DA), Da, nullptr, 0));
    add(gb, t_dx(p.W(G_DH1N3), H, B, H, q + L.q_fc0_w + Do, Dq, Da, p.W(G_DA3), Da, nullptr, 0));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    DetHeadBwdArgs a;
    std::memset(&a, 0, sizeof(a));
    a.da[0] = p.W(G_DA); a.act[0] = p.W(OAC_WS_ACT1); a.dhead[0] = p.W(G_DHEAD);
    a.da[1] = p.W(G_DA3); a.act[1] = p.W(OAC_WS_ACT3); a.dhead[1] = p.W(G_DHEAD3);
    a.nseg = 2; a.B = B; a.act_dim = Da;
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_det_head_backward(a, s)));
    p.launches++;
  }
  const long pg = p_group(p);
  float* gp = grad_p(p);
  float* gtp = gp + L.tpol_base;
  {
    GemmBatch gb{};
    add(gb, t_dw(p.W(G_DHEAD), 2 * Da, 2 * Da, B, p.W(G_H2P), H, H, gp + L.pol_head_w,
                 gp + L.pol_head_b, pg, p.sp_ph));
    add(gb, t_dx(p.W(G_DHEAD), 2 * Da, B, 2 * Da, pol + L.pol_head_w, H, H, p.W(G_DH2P), H, p.W(G_H2P), H));
    add(gb, t_dw(p.W(G_DHEAD3), 2 * Da, 2 * Da, B, p.W(G_H2TP), H, H, gtp + L.pol_head_w,
                 gtp + L.pol_head_b, pg, p.sp_ph));
    add(gb, t_dx(p.W(G_DHEAD3), 2 * Da, B, 2 * Da, tpol + L.pol_head_w, H, H, p.W(G_DH2TP), H, p.W(G_H2TP), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    add(gb, t_dw(p.W(G_DH2P), H, H, B, p.W(G_H1P), H, H, gp + L.pol_fc1_w, gp + L.pol_fc1_b, pg, p.sp_p1));
    add(gb, t_dx(p.W(G_DH2P), H, B, H, pol + L.pol_fc1_w, H, H, p.W(G_DH1P), H, p.W(G_H1P), H));
    add(gb, t_dw(p.W(G_DH2TP), H, H, B, p.W(G_H1TP), H, H, gtp + L.pol_fc1_w, gtp + L.pol_fc1_b, pg, p.sp_p1));
    add(gb, t_dx(p.W(G_DH2TP), H, B, H, tpol + L.pol_fc1_w, H, H, p.W(G_DH1TP), H, p.W(G_H1TP), H));
    if (run_gemm(p, gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    add(gb, t_dw(p.W(G_DH1P), H, H, B, X + c.off_obs, RS, Do, gp + L.pol_fc0_w, gp + L.pol_fc0_b, pg, p.sp_p0));
    add(gb, t_dw(p.W(G_DH1TP), H, H, B, X + c.off_obs, RS, Do, gtp + L.pol_fc0_w, gtp + L.pol_fc0_b, pg, p.sp_p0));
    if (fused) {   // [policy | target_policy] Adam in the epilogue; advances the step
      const long off[2] = {(long)L.pol_fc1_w, (long)(L.tpol_base + L.pol_fc1_w)};
      const long n[2] = {(long)(L.pol_size - L.pol_fc1_w), (long)(L.pol_size - L.pol_fc1_w)};
      fuse_adam(gb, policy_adam(p, 0, nullptr), 2, off, n);
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  return 0;
}

int det_run_step(SacPlan& p, int flags, hipStream_t s) {
  p.launches = 0;
  const bool fused = can_fuse_adam(p);
  if (dphase0(p, flags, s)) return 1;
  if (dphase1(p, flags, s, fused)) return 1;
  if (!fused) {
    AdamArgs a = critic_adam(p, 0, nullptr);
    TIMED(p, K_ADAM, s, OAC_HIP_CHECK(launch_adam(a, s)));
    p.launches++;
  }
  if (dphase2(p, s, fused)) return 1;
  if (!fused) {
    AdamArgs a = policy_adam(p, 0, nullptr);
    TIMED(p, K_ADAM, s, OAC_HIP_CHECK(launch_adam(a, s)));
    p.launches++;
  }
  return 0;
}

// data-parallel split (no whole-batch quantity besides the gradients: the
// phase-0 exchange is empty)
int det_step_phase(SacPlan& p, int phase, int flags, hipStream_t s) {
  switch (phase) {
    case 0: return dphase0(p, flags, s);
    case 1:
      if (dphase1(p, flags, s, false)) return 1;
      if (p.S_q > 1) {
        AdamArgs a = critic_adam(p, 1, nullptr);
        OAC_HIP_CHECK(launch_adam(a, s));
      }
      return 0;
    case 2: {
      AdamArgs a = critic_adam(p, -1, nullptr);
      OAC_HIP_CHECK(launch_adam(a, s));
      if (dphase2(p, s, false)) return 1;
      if (p.S_p > 1) {
        AdamArgs b = policy_adam(p, 1, nullptr);
        OAC_HIP_CHECK(launch_adam(b, s));
      }
      return 0;
    }
    case 3: {
      AdamArgs a = policy_adam(p, -1, nullptr);
      OAC_HIP_CHECK(launch_adam(a, s));
      return 0;
    }
    default:
      set_error("bad phase %d", phase);
      return 1;
  }
}

}  // namespace oac
