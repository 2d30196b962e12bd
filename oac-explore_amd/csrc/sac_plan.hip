// SAC / OAC gradient step on MI355X: the launch plan behind oac_sac_step.
//
// Restates SACTrainer.train_from_torch (/root/reference/trainer/trainer.py:
// 126-280) as a fixed sequence of grouped-GEMM / row / fused-Adam kernels over
// HBM-resident flat buffers, in the reference's torch-1.4 update order:
//   E1 policy(obs)  E2 alpha  E3 min Q(obs,a~)  E4 Q(obs,a)  E5 policy(next_obs)
//   E6 y = r*scale + (1-d)*gamma*(min TQ(next_obs,a') - alpha*logp')
//   E7/E8 Q1 grads -> Adam, Q2 grads -> Adam, then the policy gradient through
//   the POST-step Q weights with the PRE-step activations,
//   policy Adam;  E9 Polyak with the post-step critics.
// The sequence is static (step counters live on the device), so it is
// captured once into a hipGraph and replayed per step.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/oac_amd.h"
#include "kernels.h"
#include "oac_common.h"
#include "plan_common.h"
#include "sac_plan.h"

namespace oac {

static thread_local char g_err[1024] = "";
thread_local ExtTiming g_ext_timing;
int g_tuning[OAC_TUNE_COUNT] = {};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ---------------------------------------------------------------- layout
static void compute_layout(const oac_sac_config& c, oac_sac_layout& L) {
  const int64_t Do = c.obs_dim, Da = c.act_dim, H = c.hidden, Q = c.q_out;
  int64_t o = 0;
  L.pol_fc0_w = o; o = al4(o + H * Do);
  L.pol_fc0_b = o; o = al4(o + H);
  L.pol_fc1_w = o; o = al4(o + H * H);
  L.pol_fc1_b = o; o = al4(o + H);
  L.pol_head_w = o; o = al4(o + 2 * Da * H);
  L.pol_head_b = o; o = al4(o + 2 * Da);
  L.pol_size = o;
  int64_t q = 0;
  L.q_fc0_w = q; q = al4(q + H * (Do + Da));
  L.q_fc0_b = q; q = al4(q + H);
  L.q_fc1_w = q; q = al4(q + H * H);
  L.q_fc1_b = q; q = al4(q + H);
  L.q_last_w = q; q = al4(q + Q * H);
  L.q_last_b = q; q = al4(q + Q);
  L.q_size = q;
  L.n_critics = (c.kind == OAC_KIND_SAC) ? 2 : 1;
  // GAUSS: the target_policy block follows the policy, so both policies form
  // one Adam group (same lr, same step) in front of the critic
  L.tpol_base = has_target_policy(c.kind) ? L.pol_size : -1;
  L.q1_base = has_target_policy(c.kind) ? 2 * L.pol_size : L.pol_size;
  L.q2_base = (L.n_critics == 2) ? L.q1_base + L.q_size : -1;
  L.params_total = L.q1_base + L.n_critics * L.q_size;
  L.targets_total = L.n_critics * L.q_size;
}

// Internal workspace buffers (the first OAC_WS_COUNT_PUBLIC are the public ids).
enum Ws {
  W_H1P = OAC_WS_COUNT_PUBLIC, W_H2P, W_H1P2, W_H2P2,
  W_P1, W_P2, W_PT1, W_PT2, W_H1Q1, W_H1Q2, W_H2Q1, W_H2Q2,
  W_H1N1, W_H1N2, W_H2N1, W_H2N2, W_H1T1, W_H1T2, W_H2T1, W_H2T2,
  W_STD1, W_U1, W_STD2, W_U2, W_DQ1, W_DQ2, W_GQ1, W_GQ2,
  W_DH1Q1, W_DH1Q2, W_DH1N1, W_DH1N2, W_DA1, W_DA2, W_DHEAD, W_DH2P, W_DH1P,
  W_QPART,   // [6][B][tiles]: per-tile partial dots of the width-1 critic heads
  W_QSHADOW, // fused small-batch step: both critics' post-step layer 1 + last layer (minq_merged)
  W_COUNT
};

static void layout_workspace(SacPlan& p) {
  const oac_sac_config& c = p.c;
  const int64_t B = c.batch, H = c.hidden, Da = c.act_dim, Q = c.q_out;
  auto set = [&](int id, int64_t r, int64_t cl) { p.ws[id] = {0, r, cl}; };
  for (int i = 0; i < kMaxWs; ++i) p.ws[i] = {0, 0, 0};
  set(OAC_WS_BATCH, kXSlots * B, c.row_stride);   // public view: slot 0 (B rows)
  set(OAC_WS_EPS1, kXSlots * B, Da); set(OAC_WS_EPS2, kXSlots * B, Da);
  set(OAC_WS_HEAD1, B, 2 * Da); set(OAC_WS_HEAD2, B, 2 * Da);
  set(OAC_WS_ACT1, B, Da); set(OAC_WS_ACT2, B, Da);
  set(OAC_WS_LOGP1, B, 1); set(OAC_WS_LOGP2, B, 1);
  for (int id : {OAC_WS_Q1, OAC_WS_Q2, OAC_WS_QN1, OAC_WS_QN2, OAC_WS_TQ1, OAC_WS_TQ2}) set(id, B, Q);
  for (int id : {OAC_WS_Y, OAC_WS_SQE1, OAC_WS_SQE2, OAC_WS_QNEW}) set(id, B, Q);
  set(OAC_WS_COUNTS, B, 1);   // unused by SAC (the reference SACTrainer ignores counts)
  set(OAC_WS_LOGP_PART, (B + 15) / 16, 1);
  for (int id = W_H1P; id <= W_H2T2; ++id) set(id, B, H);
  for (int id : {W_STD1, W_U1, W_STD2, W_U2, W_DA1, W_DA2}) set(id, B, Da);
  for (int id : {W_DQ1, W_DQ2, W_GQ1, W_GQ2}) set(id, B, Q);
  for (int id : {W_DH1Q1, W_DH1Q2, W_DH1N1, W_DH1N2, W_DH2P, W_DH1P}) set(id, B, H);
  set(W_DHEAD, B, 2 * Da);
  set(W_QPART, QV_COUNT * B, (H + 31) / 32);
  if (can_fuse_adam(p)) set(W_QSHADOW, 1, p.L.n_critics * p.L.q_size);   // (same indexing as the group)
  if (p.S_q > 1) set(WS_GSLAB_Q, p.S_q, p.L.n_critics * p.L.q_size);
  if (p.S_p > 1) set(WS_GSLAB_P, p.S_p, p.L.pol_size);
  if (p.cfg == kCfgLargeBatch) set(WS_TICKETS, 1, kLaTickets);
  int64_t off = 0;
  for (int i = 0; i < kMaxWs; ++i) {
    p.ws[i].off = off;
    off = al64(off + p.ws[i].rows * p.ws[i].cols);
  }
  p.L.workspace_floats = off + 64;   // tail pad: GEMM k-contiguous loads may read 7 floats past a row
}

// ----------------------------------------------------------------- phases
// phase 0: gather, forward of everything that does not need alpha, policy
//          sample (+ alpha update when world_size == 1)
// The width-1 critic heads ride on the layer-1 epilogue (EPI_BIAS_RELU_DOT;
// critic_targets adds the per-32-column partials): on the small-batch kernel
// and, since round 2, on the large-batch kernels (two N = 1 launches fewer at
// B=4096).  The large-batch step also runs dL/da + the tanh-Gaussian head
// backward as one small-kernel launch (the dL/da product is 17 wide; its
// epilogue is the head backward) instead of a GEMM launch and a row launch.
static bool head_bwd_fused_big() { return true; }
static bool qdot(const SacPlan& p) {
  return (p.cfg == 0 || p.cfg == kCfgLargeBatch) && p.c.q_out == 1 && (p.c.hidden + 31) / 32 <= 16;
}
static GemmTask q_l1(SacPlan& p, const float* in, const float* net, float* out, int qv) {
  const oac_sac_config& c = p.c;
  const int B = c.batch, H = c.hidden;
  GemmTask t = t_fwd(in, H, B, H, net + p.L.q_fc1_w, H, H, out, H, EPI_BIAS_RELU, net + p.L.q_fc1_b);
  if (qdot(p)) {
    t.epi = EPI_BIAS_RELU_DOT; t.aux = net + p.L.q_last_w;
    t.C2 = p.W(W_QPART) + (long)qv * B * p.ws[W_QPART].cols; t.ldc2 = B;   // [tile][row]
  }
  return t;
}

// the minibatches (and Philox eps) of steps [i, i + n) into slots 0..n-1
static int gather_steps(SacPlan& p, int flags, int n, hipStream_t s) {
  const oac_sac_config& c = p.c;
  const int B = c.batch, Da = c.act_dim;
  GatherArgs g;
  std::memset(&g, 0, sizeof(g));
  g.replay = p.b.replay; g.row_stride = c.row_stride; g.idx = gather_idx(p, flags); g.ring_slots = p.b.ring_slots;
  g.out = p.W(OAC_WS_BATCH); g.B = (flags & OAC_STEP_GATHER) ? B : 0;
  g.n_steps = n; g.out_stride = (long)B * c.row_stride; g.eps_stride = (long)B * Da;
  if (flags & OAC_STEP_DEVICE_EPS) {
    g.eps1 = p.W(OAC_WS_EPS1); g.eps2 = p.W(OAC_WS_EPS2); g.n_eps = B * Da;
  }
  g.seed = c.seed; g.state = p.state();
  TIMED(p, K_GATHER, s, OAC_HIP_CHECK(launch_gather(g, s)));
  p.launches++;
  return 0;
}

// The step's critic-side forward that needs only the critic parameters and the
// batch -- Q_i(obs, a) (obs projection + the batch actions' rank-Da part; the
// projection P_i is kept for Q_i(obs, a~)) and the target critics' next_obs
// projections.  Issued by phase 0, or, on the small-batch ring path, ahead of
// time inside the previous step's policy-backward launches (the critic Adam +
// Polyak of that step are done by then; nothing later in it reads these
// buffers), which takes four of the six layer-0 and two of the four layer-1
// products off the step's dependency chain.
static void add_critic_l0(SacPlan& p, GemmBatch& gb, const float* X) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int Dq = Do + Da;
  const float* qs[2] = {p.b.params + L.q1_base, p.b.params + L.q2_base};
  const int P_[2] = {W_P1, W_P2}, H1[2] = {W_H1Q1, W_H1Q2};
  for (int i = 0; i < 2; ++i) {
    GemmTask t = t_fwd(X + c.off_obs, RS, B, Do, qs[i] + L.q_fc0_w, Dq, H, p.W(P_[i]), H,
                       EPI_BIAS_RANK_RELU, qs[i] + L.q_fc0_b);
    t.U = X + c.off_act; t.ldu = RS; t.V = qs[i] + L.q_fc0_w + Do; t.ldv = Dq; t.R = Da;
    t.C2 = p.W(H1[i]); t.ldc2 = H;
    add(gb, t);
  }
}
static void add_target_l0(SacPlan& p, GemmBatch& gb, const float* X) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Dq = c.obs_dim + c.act_dim, RS = c.row_stride;
  const float* ts[2] = {p.b.targets, p.b.targets + L.q_size};
  const int PT[2] = {W_PT1, W_PT2};
  for (int i = 0; i < 2; ++i)
    add(gb, t_fwd(X + c.off_next_obs, RS, B, Do, ts[i] + L.q_fc0_w, Dq, H, p.W(PT[i]), H, EPI_BIAS,
                  ts[i] + L.q_fc0_b));
}
static void add_critic_l1(SacPlan& p, GemmBatch& gb) {
  const float* q1 = p.b.params + p.L.q1_base;
  const float* q2 = p.b.params + p.L.q2_base;
  add(gb, q_l1(p, p.W(W_H1Q1), q1, p.W(W_H2Q1), QV_Q1));
  add(gb, q_l1(p, p.W(W_H1Q2), q2, p.W(W_H2Q2), QV_Q2));
}

// Fused small-batch step (can_fuse_adam): the critic layer-1 backward launch
// applies Adam to its layer-1 / last-layer dW tiles in their epilogue, with
// the updated weights written to W_QSHADOW instead of in place (that
// launch's dh1 tiles still read the pre-step weights).  The -min Q backward to
// layer 1 -- which needs exactly those post-step weights -- then reads them
// from the shadow and runs inside the critic layer-0 dW launch (whose side
// blocks copy the shadow into the parameters) instead of a launch of its own:
// one launch fewer on the step's chain.
static bool minq_merged(const SacPlan& p) {
  return can_fuse_adam(p) && p.ws[W_QSHADOW].rows > 0;
}

// -min Q backward to layer 1 with post-step weights (critic i's layer 1 and
// last layer at qw[i]: the parameters, or the shadow), pre-step masks
static void add_minq_bwd(SacPlan& p, GemmBatch& gb, const float* const (&qw)[2]) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden;
  const int gq[2] = {W_GQ1, W_GQ2}, h2[2] = {W_H2N1, W_H2N2}, h1[2] = {W_H1N1, W_H1N2};
  const int out[2] = {W_DH1N1, W_DH1N2};
  for (int i = 0; i < 2; ++i) {
    GemmTask d = t_dx(nullptr, 0, B, H, qw[i] + L.q_fc1_w, H, H, p.W(out[i]), H, p.W(h1[i]), H);
    set_rank1(d, p.W(gq[i]), qw[i] + L.q_last_w, p.W(h2[i]), H);
    add(gb, d);
  }
}

// Critic i's layer-0 dW over input columns [c0, c0 + n) of the [obs | act]
// row (+ the bias column when `bias`); (0, Dq, true) is the whole product.
// Each element's sum over the batch does not depend on the column range, so
// the parts are bitwise the whole.
static GemmTask critic_dw0(SacPlan& p, int i, int c0, int n, bool bias) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  float* g = grad_q(p) + i * L.q_size;
  const int dh1 = i ? W_DH1Q2 : W_DH1Q1;
  GemmTask t = t_dw(p.W(dh1), c.hidden, c.hidden, c.batch, p.X() + c.off_obs + c0, c.row_stride, n,
                    g + L.q_fc0_w + c0, g + L.q_fc0_b, q_group(p), p.sp_q0);
  t.ldc = c.obs_dim + c.act_dim;
  if (!bias) { t.N = n; t.b_ones = 0; t.bias_grad = nullptr; }
  return t;
}

// With the -min Q backward merged (minq_merged), the dL/da launch after it
// reads only the action columns of the post-step critic layer 0 -- so the
// layer-0 launch computes the action columns' Adam as a preview of p into the
// shadow (the dL/da launch reads them there; m, v, target untouched) and
// only one critic's obs-column dW (the other's rides in the dL/da launch),
// 240 tiles on 16-wave workgroups instead of 336 on 8; the whole layer-0
// Adam + Polyak of both critics then runs as side blocks of the policy-head
// launch (nothing in it or later in the step reads the critic's layer 0).
// Not with a next-step prefetch: its critic forward reads the post-step
// layer 0 in the dL/da launch.
static void add_dw0_side_adam(SacPlan& p, GemmBatch& gb) {
  for (int k = 0; k < gb.ntasks; ++k) gb.t[k].no_adam = 1;   // (the policy's gradients)
  const oac_sac_layout& L = p.L;
  const long off[2] = {0, (long)L.q_size};
  const long n[2] = {(long)L.q_fc1_w, (long)L.q_fc1_w};
  AdamArgs a = critic_adam(p, 0, nullptr);
  a.no_book = 1;
  fuse_adam(gb, a, 2, off, n);
}

int side_adam(SacPlan& p, GemmBatch& gb, const AdamArgs& a, int nseg, const long* off,
              const long* n, bool book, hipStream_t s) {
  const int cfg = launch_cfg(p.cfg, gb);
  if (((cfg >= 9 && cfg <= 12) || cfg == 15 || cfg == 17) && nseg <= 2) {
    // one float4 per thread, dispatched after the tiles (B=4096 SAC, same
    // box: one Adam launch per group 3,429 steps/s; side blocks after the
    // tiles, 32 per launch 3,186 -- the side work became the launch's tail --,
    // 64 3,419, 128 3,508, one float4 per thread 3,485; ahead of the tiles
    // 3,442)
    long n4 = 0;
    for (int i = 0; i < nseg; ++i) n4 += n[i] >> 2;
    const int blocks = (int)std::min<long>(1024, (n4 + 255) / 256);
    gb.side_adam = std::max(8, (blocks + 7) & ~7);
    gb.side_first = 0;
    gb.side_book = book ? 1 : 0;
    gb.adam = a;
    gb.nseg = nseg;
    for (int i = 0; i < nseg; ++i) { gb.seg_off[i] = off[i]; gb.seg_n[i] = n[i]; }
    return 0;
  }
  for (int i = 0; i < nseg; ++i) {
    AdamArgs r = a;
    r.p += off[i]; r.g += off[i]; r.m += off[i]; r.v += off[i];
    r.gslab += off[i];
    r.s2_lo -= off[i]; r.s2_hi -= off[i];
    if (r.target) r.target += off[i];
    r.n = n[i];
    r.no_book = (book && i == 0) ? 0 : 1;
    TIMED(p, K_ADAM, s, OAC_HIP_CHECK(launch_adam(r, s)));
    p.launches++;
  }
  return 0;
}

// policy_head workgroups per 16-row block: 64 hidden columns each at small
// batch (more workgroups in flight); at large batch one workgroup takes the
// whole hidden layer of both nets (4 (net, column tile) pairs per wave), so
// the row block's heads are computed once and the 512 workgroups of 8 waves
// (114 VGPRs: 4 waves per SIMD) run as a single round -- two chunks of 128
// columns made 1,024 workgroups and two rounds (B=4096: 24.4 us)
static int head_col_chunks(int B, int H) {
  const int forced = tuning(OAC_TUNE_HEAD_CC);
  if (forced > 0) return forced;
  return B >= 1024 ? std::max(1, (H + 255) / 256) : std::max(1, (H + 63) / 64);
}

static int phase0(SacPlan& p, int flags, hipStream_t s, int gather_n = 1, bool critic_done = false) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int Dq = Do + Da;
  float* X = p.X();
  // direct drop-in step: the layer-0 launch reads the batch rows through the
  // host-written index slot and its side blocks do the gather's copy + eps
  const bool direct = (p.rows_direct || p.ring_direct) && p.cfg == 0 && gather_n == 1 &&
                      !critic_done && (flags & OAC_STEP_GATHER) && p.b.ring_slots > 0;
  // the same at large batch: the LDS-DMA forward kernel stages layer 0's rows
  // straight from the replay through the step's index slot, and side
  // workgroups of that launch copy the batch and draw eps (gemm_fwd.hip;
  // the conditions keep every layer-0 product on that kernel)
  const bool direct_big = !direct && big_direct_ok(p) && gather_n == 1 && !critic_done &&
                          (flags & OAC_STEP_GATHER) && p.b.ring_slots > 0;
  if (!direct && !direct_big && gather_n > 0 && (flags & (OAC_STEP_GATHER | OAC_STEP_DEVICE_EPS)))
    if (gather_steps(p, flags, gather_n, s)) return 1;
  const float* pol = p.b.params;
  const float* q1 = p.b.params + L.q1_base;
  const float* q2 = p.b.params + L.q2_base;
  const float* t1 = p.b.targets;
  const float* t2 = p.b.targets + L.q_size;
  {  // layer 0: policy(obs), policy(next_obs), critic obs-projections
    GemmBatch gb{};
    gb.publish = p.state(); gb.pub_beta1 = c.beta1; gb.pub_beta2 = c.beta2;   // step's Adam constants
    const float* R0 = (direct || direct_big) ? p.b.replay : X;   // rows base: the replay (indexed) or the batch
    add(gb, t_fwd(R0 + c.off_obs, RS, B, Do, pol + L.pol_fc0_w, Do, H, p.W(W_H1P), H, EPI_BIAS_RELU, pol + L.pol_fc0_b));
    add(gb, t_fwd(R0 + c.off_next_obs, RS, B, Do, pol + L.pol_fc0_w, Do, H, p.W(W_H1P2), H, EPI_BIAS_RELU, pol + L.pol_fc0_b));
    if (!critic_done) {
      add_critic_l0(p, gb, R0);
      add_target_l0(p, gb, R0);
    }
    p.direct_big = direct_big;
    p.direct_ring = gather_idx(p, flags);
    if (direct) p.trace |= OAC_TRACE_DIRECT;
    if (direct_big) p.trace |= OAC_TRACE_DIRECT_BIG;
    if (direct_big) {   // every layer-0 product reads its rows through the index slot
      for (int i = 0; i < gb.ntasks; ++i) gb.t[i].a_rows = 1;
      RowGather& g = gb.rg;
      g.ring = gather_idx(p, flags); g.slots = p.b.ring_slots; g.B = B; g.state = p.state();
    }
    if (direct) {
      for (int i = 0; i < gb.ntasks; ++i) gb.t[i].a_rows = 1;
      RowGather& g = gb.rg;
      g.ring = p.rows_direct ? p.host_ring : gather_idx(p, flags);
      g.slots = p.b.ring_slots; g.B = B; g.state = p.state();
      g.replay = p.b.replay; g.row_stride = RS; g.out = X;
      // the staged indices in the kernel arguments (not under capture: a
      // captured launch would replay this step's indices)
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (p.inline_ok && B <= kInlineRows && hipStreamIsCapturing(s, &cs) == hipSuccess &&
          cs == hipStreamCaptureStatusNone)
        g.inl = p.inline_rows;
      if (flags & OAC_STEP_DEVICE_EPS) {
        g.eps1 = p.E1(); g.eps2 = p.E2(); g.n_eps = B * Da;
      }
      g.seed = c.seed;
      // a wave per row (>= 8 waves per workgroup), the eps on the same threads
      g.blocks = std::max(1, (B + 7) / 8);
    }
    if (run_gemm(p, gb, s)) return 1;
    p.inline_ok = false;   // (one staging call, one step)
  }
  {  // layer 1
    GemmBatch gb{};
    add(gb, t_fwd(p.W(W_H1P), H, B, H, pol + L.pol_fc1_w, H, H, p.W(W_H2P), H, EPI_BIAS_RELU, pol + L.pol_fc1_b));
    add(gb, t_fwd(p.W(W_H1P2), H, B, H, pol + L.pol_fc1_w, H, H, p.W(W_H2P2), H, EPI_BIAS_RELU, pol + L.pol_fc1_b));
    if (!critic_done) add_critic_l1(p, gb);
    if (direct_big && (flags & OAC_STEP_DEVICE_EPS)) {   // the step's eps: side workgroups
      RowGather& g = gb.rg;                               // (2 tiles per CU: a slot is free)
      g.state = p.state(); g.eps1 = p.E1(); g.eps2 = p.E2(); g.n_eps = B * Da; g.seed = c.seed;
      g.blocks = 256;
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  if (!qdot(p)) {  // q1/q2 predictions (the small-batch path has them from layer 1)
    GemmBatch gb{};
    add(gb, t_fwd(p.W(W_H2Q1), H, B, H, q1 + L.q_last_w, H, 1, p.W(OAC_WS_Q1), 1, EPI_BIAS, q1 + L.q_last_b));
    add(gb, t_fwd(p.W(W_H2Q2), H, B, H, q2 + L.q_last_w, H, 1, p.W(OAC_WS_Q2), 1, EPI_BIAS, q2 + L.q_last_b));
    if (run_gemm(p, gb, s)) return 1;
  }
  {  // policy heads, tanh-Gaussian sample + log-prob, critics' action columns
    HeadArgs a;
    std::memset(&a, 0, sizeof(a));
    a.wh = pol + L.pol_head_w; a.bh = pol + L.pol_head_b; a.ld_wa = Dq;
    a.B = B; a.H = H; a.Da = Da;
    // 64 hidden columns per workgroup at small batch (more workgroups in
    // flight); at large batch the fewest chunks the per-wave prefetch allows
    // (each chunk recomputes the row block's heads)
    a.col_chunks = head_col_chunks(B, H);
    HeadSeg& s0 = a.seg[0];   // policy(obs; eps1) -> Q1/Q2(obs, a~)
    s0.h2 = p.W(W_H2P); s0.eps = p.E1(); s0.head = p.W(OAC_WS_HEAD1);
    s0.act = p.W(OAC_WS_ACT1); s0.stdv = p.W(W_STD1); s0.u = p.W(W_U1); s0.logp = p.W(OAC_WS_LOGP1);
    s0.n_nets = 2;
    s0.wa[0] = q1 + L.q_fc0_w + Do; s0.pre[0] = p.W(W_P1); s0.h1[0] = p.W(W_H1N1);
    s0.wa[1] = q2 + L.q_fc0_w + Do; s0.pre[1] = p.W(W_P2); s0.h1[1] = p.W(W_H1N2);
    HeadSeg& s1 = a.seg[1];   // policy(next_obs; eps2) -> TQ1/TQ2(next_obs, a')
    s1.h2 = p.W(W_H2P2); s1.eps = p.E2(); s1.head = p.W(OAC_WS_HEAD2);
    s1.act = p.W(OAC_WS_ACT2); s1.stdv = p.W(W_STD2); s1.u = p.W(W_U2); s1.logp = p.W(OAC_WS_LOGP2);
    s1.n_nets = 2;
    s1.wa[0] = t1 + L.q_fc0_w + Do; s1.pre[0] = p.W(W_PT1); s1.h1[0] = p.W(W_H1T1);
    s1.wa[1] = t2 + L.q_fc0_w + Do; s1.pre[1] = p.W(W_PT2); s1.h1[1] = p.W(W_H1T2);
    if (c.world_size > 1 && c.auto_alpha) {   // the local alpha partials for the all-reduce
      a.logp_part = p.W(OAC_WS_LOGP_PART); a.target_entropy = c.target_entropy;
    }
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_policy_head(a, 2, s)));
    p.launches++;
  }
  return 0;
}

// Large-batch SAC: the width-1 last layers' dW as slabs of the targets kernel
// (one 256-row block per split) instead of 64-row GEMM tiles with one useful
// row -- the critic layer-1 backward launch keeps 1,024 workgroups (one round
// at four per CU) instead of 1,152: B=4096 34.1 -> 27.5 us for that launch
// (At B=256 the same, with layer 1's bias gradient -- the small kernel's ones
// column tiles -- also from the targets kernel, made the layer-1 backward one
// round of 256 tiles, 8.0 -> 5.6 us, but the targets launch 5.3 -> 8.3-9.1
// us: eight blocks each redoing the row math and the h2 pass; not kept.)
static bool wl_in_targets(const SacPlan& p) {
  const oac_sac_config& c = p.c;
  return c.kind == OAC_KIND_SAC && c.q_out == 1 && p.cfg == kCfgLargeBatch &&
         p.sp_ql.kchunk == 256 && p.sp_ql.S * 256 == c.batch && c.hidden % 32 == 0;
}

// phase 1: fresh-action critics, TD target, critic gradients (split-K slabs);
// fused: the critic Adam + Polyak runs inside the layer-0 gradient launch
// part 0: the whole phase; 1: the fresh-action critic forward only (layer 1 +
// last layer: no alpha needed, so the data-parallel alpha all-reduce overlaps
// it); 2: the rest (targets through the critic gradients)
static int phase1(SacPlan& p, hipStream_t s, bool fused, int part = 0, bool split = false,
                  bool defer = false) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int Dq = Do + Da;
  float* X = p.X();
  const float* q1 = p.b.params + L.q1_base;
  const float* q2 = p.b.params + L.q2_base;
  const float* t1 = p.b.targets;
  const float* t2 = p.b.targets + L.q_size;
  if (part != 2) {  // layer 1
    GemmBatch gb{};
    const float* nets[4] = {q1, q2, t1, t2};
    const int ins[4] = {W_H1N1, W_H1N2, W_H1T1, W_H1T2};
    const int outs[4] = {W_H2N1, W_H2N2, W_H2T1, W_H2T2};
    const int qv[4] = {QV_QN1, QV_QN2, QV_TQ1, QV_TQ2};
    for (int i = 0; i < 4; ++i) add(gb, q_l1(p, p.W(ins[i]), nets[i], p.W(outs[i]), qv[i]));
    if (p.direct_big) {   // the direct-gather step's batch copy (its first reader is the
      RowGather& g = gb.rg;   // targets kernel next): side workgroups in the free slot per CU
      g.ring = p.direct_ring; g.slots = p.b.ring_slots; g.B = B; g.state = p.state();
      g.replay = p.b.replay; g.row_stride = RS; g.out = X;
      g.blocks = 256;
      p.trace |= OAC_TRACE_BATCH_COPY;
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  if (part != 2 && !qdot(p)) {  // last layer
    GemmBatch gb{};
    const float* nets[4] = {q1, q2, t1, t2};
    const int ins[4] = {W_H2N1, W_H2N2, W_H2T1, W_H2T2};
    const int outs[4] = {OAC_WS_QN1, OAC_WS_QN2, OAC_WS_TQ1, OAC_WS_TQ2};
    for (int i = 0; i < 4; ++i)
      add(gb, t_fwd(p.W(ins[i]), H, B, H, nets[i] + L.q_last_w, H, 1, p.W(outs[i]), 1, EPI_BIAS,
                    nets[i] + L.q_last_b));
    if (run_gemm(p, gb, s)) return 1;
  }
  if (part == 1) return 0;
  {  // TD target, MSE gradients, policy seeds
    CriticTargetArgs a;
    std::memset(&a, 0, sizeof(a));
    const int qid[QV_COUNT] = {OAC_WS_Q1, OAC_WS_Q2, OAC_WS_QN1, OAC_WS_QN2, OAC_WS_TQ1, OAC_WS_TQ2};
    const float* nets[QV_COUNT] = {q1, q2, q1, q2, t1, t2};
    for (int k = 0; k < QV_COUNT; ++k) {
      a.q[k] = p.W(qid[k]);
      if (qdot(p)) {
        a.part[k] = p.W(W_QPART) + (long)k * B * p.ws[W_QPART].cols;
        a.part_bias[k] = nets[k] + L.q_last_b;
      }
    }
    a.n_part = qdot(p) ? (int)p.ws[W_QPART].cols : 0;
    if (qdot(p)) p.trace |= OAC_TRACE_QDOT;
    a.logp2 = p.W(OAC_WS_LOGP2);
    a.batch = X; a.ld_batch = RS; a.off_rew = c.off_rew; a.off_term = c.off_term;
    a.alpha = c.auto_alpha ? p.alpha() : nullptr;
    a.state = p.state(); a.logp1 = p.W(OAC_WS_LOGP1); a.target_entropy = c.target_entropy;
    a.lr = c.policy_lr; a.beta1 = c.beta1; a.beta2 = c.beta2; a.adam_eps = c.adam_eps;
    a.world_size = c.world_size;
    if (c.world_size > 1) { a.logp_part = p.W(OAC_WS_LOGP_PART); a.n_logp_part = (B + 15) / 16; }
    a.reward_scale = c.reward_scale; a.discount = c.discount; a.B = B;
    a.y = p.W(OAC_WS_Y); a.dq1 = p.W(W_DQ1); a.dq2 = p.W(W_DQ2); a.gq1 = p.W(W_GQ1); a.gq2 = p.W(W_GQ2);
    a.sqe1 = p.W(OAC_WS_SQE1); a.sqe2 = p.W(OAC_WS_SQE2); a.qnew = p.W(OAC_WS_QNEW);
    if (wl_in_targets(p)) {   // the last-layer dW slabs (the rows of block s = split s)
      float* gq = grad_q(p);
      const int h2[2] = {W_H2Q1, W_H2Q2};
      for (int i = 0; i < 2; ++i) {
        a.wl_h2[i] = p.W(h2[i]);
        a.wl_g[i] = gq + i * L.q_size + L.q_last_w;
        a.wl_gb[i] = gq + i * L.q_size + L.q_last_b;
      }
      a.wl_slab_stride = q_group(p); a.wl_H = H;
      p.trace |= OAC_TRACE_WL_TARGETS;
    }
    TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_critic_targets(a, s)));
    p.launches++;
  }
  {  // critic backward, hidden layer 1 + last layer (dW slabs) and dh1
    GemmBatch gb{};
    const float* qs[2] = {q1, q2};
    const int dq[2] = {W_DQ1, W_DQ2}, h2[2] = {W_H2Q1, W_H2Q2}, h1[2] = {W_H1Q1, W_H1Q2};
    const int dh1[2] = {W_DH1Q1, W_DH1Q2};
    float* gq = grad_q(p);
    const long gs = q_group(p);
    // small batch, unsplit: the layer-1 bias column and the width-1 last layer
    // (dW = dq^T h2, its bias sum dq) folded into the layer-1 dW tiles of the
    // first column block, which load dq and h2 as the rank-1 seed's factors
    // anyway (GemmTask::fold): 290 -> 256 tiles, one round of 16-wave workgroups
    const bool fold = p.cfg == 0 && !wl_in_targets(p) && p.sp_q1.S == 1 && p.sp_ql.S == 1;
    for (int i = 0; i < 2; ++i) {
      float* g = gq + i * L.q_size;   // critic i's block in the gradient (slab) layout
      GemmTask t = t_dw(nullptr, 0, H, B, p.W(h1[i]), H, H, g + L.q_fc1_w, g + L.q_fc1_b, gs, p.sp_q1);
      set_rank1(t, p.W(dq[i]), qs[i] + L.q_last_w, p.W(h2[i]), H);
      if (fold) {
        t.N = H; t.b_ones = 0; t.fold = 1;   // bias_grad keeps the layer-1 bias gradient
        t.C2 = g + L.q_last_w; t.ldc2 = (long)L.q_last_b - (long)L.q_last_w;
      }
      add(gb, t);
      if (!wl_in_targets(p) && !fold)   // (else the targets kernel or the fold wrote these)
        add(gb, t_dw(p.W(dq[i]), 1, 1, B, p.W(h2[i]), H, H, g + L.q_last_w, g + L.q_last_b, gs, p.sp_ql));
      GemmTask d = t_dx(nullptr, 0, B, H, qs[i] + L.q_fc1_w, H, H, p.W(dh1[i]), H, p.W(h1[i]), H);
      set_rank1(d, p.W(dq[i]), qs[i] + L.q_last_w, p.W(h2[i]), H);
      add(gb, d);
    }
    if (fused && minq_merged(p)) {   // layer 1 + last layer: Adam in the dW epilogues, into the shadow
      AdamArgs a = critic_adam(p, 0, nullptr);
      a.no_book = 1;   // (the layer-0 launch does the step's bookkeeping)
      a.p_out = p.W(W_QSHADOW);
      fuse_adam(gb, a, 0, nullptr, nullptr);
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  {  // critic backward, layer 0 (input = [obs | act] contiguous in the row)
    GemmBatch gb{};
    const bool dfr = defer && fused && minq_merged(p);
    for (int i = 0; i < 2; ++i)
      add(gb, dfr ? critic_dw0(p, i, Do, Da, true) : critic_dw0(p, i, 0, Dq, true));
    if (dfr) {   // critic 1's obs columns: gradient only (their Adam: the policy-head launch)
      GemmTask t = critic_dw0(p, 0, 0, Do, false);
      t.no_adam = 1;
      add(gb, t);
    }
    if (fused) {  // SAC commits the alpha update in the critic Adam
      const long off[2] = {(long)L.q_fc1_w, (long)(L.q_size + L.q_fc1_w)};
      const long n[2] = {(long)(L.q_size - L.q_fc1_w), (long)(L.q_size - L.q_fc1_w)};
      AdamArgs a = critic_adam(p, 0, c.auto_alpha ? p.alpha() : nullptr);
      if (dfr) { a.p_out = p.W(W_QSHADOW); a.preview = 1; }   // action columns: p preview only
      if (minq_merged(p)) {   // side blocks: the shadow's layer 1 + last layer into the parameters;
        a.copy_src = p.W(W_QSHADOW);   // the -min Q backward reads them from the shadow
        const float* sh = p.W(W_QSHADOW);
        const float* const qw[2] = {sh, sh + L.q_size};
        add_minq_bwd(p, gb, qw);
      }
      fuse_adam(gb, a, 2, off, n);
    } else if (split) {   // layer 1 + last layer of both critics (their gradients are final)
      const long off[2] = {(long)L.q_fc1_w, (long)(L.q_size + L.q_fc1_w)};
      const long n[2] = {(long)(L.q_size - L.q_fc1_w), (long)(L.q_size - L.q_fc1_w)};
      // (a range reads the slabs its own dW tasks wrote: the rest are zeros)
      AdamArgs a = critic_adam(p, 0, c.auto_alpha ? p.alpha() : nullptr);
      a.S = std::max(p.sp_q1.S, p.sp_ql.S);
      if (side_adam(p, gb, a, 2, off, n, true, s)) return 1;
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  return 0;
}

// phase 2: critic Adam + Polyak, policy gradient through the post-step critics
static int phase2_adam(SacPlan& p, hipStream_t s, int dp) {
  // SAC commits the alpha update here (no kernel after this reads next_*)
  AdamArgs a = critic_adam(p, dp ? -1 : 0, p.c.auto_alpha ? p.alpha() : nullptr);
  TIMED(p, K_ADAM, s, OAC_HIP_CHECK(launch_adam(a, s)));
  p.launches++;
  return 0;
}

// The small-batch step's policy-head dX (dh2 = dhead W_head (x) [h2 > 0], K =
// 2 Da) in the dL/da launch: that launch's head-backward tiles hold whole
// dhead rows, so each finishes dh2 for its rows, as MFMA tiles after the
// head backward (GemmTask::C2, gemm_small.hip HD2).  Each row block runs once
// per 64-column chunk of the hidden layer, the copies (dup) recomputing dL/da
// and storing only their dh2 columns: four workgroups finish a row block's
// dh2 in parallel (one workgroup for all 256 columns spent ~1 us of MFMA
// issue alone).  The head
// dW, which then needs nothing the policy layer-1 backward produces, joins
// that launch: one launch fewer on the chain.
static bool head_dh2(const SacPlan& p, const float* prefetch) {
  // (at large batch it measured slower: B=4096, the dL/da launch's 128 row
  // blocks x 4 chunks 8.4 -> 16.7 us, the merged launch 17.1 us against 7.3 +
  // 14.4; 3,939 -> 3,888 steps/s, tools/r6s2/big.sh -- on by tuning value 2)
  const int v = tuning(OAC_TUNE_HEAD_DH2);
  return (p.cfg == 0 || (p.cfg == kCfgLargeBatch && v == 2)) && v != -1 && !prefetch &&
         p.c.act_dim <= 24 && p.c.hidden <= 6 * 64 && (v < 16 || p.c.hidden <= 6 * v);
}

// prefetch: batch of the next step (its critic-side forward rides on this
// step's policy-backward launches, small-batch path only), or null
static int phase2(SacPlan& p, hipStream_t s, bool fused, const float* prefetch = nullptr,
                  bool split = false, bool defer = false) {
  const oac_sac_config& c = p.c;
  const oac_sac_layout& L = p.L;
  const int B = c.batch, H = c.hidden, Do = c.obs_dim, Da = c.act_dim, RS = c.row_stride;
  const int Dq = Do + Da;
  float* X = p.X();
  const float* pol = p.b.params;
  const float* q1 = p.b.params + L.q1_base;
  const float* q2 = p.b.params + L.q2_base;
  const bool merged = fused && minq_merged(p);   // (then the critic layer-0 dW launch ran it)
  const bool dfr = defer && merged && !prefetch;
  const float* qa = dfr ? p.W(W_QSHADOW) : q1;   // critic 1's post-step layer 0 (critic 2: + q_size)
  const bool hd2 = head_dh2(p, prefetch);
  if (!merged) {  // -min Q backward to layer 1 with post-step weights, pre-step masks
    GemmBatch gb{};
    const float* const qs[2] = {q1, q2};
    add_minq_bwd(p, gb, qs);
    if (prefetch) add_critic_l0(p, gb, prefetch);
    if (split) {   // the critics' layer 0 (not read here; the dL/da launch reads it next)
      const long off[2] = {0, (long)L.q_size};
      const long n[2] = {(long)L.q_fc1_w, (long)L.q_fc1_w};
      AdamArgs a = critic_adam(p, 0, nullptr);
      a.S = p.sp_q0.S;
      if (side_adam(p, gb, a, 2, off, n, false, s)) return 1;
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  if (p.cfg == 0 || head_bwd_fused_big()) {  // dL/da through both critics' action columns + head backward, one launch (small kernel)
    GemmBatch gb{};
    GemmTask t = t_dx(p.W(W_DH1N1), H, B, H, qa + L.q_fc0_w + Do, Dq, Da, p.W(W_DHEAD), 2 * Da,
                      nullptr, 0);
    t.A2 = p.W(W_DH1N2); t.B2 = qa + L.q_size + L.q_fc0_w + Do; t.K2 = H;   // same leading dims
    t.epi = EPI_HEAD_BWD;
    t.ex[0] = p.W(OAC_WS_ACT1); t.ex[1] = p.W(W_STD1); t.ex[2] = p.W(W_U1);
    t.ex[3] = p.E1(); t.ex[4] = p.W(OAC_WS_HEAD1);
    t.ex[5] = c.auto_alpha ? &p.alpha()->alpha : nullptr;
    if (hd2) {   // the head-backward tiles, once per 64-column chunk of dh2
      const int tv = tuning(OAC_TUNE_HEAD_DH2);   // (a chunk width of 16 .. 128: A/B runs)
      const int cw = (tv >= 16 && tv <= 128 && tv % 16 == 0) ? tv : 64;
      for (int c0 = 0; c0 < H; c0 += cw) {
        GemmTask u = t;
        u.C2 = p.W(W_DH2P) + c0; u.ldc2 = H;
        u.aux = p.W(W_H2P) + c0; u.ld_aux = H;
        u.U = pol + L.pol_head_w + c0; u.ldu = H;
        u.R = std::min(cw, H - c0);
        u.dup = c0 > 0;
        add(gb, u);
      }
      p.trace |= OAC_TRACE_HEAD_DH2;
    } else {
      add(gb, t);
    }
    if (prefetch && merged) add_critic_l0(p, gb, prefetch);
    if (prefetch) add_target_l0(p, gb, prefetch);
    if (dfr) add(gb, critic_dw0(p, 1, 0, Do, false));   // critic 2's obs columns: gradient only
    if (run_gemm(p, gb, s)) return 1;
  } else {
    {  // to the action columns of layer 0
      GemmBatch gb{};
      add(gb, t_dx(p.W(W_DH1N1), H, B, H, q1 + L.q_fc0_w + Do, Dq, Da, p.W(W_DA1), Da, nullptr, 0));
      add(gb, t_dx(p.W(W_DH1N2), H, B, H, q2 + L.q_fc0_w + Do, Dq, Da, p.W(W_DA2), Da, nullptr, 0));
      if (run_gemm(p, gb, s)) return 1;
    }
    {
      PolicyHeadBwdArgs a;
      std::memset(&a, 0, sizeof(a));
      a.da1 = p.W(W_DA1); a.da2 = p.W(W_DA2); a.act = p.W(OAC_WS_ACT1); a.stdv = p.W(W_STD1);
      a.u = p.W(W_U1); a.eps = p.E1(); a.head = p.W(OAC_WS_HEAD1);
      a.alpha = c.auto_alpha ? p.alpha() : nullptr; a.B = B; a.act_dim = Da; a.dhead = p.W(W_DHEAD);
      TIMED(p, K_ROW, s, OAC_HIP_CHECK(launch_policy_head_backward(a, s)));
      p.launches++;
    }
  }
  {  // policy heads: dW_head slab, dh2 (hd2: the dL/da launch ran dh2, and
     // the head dW shares the policy layer-1 backward's launch)
    GemmBatch gb{};
    float* gp = grad_p(p);
    add(gb, t_dw(p.W(W_DHEAD), 2 * Da, 2 * Da, B, p.W(W_H2P), H, H, gp + L.pol_head_w,
                 gp + L.pol_head_b, L.pol_size, p.sp_ph));
    if (!hd2) {
      add(gb, t_dx(p.W(W_DHEAD), 2 * Da, B, 2 * Da, pol + L.pol_head_w, H, H, p.W(W_DH2P), H,
                   p.W(W_H2P), H));
      if (prefetch) add_critic_l1(p, gb);
      if (dfr) add_dw0_side_adam(p, gb);   // both critics' layer 0 (+ bias): Adam + Polyak
      if (run_gemm(p, gb, s)) return 1;
      gb = GemmBatch{};
    }
    // policy layer 1
    add(gb, t_dw(p.W(W_DH2P), H, H, B, p.W(W_H1P), H, H, gp + L.pol_fc1_w, gp + L.pol_fc1_b,
                 L.pol_size, p.sp_p1));
    add(gb, t_dx(p.W(W_DH2P), H, B, H, pol + L.pol_fc1_w, H, H, p.W(W_DH1P), H, p.W(W_H1P), H));
    if (hd2 && dfr) add_dw0_side_adam(p, gb);   // (after every task: they store gradients only)
    if (run_gemm(p, gb, s)) return 1;
  }
  {  // policy layer 0
    GemmBatch gb{};
    float* gp = grad_p(p);
    add(gb, t_dw(p.W(W_DH1P), H, H, B, X + c.off_obs, RS, Do, gp + L.pol_fc0_w, gp + L.pol_fc0_b,
                 L.pol_size, p.sp_p0));
    if (fused) {
      const long off[1] = {(long)L.pol_fc1_w};
      const long n[1] = {(long)(L.pol_size - L.pol_fc1_w)};
      fuse_adam(gb, policy_adam(p, 0, nullptr), 1, off, n);
    } else if (split) {   // the policy's layer 1 + heads (layer 0: the step's last launch)
      const long off[1] = {(long)L.pol_fc1_w};
      const long n[1] = {(long)(L.pol_size - L.pol_fc1_w)};
      AdamArgs a = policy_adam(p, 0, nullptr);
      a.S = std::max(p.sp_p1.S, p.sp_ph.S);
      if (side_adam(p, gb, a, 1, off, n, false, s)) return 1;
      // and layer 0's own Adam by its tiles' last arrivals (GemmBatch::la_adam),
      // when this launch runs on gemm_bwdp with the side workgroups attached
      // (gb.adam is then the policy group's; otherwise run_step launches it)
      if (p.la_now && gb.side_adam == 0) p.la_now = false;
      if (p.la_now) {
        p.trace |= OAC_TRACE_LA_ADAM;
        gb.la_adam = 1;
        gb.la_book = 1;   // (the side workgroups do none)
        gb.la_ticket = reinterpret_cast<unsigned*>(p.W(WS_TICKETS));
      }
    }
    if (run_gemm(p, gb, s)) return 1;
  }
  return 0;
}

// step i of an n-step sequence: the gather of steps [i, i + kXSlots) runs at
// slot 0 (one launch per kXSlots steps), step i uses slot i % kXSlots
static long c_batch_rows(const SacPlan& p) { return (long)p.c.batch * p.c.row_stride; }

static int run_step(SacPlan& p, int flags, hipStream_t s, int i = 0, int n = 1) {
  p.launches = 0;
  const bool fused = can_fuse_adam(p);
  if (fused) p.trace |= OAC_TRACE_FUSED;
  // the small-batch device-ring step in the drop-in step's form: its layer-0
  // launch reads the rows through the device index ring (side blocks copy the
  // batch and draw eps), no gather launch, no prefetch; same-box A/B against
  // the gather launch per 8 steps with the next step's critic forward inside
  // the policy backward: see DESIGN.md section 5
  p.ring_direct = p.cfg == 0 && !p.rows_direct && (flags & OAC_STEP_GATHER) &&
                  p.c.kind == OAC_KIND_SAC && p.b.ring_slots > 0 && tuning(OAC_TUNE_RING_DIRECT) >= 0;
  p.slot = p.ring_direct ? 0 : i % kXSlots;
  const int gather_n = p.ring_direct ? 1 : p.slot == 0 ? std::min(kXSlots, n - i) : 0;
  // steps after the first of a gather batch had their critic-side forward
  // issued inside the previous step's policy backward (small-batch path;
  // measured slower than deferring the layer-0 Adam: off unless tuned on)
  const bool ahead = !p.ring_direct && p.cfg == 0 && (flags & OAC_STEP_GATHER) &&
                     tuning(OAC_TUNE_RING_PREFETCH) > 0;
  if (phase0(p, flags, s, gather_n, ahead && p.slot > 0)) return 1;
  const bool split = !fused && split_adam_on(p);
  p.la_now = split && la_adam_on(p);
  const bool pf = ahead && i + 1 < n && p.slot + 1 < kXSlots;
  const bool defer = !pf;
  if (phase1(p, s, fused, 0, split, defer)) return 1;
  if (!fused && !split && phase2_adam(p, s, 0)) return 1;
  if (phase2(p, s, fused, pf ? p.W(OAC_WS_BATCH) + (long)(p.slot + 1) * c_batch_rows(p) : nullptr,
             split, defer))
    return 1;
  if (!fused && !p.la_now) {
    AdamArgs a = policy_adam(p, 0, nullptr);
    if (split) { a.n = p.L.pol_fc1_w; a.S = p.sp_p0.S; }   // layer 0; the rest ran beside the layer-0 dW
    TIMED(p, K_ADAM, s, OAC_HIP_CHECK(launch_adam(a, s)));
    p.launches++;
  }
  p.la_now = false;
  p.slot = 0;
  p.ring_direct = false;
  return 0;
}

static int step_phase(SacPlan& p, int phase, int flags, hipStream_t s) {
  // the launch index keys the device launch records (BatchCache): it counts
  // the launches of ONE step, so a phase-0 call starts it again
  if (phase == 0) p.launches = 0;
  if (p.c.kind == OAC_KIND_PARTICLE) return particle_step_phase(p, phase, flags, s);
  if (has_target_policy(p.c.kind)) return det_step_phase(p, phase, flags, s);
  switch (phase) {
    case 0: return phase0(p, flags, s);
    case 1:
    case 5:   // phase 1 without its first part (after phase 4)
      if (phase1(p, s, false, phase == 5 ? 2 : 0)) return 1;
      if (p.S_q > 1) {
        AdamArgs a = critic_adam(p, 1, nullptr);
        OAC_HIP_CHECK(launch_adam(a, s));
      }
      return 0;
    case 4:   // phase 1's fresh-action critic forward (needs no alpha)
      p.trace |= OAC_TRACE_SPLIT_PHASE1;
      return phase1(p, s, false, 1);
    case 2:
      if (phase2_adam(p, s, 1)) return 1;
      if (phase2(p, s, false)) return 1;
      if (p.S_p > 1) {
        AdamArgs a = policy_adam(p, 1, nullptr);
        OAC_HIP_CHECK(launch_adam(a, s));
      }
      return 0;
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


// The data-parallel step with the library's own exchanges (oac_sac_set_allreduce):
// phase 0, the alpha partials' all-reduce (beside phase 4 on the side stream
// with OAC_DP_OVERLAP, SAC), the rest of phase 1, the critic gradients'
// all-reduce, phase 2 (critic Adam with the averaged gradients, the policy
// gradient through the post-step critics), the policy gradients' all-reduce,
// phase 3 -- trainer/trainer.py:139-210's order with a whole-batch quantity
// exchanged at each point the single-GPU step needs one.  Direct
// launches on `s`: the exchanges are stream-ordered calls of the hook.
static bool dp_exchanges(const SacPlan& p) {
  return p.ar_fn && (p.c.world_size > 1 || (p.ar_flags & OAC_DP_FORCE));
}
static int exchange(SacPlan& p, float* buf, int64_t n, hipStream_t s) {
  g_err[0] = 0;
  if (p.ar_fn(p.ar_ctx, buf, n, s)) {
    if (!g_err[0]) set_error("data-parallel all-reduce hook failed (%lld floats)", (long long)n);
    return 1;
  }
  p.trace |= OAC_TRACE_EXCHANGE;
  return 0;
}
static int run_step_dp(SacPlan& p, int flags, hipStream_t s) {
  const oac_sac_config& c = p.c;
  p.launches = 0;
  p.slot = 0;
  if (step_phase(p, 0, flags, s)) return 1;
  if (c.auto_alpha) {
    float* part = p.W(OAC_WS_LOGP_PART);
    const int64_t np = (c.batch + 15) / 16;
    if ((p.ar_flags & OAC_DP_OVERLAP) && c.kind == OAC_KIND_SAC && p.side) {
      OAC_HIP_CHECK(hipEventRecord(p.ev_fork, s));
      OAC_HIP_CHECK(hipStreamWaitEvent(p.side, p.ev_fork, 0));
      if (exchange(p, part, np, p.side)) return 1;
      OAC_HIP_CHECK(hipEventRecord(p.ev_join, p.side));
      if (step_phase(p, 4, flags, s)) return 1;
      OAC_HIP_CHECK(hipStreamWaitEvent(s, p.ev_join, 0));
      if (step_phase(p, 5, flags, s)) return 1;
    } else {
      if (exchange(p, part, np, s)) return 1;
      if (step_phase(p, 1, flags, s)) return 1;
    }
  } else if (step_phase(p, 1, flags, s)) {
    return 1;
  }
  if (exchange(p, p.b.grads + p.L.q1_base, q_group(p), s)) return 1;
  if (step_phase(p, 2, flags, s)) return 1;
  if (exchange(p, p.b.grads, p_group(p), s)) return 1;
  return step_phase(p, 3, flags, s);
}

}  // namespace oac

using namespace oac;

struct oac_sac {
  SacPlan plan;
};

extern "C" {

const char* oac_last_error(void) { return g_err; }
int oac_abi_version(void) { return OAC_ABI_VERSION; }

int oac_tuning_set(int key, int value) {
  if (key < 0 || key >= OAC_TUNE_COUNT) { set_error("unknown tuning key %d", key); return 1; }
  g_tuning[key] = value;
  return 0;
}

static int validate(const oac_sac_config* c) {
  if (!c) { set_error("null config"); return 1; }
  if (c->kind != OAC_KIND_SAC && c->kind != OAC_KIND_PARTICLE && c->kind != OAC_KIND_GAUSS &&
      c->kind != OAC_KIND_PARTICLE_UB) {
    set_error("bad kind %d", c->kind);
    return 1;
  }
  if (c->kind == OAC_KIND_PARTICLE_UB &&
      (c->q_out < 2 || c->q_out > 16 || c->delta_index < 0 || c->delta_index >= c->q_out)) {
    set_error("particle critic: 2 <= q_out <= 16 particles, 0 <= delta_index < q_out");
    return 1;
  }
  if (c->kind == OAC_KIND_GAUSS && c->q_out != 2) {
    set_error("gaussian critic (share_layers): q_out == 2 (mean | log std)");
    return 1;
  }
  if (c->kind == OAC_KIND_SAC && c->q_out != 1) { set_error("SAC needs q_out == 1"); return 1; }
  if (c->kind == OAC_KIND_PARTICLE && (c->q_out < 1 || c->q_out > 16)) {
    set_error("particle critic: 1 <= q_out <= 16 heads");
    return 1;
  }
  if (c->obs_dim < 1 || c->act_dim < 1 || c->act_dim > 32 || c->hidden < 1 || c->batch < 1) {
    set_error("bad dims obs=%d act=%d hidden=%d batch=%d", c->obs_dim, c->act_dim, c->hidden, c->batch);
    return 1;
  }
  if (c->row_stride % 4 != 0) { set_error("row_stride must be a multiple of 4"); return 1; }
  if (c->world_size < 1) { set_error("world_size must be >= 1"); return 1; }
  if (c->gemm_cfg < -1 || c->gemm_cfg > 2) { set_error("gemm_cfg must be -1, 0, 1 or 2"); return 1; }
  if (c->off_act != c->off_obs + c->obs_dim) { set_error("row layout: act must follow obs"); return 1; }
  if (c->off_obs < 0 || c->off_next_obs + c->obs_dim > c->row_stride ||
      c->off_act + c->act_dim > c->row_stride || c->off_rew >= c->row_stride ||
      c->off_term >= c->row_stride) {
    set_error("row layout out of bounds");
    return 1;
  }
  return 0;
}

static void plan_splits(SacPlan& p) {
  const oac_sac_config& c = p.c;
  p.cfg = c.gemm_cfg >= 0 ? c.gemm_cfg : (c.batch >= 1024 ? kCfgLargeBatch : 0);
  const int tm = split_tile_m(p.cfg), tn = split_tile_n(p.cfg);
  auto tiles = [&](int M, int N) { return ((M + tm - 1) / tm) * ((N + tn - 1) / tn); };
  const int H = c.hidden, Dq = c.obs_dim + c.act_dim, Do = c.obs_dim, Da = c.act_dim;
  const int nq = (c.kind == OAC_KIND_SAC) ? 2 : 1;
  p.sp_q1 = choose_split(c.batch, nq * (tiles(H, H + 1) + tiles(c.q_out, H + 1)), p.cfg);
  p.sp_ql = p.sp_q1;
  p.sp_q0 = choose_split(c.batch, nq * tiles(H, Dq + 1), p.cfg);
  p.sp_ph = choose_split(c.batch, tiles(2 * Da, H + 1), p.cfg);
  p.sp_p1 = choose_split(c.batch, tiles(H, H + 1), p.cfg);
  p.sp_p0 = choose_split(c.batch, tiles(H, Do + 1), p.cfg);
  if (p.cfg == kCfgLargeBatch) {   // the large-batch dW products run on gemm_bwdp.hip
    auto t64 = [](int M, int Nx) { return ((M + 63) / 64) * ((Nx + 63) / 64); };
    p.sp_q1 = choose_split_pipe(c.batch, nq * (t64(H, H) + t64(c.q_out, H)));
    p.sp_ql = p.sp_q1;
    p.sp_q0 = choose_split_pipe(c.batch, nq * t64(H, Dq));
    // the particle trainer's K-output last-layer dW rides in the layer-0 dW
    // launch (particle_plan.hip, hidden % 4 == 0): the same chunks as the
    // layer-0 dW, so neither is that launch's tail (configs[4]: 16 splits of
    // 256 rows beside layer 0's 32 of 128 made it 13.5 us, the same 32: 9.9)
    if (c.kind == OAC_KIND_PARTICLE && (H & 3) == 0) p.sp_ql = p.sp_q0;
    // (the head dW rides with the short-K dh2 product: register-direct kernel, sp_ph as is)
    p.sp_p1 = choose_split_pipe(c.batch, t64(H, H));
    p.sp_p0 = choose_split_pipe(c.batch, t64(H, Do));
  }
  // forced split counts (OAC_TUNE_SPLITS_*; 0 = keep), tuning runs
  {
    const int v[5] = {tuning(OAC_TUNE_SPLITS_Q1), tuning(OAC_TUNE_SPLITS_Q0),
                      tuning(OAC_TUNE_SPLITS_PH), tuning(OAC_TUNE_SPLITS_P1),
                      tuning(OAC_TUNE_SPLITS_P0)};
    Split* sp[5] = {&p.sp_q1, &p.sp_q0, &p.sp_ph, &p.sp_p1, &p.sp_p0};
    const int bk = p.cfg == 0 ? 64 : 32;
    bool forced = false;
    for (int i = 0; i < 5; ++i)
      if (v[i] > 0) {
        int kc = (c.batch + v[i] - 1) / v[i];
        kc = ((kc + bk - 1) / bk) * bk;
        *sp[i] = Split{(c.batch + kc - 1) / kc, kc};
        forced = true;
      }
    if (forced) p.sp_ql = p.sp_q1;   // (only then: the plan's own sp_ql choice stands otherwise)
  }
  p.S_q = std::max(std::max(p.sp_q0.S, p.sp_q1.S), p.sp_ql.S);
  p.S_p = std::max(std::max(p.sp_p0.S, p.sp_p1.S), p.sp_ph.S);
}

int oac_sac_query_layout(const oac_sac_config* cfg, oac_sac_layout* out) {
  if (validate(cfg)) return 1;
  SacPlan p;
  p.c = *cfg;
  compute_layout(p.c, p.L);
  plan_splits(p);
  if (p.c.kind == OAC_KIND_PARTICLE) particle_layout_workspace(p);
  else if (has_target_policy(p.c.kind)) det_layout_workspace(p);
  else layout_workspace(p);
  *out = p.L;
  return 0;
}

int oac_sac_create(const oac_sac_config* cfg, const oac_sac_buffers* bufs, oac_sac** out) {
  if (validate(cfg)) return 1;
  if (!bufs || !out) { set_error("null buffers/out"); return 1; }
  oac_sac* h = new oac_sac();
  SacPlan& p = h->plan;
  p.c = *cfg;
  compute_layout(p.c, p.L);
  plan_splits(p);
  if (p.c.kind == OAC_KIND_PARTICLE) particle_layout_workspace(p);
  else if (has_target_policy(p.c.kind)) det_layout_workspace(p);
  else layout_workspace(p);
  p.b = *bufs;
  if (p.ws[W_QSHADOW].rows > 0 && p.b.workspace && p.b.params) {
    // the shadow's float4 copies also carry the segments' al4 padding back
    // into the parameters: start it as the parameters' own
    const size_t bytes = sizeof(float) * (size_t)p.L.n_critics * p.L.q_size;
    if (hipMemcpy(p.W(W_QSHADOW), p.b.params + p.L.q1_base, bytes, hipMemcpyDeviceToDevice) != hipSuccess) {
      set_error("shadow init: %s", hipGetErrorString(hipGetLastError()));
      delete h;
      return 1;
    }
  }
  *out = h;
  return 0;
}

int oac_sac_destroy(oac_sac* h) {
  if (!h) return 0;
  for (hipEvent_t e : h->plan.ev_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->plan.ring_ev) (void)hipEventDestroy(e);
  if (h->plan.exec) (void)hipGraphExecDestroy(h->plan.exec);
  if (h->plan.graph) (void)hipGraphDestroy(h->plan.graph);
  if (h->plan.cap_stream) (void)hipStreamDestroy(h->plan.cap_stream);
  if (h->plan.side) (void)hipStreamDestroy(h->plan.side);
  if (h->plan.ev_fork) (void)hipEventDestroy(h->plan.ev_fork);
  if (h->plan.ev_join) (void)hipEventDestroy(h->plan.ev_join);
  if (h->plan.owns_host_ring && h->plan.host_ring) (void)hipHostFree(h->plan.host_ring);
  delete h;
  return 0;
}

int oac_sac_step_n(oac_sac* h, int flags, int n_steps, void* stream) {
  if (!h) { set_error("null handle"); return 1; }
  SacPlan& p = h->plan;
  if (n_steps < 1 || n_steps > 1024) { set_error("n_steps %d out of range", n_steps); return 1; }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dp_exchanges(p)) {   // the data-parallel step, exchanges through the hook (direct launches)
    for (int i = 0; i < n_steps; ++i)
      if (run_step_dp(p, flags & ~OAC_STEP_USE_GRAPH, s)) return 1;
    return 0;
  }
  if (p.c.world_size > 1) {
    set_error("world_size > 1: attach an all-reduce hook (oac_sac_set_allreduce) or drive the "
              "step with oac_sac_step_phase");
    return 1;
  }
  auto steps = [&](int f) {
    for (int i = 0; i < n_steps; ++i) {
      const int rc = p.c.kind == OAC_KIND_PARTICLE ? particle_run_step(p, f, s)
                     : has_target_policy(p.c.kind) ? det_run_step(p, f, s)
                                                   : run_step(p, f, s, i, n_steps);
      if (rc) return rc;
    }
    return 0;
  };
  if (!(flags & OAC_STEP_USE_GRAPH) || p.timing) return steps(flags & ~OAC_STEP_USE_GRAPH);
  const int gflags = flags & ~OAC_STEP_USE_GRAPH;
  if (!p.exec || p.graph_flags != gflags || p.graph_n != n_steps) {
    if (p.exec) { (void)hipGraphExecDestroy(p.exec); p.exec = nullptr; }
    if (p.graph) { (void)hipGraphDestroy(p.graph); p.graph = nullptr; }
    // the step sequence is static (counters live on the device), so n
    // consecutive steps capture into one graph.  Captured on the plan's own
    // stream (the caller's may be the null stream, which cannot capture) and
    // launched on the caller's.
    if (!p.cap_stream) OAC_HIP_CHECK(hipStreamCreateWithFlags(&p.cap_stream, hipStreamNonBlocking));
    hipStream_t cs = p.cap_stream;
    OAC_HIP_CHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    const int rc = [&] {
      for (int i = 0; i < n_steps; ++i) {
        const int r = p.c.kind == OAC_KIND_PARTICLE ? particle_run_step(p, gflags, cs)
                      : has_target_policy(p.c.kind) ? det_run_step(p, gflags, cs)
                                                    : run_step(p, gflags, cs, i, n_steps);
        if (r) return r;
      }
      return 0;
    }();
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(cs, &g);
    if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
    if (e != hipSuccess) { set_error("hipStreamEndCapture: %s", hipGetErrorString(e)); return 1; }
    p.graph = g;
    OAC_HIP_CHECK(hipGraphInstantiate(&p.exec, p.graph, nullptr, nullptr, 0));
    p.graph_stream = s;
    p.graph_flags = gflags;
    p.graph_n = n_steps;
  }
  OAC_HIP_CHECK(hipGraphLaunch(p.exec, s));
  return 0;
}

int oac_sac_step(oac_sac* h, int flags, void* stream) { return oac_sac_step_n(h, flags, 1, stream); }

static constexpr int kRingChunk = 16;


int oac_sac_set_host_ring(oac_sac* h, int32_t* pinned_ring) {
  if (!h) { set_error("null handle"); return 1; }
  SacPlan& p = h->plan;
  if (!p.b.idx_ring || p.b.ring_slots < kRingChunk || p.b.ring_slots % kRingChunk) {
    set_error("host ring: the handle needs an idx_ring of a multiple of %d slots", kRingChunk);
    return 1;
  }
  const int nch = p.b.ring_slots / kRingChunk;
  while ((int)p.ring_ev.size() < nch) {
    hipEvent_t e;
    OAC_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    p.ring_ev.push_back(e);
  }
  p.ring_ev_set.assign(nch, 0);
  p.last_bc = -1;
  if (p.owns_host_ring && p.host_ring) (void)hipHostFree(p.host_ring);
  p.host_ring = nullptr;
  p.owns_host_ring = false;
  p.rows_direct = false;
  p.idx_host = false;
  if (!pinned_ring) {   // the plan's own host-coherent ring
    int32_t* r = nullptr;
    OAC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&r), sizeof(int32_t) * (size_t)p.b.ring_slots * p.c.batch,
                                hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(r, 0, sizeof(int32_t) * (size_t)p.b.ring_slots * p.c.batch);
    p.host_ring = r;
    p.owns_host_ring = true;
    // direct mode needs the small-batch kernel (cfg 0)
    p.rows_direct = p.cfg == 0 && !has_target_policy(p.c.kind) &&
                    p.c.kind != OAC_KIND_PARTICLE &&   // sac_plan's run_step / phase0 only
                    p.c.row_stride / 4 <= 64 * 4;      // a side wave's row copy (gemm_small.hip)
    // (a direct large-batch step's 768 layer-0 tiles would each read their
    // rows' indices across the host link: its slot is copied to the device
    // ring instead, one H2D copy ahead of the step)
    p.idx_host = !p.rows_direct && !big_direct_ok(p);
    // not direct (large batch): the copy path still stages through this ring
    if (p.exec) { (void)hipGraphExecDestroy(p.exec); p.exec = nullptr; }
    if (p.graph) { (void)hipGraphDestroy(p.graph); p.graph = nullptr; }
    return 0;
  }
  p.host_ring = pinned_ring;
  return 0;
}

int32_t* oac_sac_host_ring(oac_sac* h) { return h ? h->plan.host_ring : nullptr; }

// host_read: the step that follows reads the slot from the host ring (no H2D
// copy), else an H2D copy on the stream reads it.  Either way a slot's readers
// are enqueued on `stream` after its staging call, so the event recorded at
// the first staging call outside a chunk follows all of that chunk's readers;
// entering the chunk again (one lap later) waits for it.  A batch counter that
// does not advance by one (another path of the trainer stepped in between, or
// a restore) drains every reader enqueued so far: the slots are then all free.
// inline: the indices may also travel in the next direct step's layer-0 kernel
// arguments -- only for oac_sac_step_host_idx's own step, which follows at
// once (a public staging call may be followed by other stagings, or by a
// caller's graph that never clears the flag; those read the host slot)
static int stage_host_idx(oac_sac* h, const int64_t* idx, int64_t bc, void* stream, bool host_read,
                          bool inline_ok = false) {
  if (!h) { set_error("null handle"); return 1; }
  SacPlan& p = h->plan;
  if (!p.host_ring) { set_error("oac_sac_set_host_ring first"); return 1; }
  if (bc < 0) { set_error("bad batch counter %lld", (long long)bc); return 1; }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int B = p.c.batch, S = p.b.ring_slots, nch = S / kRingChunk;
  const int slot = (int)(bc % S);
  const int64_t chunk = bc / kRingChunk;   // absolute: a wrap onto the same slots is a new chunk
  const int ch = (int)(chunk % nch);
  if (p.last_bc >= 0) {
    const int64_t last_chunk = p.last_bc / kRingChunk;
    const int lch = (int)(last_chunk % nch);
    if (bc != p.last_bc + 1) {
      OAC_HIP_CHECK(hipEventRecord(p.ring_ev[lch], s));
      OAC_HIP_CHECK(hipEventSynchronize(p.ring_ev[lch]));
      std::fill(p.ring_ev_set.begin(), p.ring_ev_set.end(), 0);
    } else if (chunk != last_chunk) {
      OAC_HIP_CHECK(hipEventRecord(p.ring_ev[lch], s));
      p.ring_ev_set[lch] = 1;
    }
    if (chunk != last_chunk && p.ring_ev_set[ch]) {
      OAC_HIP_CHECK(hipEventSynchronize(p.ring_ev[ch]));
      p.ring_ev_set[ch] = 0;
    }
  }
  p.last_bc = bc;
  int32_t* dst = p.host_ring + (long)slot * B;
  const int64_t rows = p.b.replay_rows;
  for (int i = 0; i < B; ++i) {
    const int64_t v = idx[i];
    if (v < 0 || v >= rows) {   // the gather would read outside the replay
      set_error("index %lld of step %lld outside the replay [0, %lld)", (long long)v,
                (long long)bc, (long long)rows);
      return 1;
    }
    dst[i] = (int32_t)v;
  }
  p.inline_ok = false;
  if (inline_ok && p.rows_direct && B <= kInlineRows) {   // the direct step passes them as kernel arguments
    std::memcpy(p.inline_rows, dst, sizeof(int32_t) * B);
    p.inline_ok = true;
  }
  if (host_read) return 0;   // the step's first launch reads the slot from host memory
  OAC_HIP_CHECK(hipMemcpyAsync(const_cast<int32_t*>(p.b.idx_ring) + (long)slot * B, dst,
                               sizeof(int32_t) * B, hipMemcpyHostToDevice, s));
  return 0;
}

int oac_sac_stage_host_idx(oac_sac* h, const int64_t* idx, int64_t bc, void* stream) {
  return stage_host_idx(h, idx, bc, stream, h && h->plan.rows_direct);
}

int oac_sac_set_step_graph(oac_sac* h, void* graph_exec, int flags) {
  if (!h) { set_error("null handle"); return 1; }
  h->plan.ext_exec = reinterpret_cast<hipGraphExec_t>(graph_exec);
  h->plan.ext_flags = (flags | OAC_STEP_GATHER) & ~OAC_STEP_USE_GRAPH;
  return 0;
}

int oac_sac_step_host_idx(oac_sac* h, const int64_t* idx, int64_t bc, int flags, void* stream) {
  if (!h) { set_error("null handle"); return 1; }
  SacPlan& p = h->plan;
  if (p.ext_exec) {   // the caller's captured step (phases + collectives)
    const int want = (flags | OAC_STEP_GATHER) & ~OAC_STEP_USE_GRAPH;
    if (want != p.ext_flags) {
      set_error("step flags %d differ from the flags %d the attached step graph was captured with",
                want, p.ext_flags);
      return 1;
    }
    if (stage_host_idx(h, idx, bc, stream, p.rows_direct)) return 1;
    OAC_HIP_CHECK(hipGraphLaunch(p.ext_exec, reinterpret_cast<hipStream_t>(stream)));
    return 0;
  }
  const bool hr = h->plan.idx_host;
  if (stage_host_idx(h, idx, bc, stream, hr || h->plan.rows_direct, true)) return 1;
  // the one-step drop-in call issues its launches directly: the same kernels
  // as the step graph, but one hipGraphLaunch per step cost more than the
  // host's 12 launch calls (same-box A/B, the bench line: B=256 10,443-10,491
  // -> 11,015-11,049 steps/s, B=4096 3,688-3,696 -> 3,740-3,749, configs[4]
  // 4,878-4,897 -> 5,028-5,035).
  return oac_sac_step_n(h, flags | OAC_STEP_GATHER | (hr ? kStepHostIdx : 0), 1, stream);
}

int oac_sac_step_phase(oac_sac* h, int phase, int flags, void* stream) {
  if (!h) { set_error("null handle"); return 1; }
  return step_phase(h->plan, phase, flags, reinterpret_cast<hipStream_t>(stream));
}

int oac_sac_set_allreduce(oac_sac* h, oac_allreduce_fn fn, void* ctx, int flags) {
  if (!h) { set_error("null handle"); return 1; }
  SacPlan& p = h->plan;
  if (fn && (flags & OAC_DP_OVERLAP) && !p.side) {
    OAC_HIP_CHECK(hipStreamCreateWithFlags(&p.side, hipStreamNonBlocking));
    OAC_HIP_CHECK(hipEventCreateWithFlags(&p.ev_fork, hipEventDisableTiming));
    OAC_HIP_CHECK(hipEventCreateWithFlags(&p.ev_join, hipEventDisableTiming));
  }
  p.ar_fn = fn;
  p.ar_ctx = fn ? ctx : nullptr;
  p.ar_flags = fn ? flags : 0;
  return 0;
}

int oac_sac_trace(oac_sac* h, int reset) {
  if (!h) { set_error("null handle"); return -1; }
  const int t = h->plan.trace;
  if (reset) h->plan.trace = 0;
  return t;
}

int oac_sac_workspace_view(oac_sac* h, int which, int64_t* offset, int64_t* rows, int64_t* cols) {
  if (!h || which < 0 || which >= OAC_WS_COUNT_PUBLIC) { set_error("bad workspace id"); return 1; }
  int id = which;
  if (which == OAC_WS_H2Q1 || which == OAC_WS_H2Q2)   // aliases of the SAC layout's buffers
    id = h->plan.c.kind == OAC_KIND_SAC ? (which == OAC_WS_H2Q1 ? W_H2Q1 : W_H2Q2) : which;
  // the policy's hidden layers on obs: the first two internal buffers of the
  // SAC and P-OAC layouts (W_H1P, W_H2P / X_H1P, X_H2P)
  if (which == OAC_WS_H1P || which == OAC_WS_H2P)
    id = (h->plan.c.kind == OAC_KIND_SAC || h->plan.c.kind == OAC_KIND_PARTICLE)
             ? (which == OAC_WS_H1P ? W_H1P : W_H2P) : which;
  const WsBuf& w = h->plan.ws[id];
  *offset = w.off; *rows = w.rows; *cols = w.cols;
  if (which == OAC_WS_BATCH || which == OAC_WS_EPS1 || which == OAC_WS_EPS2)
    *rows = h->plan.c.batch;   // slot 0: the batch / eps of a single-step call
  return 0;
}

int oac_sac_launch_count(oac_sac* h) { return h ? h->plan.launches : 0; }

int oac_sac_cache_stats(oac_sac* h, int64_t* out) {
  if (!h || !out) { set_error("null argument"); return 1; }
  const BatchCache& c = h->plan.bcache;
  out[0] = c.used; out[1] = (int64_t)c.at.size(); out[2] = c.hits; out[3] = c.misses;
  return 0;
}

int oac_sac_set_timing(oac_sac* h, int enable) {
  if (!h) { set_error("null handle"); return 1; }
  h->plan.timing = enable != 0;
  return 0;
}

int oac_sac_read_launch_times(oac_sac* h, double* ms, int* kinds, int max_n) {
  if (!h) { set_error("null handle"); return -1; }
  SacPlan& p = h->plan;
  int n = 0;
  for (auto& pr : p.ev_pending) {
    if (n >= max_n) break;
    float t = 0.f;
    OAC_HIP_CHECK(hipEventSynchronize(p.ev_pool[pr.second + 1]));
    OAC_HIP_CHECK(hipEventElapsedTime(&t, p.ev_pool[pr.second], p.ev_pool[pr.second + 1]));
    ms[n] = t;
    kinds[n] = pr.first;
    ++n;
  }
  return n;
}

int oac_sac_read_timing(oac_sac* h, double* ms_by_kind, int64_t* count_by_kind, int nkinds) {
  if (!h) { set_error("null handle"); return 1; }
  SacPlan& p = h->plan;
  for (auto& pr : p.ev_pending) {
    float ms = 0.f;
    OAC_HIP_CHECK(hipEventSynchronize(p.ev_pool[pr.second + 1]));
    OAC_HIP_CHECK(hipEventElapsedTime(&ms, p.ev_pool[pr.second], p.ev_pool[pr.second + 1]));
    p.kind_ms[pr.first] += ms;
    p.kind_count[pr.first] += 1;
  }
  p.ev_pending.clear();
  p.ev_next = 0;
  for (int k = 0; k < nkinds && k < OAC_NUM_KINDS; ++k) {
    ms_by_kind[k] = p.kind_ms[k];
    count_by_kind[k] = p.kind_count[k];
    p.kind_ms[k] = 0;
    p.kind_count[k] = 0;
  }
  return 0;
}

int oac_adam_polyak(float* p, const float* g, float* m, float* v, int64_t n, float* target,
                    float tau, int period, double lr, double beta1, double beta2, double eps,
                    void* step_state, int advance, void* stream) {
  AdamArgs a;
  std::memset(&a, 0, sizeof(a));
  a.p = p; a.g = const_cast<float*>(g); a.m = m; a.v = v; a.n = n;  // g is only read (S == 1)
  a.target = target; a.tau = tau; a.period = period;
  a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps;
  a.state = reinterpret_cast<StepState*>(step_state); a.advance = advance; a.gscale = 1.f;
  a.gslab = a.g; a.S = 1; a.slab_stride = n;
  OAC_HIP_CHECK(launch_adam(a, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

int oac_mt_seed_host(uint32_t seed, uint32_t* st) {
  if (!st) { set_error("null state"); return 1; }
  st[0] = seed;
  for (int i = 1; i < 624; ++i) st[i] = 1812433253u * (st[i - 1] ^ (st[i - 1] >> 30)) + (uint32_t)i;
  st[624] = 624;
  return 0;
}

int oac_replay_sample_indices(uint32_t* mt_state_dev, uint64_t size, int count, int32_t* out,
                              void* stream) {
  if (size == 0 || size > (1ull << 32)) { set_error("size must be in [1, 2^32]"); return 1; }
  OAC_HIP_CHECK(launch_mt_randint(mt_state_dev, size, count, out, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

int oac_replay_insert(float* storage, int64_t row_stride, int64_t capacity, int64_t top, int n,
                      const double* obs, const double* act, const double* rew,
                      const double* next_obs, const uint8_t* term, int obs_dim, int act_dim,
                      int off_obs, int off_act, int off_rew, int off_term, int off_next_obs,
                      void* stream) {
  if (!storage || capacity < 1 || top < 0 || top >= capacity || n < 0 || n > capacity) {
    set_error("replay insert: bad storage / top / n");
    return 1;
  }
  if (off_obs + obs_dim > row_stride || off_act + act_dim > row_stride || off_rew >= row_stride ||
      off_term >= row_stride || off_next_obs + obs_dim > row_stride) {
    set_error("replay insert: row layout out of bounds");
    return 1;
  }
  ReplayInsertArgs a;
  a.storage = storage; a.row_stride = row_stride; a.capacity = capacity; a.top = top; a.n = n;
  a.obs = obs; a.act = act; a.rew = rew; a.next_obs = next_obs; a.term = term;
  a.obs_dim = obs_dim; a.act_dim = act_dim; a.off_obs = off_obs; a.off_act = off_act;
  a.off_rew = off_rew; a.off_term = off_term; a.off_next_obs = off_next_obs;
  OAC_HIP_CHECK(launch_replay_insert(a, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

int oac_replay_counts_update(int32_t* counts, int32_t* tags, const int32_t* idx, int B,
                             int32_t epoch, float* counts_out, void* stream) {
  if (!counts || !tags || !idx || B < 0) { set_error("counts update: null buffer"); return 1; }
  OAC_HIP_CHECK(launch_counts_update(counts, tags, idx, B, epoch, counts_out,
                                     reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

int64_t oac_replay_priority_scratch_doubles(int64_t size) { return prio_scratch_doubles(size); }

int oac_replay_priority_sample(const int32_t* counts, int64_t size, const double* u, int B,
                               double* scratch, int32_t* idx_out, void* stream) {
  if (size < 1 || size > 4096LL * 1024) { set_error("priority sample: size must be in [1, 4194304]"); return 1; }
  if (B < 1) return 0;
  OAC_HIP_CHECK(launch_priority_sample(counts, size, u, B, scratch, idx_out,
                                       reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

int oac_replay_gather(const float* replay, int64_t row_stride, const int32_t* idx, int B,
                      float* out, void* stream) {
  if (row_stride % 4) { set_error("row_stride must be a multiple of 4"); return 1; }
  GatherArgs g;
  std::memset(&g, 0, sizeof(g));
  g.replay = replay; g.row_stride = row_stride; g.idx = idx; g.ring_slots = 0; g.out = out; g.B = B;
  g.state = nullptr;  // no ring: the gather reads idx[0:B]
  OAC_HIP_CHECK(launch_gather(g, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

}  // extern "C"
