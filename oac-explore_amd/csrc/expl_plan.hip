// OAC optimistic exploration action on MI355X, for N observations at once
// (N = 1: the reference's per-step call; N > 1: one launch sequence for the
// observations of N parallel environments, each row exactly as alone):
// get_optimistic_exploration_action_stochastic
// (/root/reference/optimistic_exploration.py:14-109, trainer=None, two critics):
//   mu_T, std = policy(ob);  a = tanh(mu_T)
//   Q_UB = (Q1+Q2)/2 + beta_UB |Q1-Q2|/2 ;  g = dQ_UB/dmu_T  (through tanh)
//   mu_C = sqrt(2 delta) Sigma g / (sqrt(g^T Sigma g) + 1e-5), Sigma = std^2
//   action = tanh(mu_E + std * eps),  mu_E = mu_T + mu_C
// The critics and policy are read in place from the trainer's parameter arena,
// so the action always uses the current weights.  The launch sequence is
// captured into a hipGraph (one replay per environment step).
#include <cmath>
#include <cstring>

#include "../../include/oac_amd.h"
#include "kernels.h"
#include "oac_common.h"

namespace oac {

static inline int64_t a64(int64_t x) { return (x + 63) & ~int64_t(63); }

struct ExplPlan {
  int Do, Da, H, N = 1;
  const float* pol; const float* q1; const float* q2;
  float* ws;
  StepState* state;
  unsigned long long seed;
  oac_sac_layout L;
  // workspace offsets
  int64_t o_x, o_h1p, o_h2p, o_head, o_std, o_mut, o_h1q1, o_h1q2, o_h2q1, o_h2q2, o_q1, o_q2, o_w,
      o_dh1, o_dh2, o_da1, o_da2, o_grad, o_mue, o_act, o_cnt, total;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipStream_t gstream = nullptr;
  const float* g_eps = nullptr;
  float g_beta = NAN, g_delta = NAN;
};

static void expl_layout(ExplPlan& p) {
  int64_t o = 0;
  const int64_t N = p.N;
  auto take = [&](int64_t n) { int64_t r = o; o = a64(o + N * n); return r; };
  p.o_x = take(p.Do + p.Da);
  p.o_h1p = take(p.H); p.o_h2p = take(p.H); p.o_head = take(2 * p.Da);
  p.o_std = take(p.Da); p.o_mut = take(p.Da);
  p.o_h1q1 = take(p.H); p.o_h1q2 = take(p.H); p.o_h2q1 = take(p.H); p.o_h2q2 = take(p.H);
  p.o_q1 = take(1); p.o_q2 = take(1); p.o_w = take(2);
  p.o_dh1 = take(p.H); p.o_dh2 = take(p.H); p.o_da1 = take(p.Da); p.o_da2 = take(p.Da);
  p.o_grad = take(p.Da); p.o_mue = take(p.Da); p.o_act = take(p.Da);
  p.o_cnt = o; o = a64(o + 2);   // Philox counter snapshot (8 bytes)
  p.total = o + 64;              // tail pad: k-contiguous GEMM loads may read 7 floats past a row
}

static GemmTask e_task() {
  GemmTask t;
  std::memset(&t, 0, sizeof(t));
  t.ksplit = 1;
  return t;
}

// rows of x: M observations, row stride ldx
static GemmTask e_fwd(const float* x, long ldx, int M, int K, const float* W, long ldw, int N,
                      float* y, int epi, const float* bias) {
  GemmTask t = e_task();
  t.A = x; t.lda = ldx; t.a_kc = 1; t.B = W; t.ldb = ldw; t.b_kc = 1;
  t.C = y; t.ldc = N; t.M = M; t.N = N; t.K = K; t.epi = epi; t.bias = bias;
  return t;
}

static int e_run(GemmBatch& gb, hipStream_t s) {
  gemm_batch_finalize(gb, 0);
  OAC_HIP_CHECK(gemm_batch_launch(gb, 0, s));
  return 0;
}

static int expl_sequence(ExplPlan& p, const float* eps, float beta, float delta, hipStream_t s) {
  const int Do = p.Do, Da = p.Da, H = p.H, Dq = Do + Da, N = p.N;
  const oac_sac_layout& L = p.L;
  float* w = p.ws;
  {
    GemmBatch gb{};
    gb.t[gb.ntasks++] = e_fwd(w + p.o_x, Dq, N, Do, p.pol + L.pol_fc0_w, Do, H, w + p.o_h1p, EPI_BIAS_RELU, p.pol + L.pol_fc0_b);
    if (e_run(gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    gb.t[gb.ntasks++] = e_fwd(w + p.o_h1p, H, N, H, p.pol + L.pol_fc1_w, H, H, w + p.o_h2p, EPI_BIAS_RELU, p.pol + L.pol_fc1_b);
    if (e_run(gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    gb.t[gb.ntasks++] = e_fwd(w + p.o_h2p, H, N, H, p.pol + L.pol_head_w, H, 2 * Da, w + p.o_head, EPI_BIAS, p.pol + L.pol_head_b);
    if (e_run(gb, s)) return 1;
  }
  OacArgs a;
  std::memset(&a, 0, sizeof(a));
  a.head = w + p.o_head; a.xrow = w + p.o_x; a.stdv = w + p.o_std; a.mu_T = w + p.o_mut;
  a.q1 = w + p.o_q1; a.q2 = w + p.o_q2; a.w = w + p.o_w; a.da1 = w + p.o_da1; a.da2 = w + p.o_da2;
  a.eps = eps; a.grad = w + p.o_grad; a.mu_E = w + p.o_mue; a.action = w + p.o_act;
  a.state = p.state; a.counter = reinterpret_cast<long long*>(w + p.o_cnt);
  a.seed = p.seed; a.beta_UB = beta; a.sqrt_2delta = (float)std::sqrt(2.0 * (double)delta);
  a.obs_dim = Do; a.act_dim = Da; a.n = N;
  OAC_HIP_CHECK(launch_oac_prep(a, s));
  const float* qs[2] = {p.q1, p.q2};
  const int64_t h1[2] = {p.o_h1q1, p.o_h1q2}, h2[2] = {p.o_h2q1, p.o_h2q2}, qo[2] = {p.o_q1, p.o_q2};
  {
    GemmBatch gb{};
    for (int i = 0; i < 2; ++i)
      gb.t[gb.ntasks++] = e_fwd(w + p.o_x, Dq, N, Dq, qs[i] + L.q_fc0_w, Dq, H, w + h1[i], EPI_BIAS_RELU, qs[i] + L.q_fc0_b);
    if (e_run(gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    for (int i = 0; i < 2; ++i)
      gb.t[gb.ntasks++] = e_fwd(w + h1[i], H, N, H, qs[i] + L.q_fc1_w, H, H, w + h2[i], EPI_BIAS_RELU, qs[i] + L.q_fc1_b);
    if (e_run(gb, s)) return 1;
  }
  {
    GemmBatch gb{};
    for (int i = 0; i < 2; ++i)
      gb.t[gb.ntasks++] = e_fwd(w + h2[i], H, N, H, qs[i] + L.q_last_w, H, 1, w + qo[i], EPI_BIAS, qs[i] + L.q_last_b);
    if (e_run(gb, s)) return 1;
  }
  OAC_HIP_CHECK(launch_oac_seed(a, s));
  const int64_t dh[2] = {p.o_dh1, p.o_dh2}, da[2] = {p.o_da1, p.o_da2};
  {  // dQ_i/dh1 = (w_i * wl_i * [h2 > 0]) . W1_i  masked by h1 > 0
    GemmBatch gb{};
    for (int i = 0; i < 2; ++i) {
      GemmTask t = e_task();
      t.a_mode = A_RANK1_MASK; t.a_s = w + p.o_w + (long)i * N; t.a_v = qs[i] + L.q_last_w;
      t.a_mask = w + h2[i]; t.ld_mask = H; t.a_kc = 1;
      t.B = qs[i] + L.q_fc1_w; t.ldb = H; t.b_kc = 0;
      t.C = w + dh[i]; t.ldc = H; t.M = N; t.N = H; t.K = H;
      t.epi = EPI_MASK; t.aux = w + h1[i]; t.ld_aux = H;
      gb.t[gb.ntasks++] = t;
    }
    if (e_run(gb, s)) return 1;
  }
  {  // dQ_i/da = dh1_i . W0_i[:, Do:]
    GemmBatch gb{};
    for (int i = 0; i < 2; ++i) {
      GemmTask t = e_task();
      t.A = w + dh[i]; t.lda = H; t.a_kc = 1;
      t.B = qs[i] + L.q_fc0_w + Do; t.ldb = Dq; t.b_kc = 0;
      t.C = w + da[i]; t.ldc = Da; t.M = N; t.N = Da; t.K = H; t.epi = EPI_STORE;
      gb.t[gb.ntasks++] = t;
    }
    if (e_run(gb, s)) return 1;
  }
  OAC_HIP_CHECK(launch_oac_final(a, s));
  return 0;
}

}  // namespace oac

using namespace oac;

struct oac_expl {
  ExplPlan p;
};

extern "C" {

int64_t oac_expl_workspace_floats_batch(int n_obs, int obs_dim, int act_dim, int hidden) {
  ExplPlan p;
  p.Do = obs_dim; p.Da = act_dim; p.H = hidden; p.N = n_obs < 1 ? 1 : n_obs;
  expl_layout(p);
  return p.total;
}

int64_t oac_expl_workspace_floats(int obs_dim, int act_dim, int hidden) {
  return oac_expl_workspace_floats_batch(1, obs_dim, act_dim, hidden);
}

int oac_expl_create_batch(int n_obs, int obs_dim, int act_dim, int hidden, const float* policy,
                          const float* q1, const float* q2, float* workspace, void* step_state,
                          uint64_t seed, oac_expl** out) {
  if (!policy || !q1 || !q2 || !workspace || !step_state || !out) {
    set_error("oac_expl_create: null pointer");
    return 1;
  }
  if (act_dim < 1 || act_dim > 63) { set_error("act_dim must be in [1, 63]"); return 1; }
  if (n_obs < 1 || n_obs > 65536) { set_error("n_obs must be in [1, 65536]"); return 1; }
  oac_expl* h = new oac_expl();
  ExplPlan& p = h->p;
  p.Do = obs_dim; p.Da = act_dim; p.H = hidden; p.N = n_obs;
  p.pol = policy; p.q1 = q1; p.q2 = q2; p.ws = workspace;
  p.state = reinterpret_cast<StepState*>(step_state); p.seed = seed;
  oac_sac_config c;
  std::memset(&c, 0, sizeof(c));
  c.kind = OAC_KIND_SAC; c.obs_dim = obs_dim; c.act_dim = act_dim; c.hidden = hidden; c.q_out = 1;
  c.batch = 1; c.row_stride = ((2 * obs_dim + act_dim + 2 + 3) / 4) * 4;
  c.off_obs = 0; c.off_act = obs_dim; c.off_rew = obs_dim + act_dim; c.off_term = c.off_rew + 1;
  c.off_next_obs = c.off_term + 1; c.gemm_cfg = 0; c.world_size = 1;
  if (oac_sac_query_layout(&c, &p.L)) { delete h; return 1; }
  expl_layout(p);
  *out = h;
  return 0;
}

int oac_expl_create(int obs_dim, int act_dim, int hidden, const float* policy, const float* q1,
                    const float* q2, float* workspace, void* step_state, uint64_t seed,
                    oac_expl** out) {
  return oac_expl_create_batch(1, obs_dim, act_dim, hidden, policy, q1, q2, workspace, step_state,
                               seed, out);
}

int oac_expl_destroy(oac_expl* h) {
  if (!h) return 0;
  if (h->p.exec) (void)hipGraphExecDestroy(h->p.exec);
  if (h->p.graph) (void)hipGraphDestroy(h->p.graph);
  delete h;
  return 0;
}

float* oac_expl_obs_slot(oac_expl* h) { return h ? h->p.ws + h->p.o_x : nullptr; }

int oac_expl_action(oac_expl* h, const float* eps, float beta_UB, float delta, float* action,
                    float* mu_E, float* std_out, float* grad_out, void* stream) {
  if (!h) { set_error("null handle"); return 1; }
  ExplPlan& p = h->p;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool same = p.exec && p.gstream == s && p.g_eps == eps && p.g_beta == beta_UB &&
                    p.g_delta == delta;
  if (!same) {
    if (p.exec) { (void)hipGraphExecDestroy(p.exec); p.exec = nullptr; }
    if (p.graph) { (void)hipGraphDestroy(p.graph); p.graph = nullptr; }
    OAC_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    const int rc = expl_sequence(p, eps, beta_UB, delta, s);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s, &g);
    if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
    if (e != hipSuccess) { set_error("hipStreamEndCapture: %s", hipGetErrorString(e)); return 1; }
    p.graph = g;
    OAC_HIP_CHECK(hipGraphInstantiate(&p.exec, p.graph, nullptr, nullptr, 0));
    p.gstream = s; p.g_eps = eps; p.g_beta = beta_UB; p.g_delta = delta;
  }
  OAC_HIP_CHECK(hipGraphLaunch(p.exec, s));
  const size_t nb = sizeof(float) * p.Da * p.N;
  if (action) OAC_HIP_CHECK(hipMemcpyAsync(action, p.ws + p.o_act, nb, hipMemcpyDeviceToDevice, s));
  if (mu_E) OAC_HIP_CHECK(hipMemcpyAsync(mu_E, p.ws + p.o_mue, nb, hipMemcpyDeviceToDevice, s));
  if (std_out) OAC_HIP_CHECK(hipMemcpyAsync(std_out, p.ws + p.o_std, nb, hipMemcpyDeviceToDevice, s));
  if (grad_out) OAC_HIP_CHECK(hipMemcpyAsync(grad_out, p.ws + p.o_grad, nb, hipMemcpyDeviceToDevice, s));
  return 0;
}

}  // extern "C"
