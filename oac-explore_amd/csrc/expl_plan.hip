// OAC optimistic exploration action on MI355X, for N observations at once
// (N = 1: the reference's per-step call; N > 1: one launch for the
// observations of N parallel environments, each row bitwise as alone):
// get_optimistic_exploration_action_stochastic
// (/root/reference/optimistic_exploration.py:14-109, trainer=None, two critics):
//   mu_T, std = policy(ob);  a = tanh(mu_T)
//   Q_UB = (Q1+Q2)/2 + beta_UB |Q1-Q2|/2 ;  g = dQ_UB/dmu_T  (through tanh)
//   mu_C = sqrt(2 delta) Sigma g / (sqrt(g^T Sigma g) + 1e-5), Sigma = std^2
//   action = tanh(mu_E + std * eps),  mu_E = mu_T + mu_C
// The critics and policy are read in place from the trainer's parameter arena,
// so the action always uses the current weights.  The computation is one
// launch (expl_split.hip: a group of workgroups per observation).  Two ways to
// call it:
//   oac_expl_action      a captured hipGraph (with the observation upload and
//                        result download when pinned buffers are registered),
//                        replayed on the caller's stream;
//   oac_expl_action_now  the latency path: the kernel reads the observations
//                        from, and writes the results to, the plan's own
//                        host-coherent buffers, and the call returns when the
//                        kernel's completion word lands in host memory (no
//                        graph replay, no copies, no stream synchronisation).
#include <cmath>
#include <cstring>
#include <algorithm>
#include <cstdlib>

#include "../../include/oac_amd.h"
#include "kernels.h"
#include "oac_common.h"

namespace oac {

static inline int64_t a64(int64_t x) { return (x + 63) & ~int64_t(63); }

struct ExplPlan {
  int Do, Da, H, N = 1;
  int K = 1;   // critic heads: 1 with twin critics (q1, q2); K with one shared-layer critic (q2 null)
  int ub_index = -1;   // K heads: sorted-head upper bound (oac_expl_set_ub_index)
  const float* pol; const float* q1; const float* q2;
  float* ws;
  StepState* state;
  unsigned long long seed;
  oac_sac_layout L;
  // workspace offsets (floats): observation rows [N, Do + Da], outputs
  // [3][N][Da] (action | mu_E | std), dQ_UB/dmu_T [N, Da], ticket word
  int64_t o_x, o_out, o_grad, o_cnt, o_split, total;
  // optional pinned host staging (oac_expl_set_host_io): uploads / downloads
  // captured into the graph
  const float* host_obs = nullptr; float* host_out = nullptr;
  // oac_expl_action_now: host-coherent observation rows [N, Do + Da], results
  // [3][N][Da] and completion word (hipHostMalloc, allocated on first use)
  float* hc_obs = nullptr; float* hc_out = nullptr; unsigned* hc_done = nullptr;
  // single-observation calls: the outputs as tagged granules (ExplFusedArgs::tags)
  unsigned long long* hc_tag = nullptr;
  unsigned seq = 0;
  hipStream_t cap_stream = nullptr;   // graph capture (the graphs launch on the caller's stream)
  // captured call graphs by (eps slot, beta_UB, delta, ub_index): alternating
  // bounds on one handle (e.g. --trainer_UB and plain calls) replay their own
  // graph instead of re-capturing
  struct Graph {
    hipGraph_t g; hipGraphExec_t e;
    const float* eps; float beta, delta; int ub;
  };
  Graph graphs[4];
  int n_graphs = 0, next_evict = 0;
  void drop_graphs() {
    for (int i = 0; i < n_graphs; ++i) {
      (void)hipGraphExecDestroy(graphs[i].e);
      (void)hipGraphDestroy(graphs[i].g);
    }
    n_graphs = 0; next_evict = 0;
  }
};

static void expl_layout(ExplPlan& p) {
  int64_t o = 0;
  const int64_t N = p.N;
  auto take = [&](int64_t n) { int64_t r = o; o = a64(o + n); return r; };
  p.o_x = take(N * (p.Do + p.Da));
  p.o_out = take(3 * N * p.Da);
  p.o_grad = take(N * p.Da);
  p.o_cnt = take(2);
  // expl_split.hip: published vectors + hand-off counters of the groups of one launch
  p.o_split = take((int64_t)std::min(N, (int64_t)kExplRows) * expl_split_scratch_floats(p.H));
  p.total = o + 64;
}

static ExplFusedArgs expl_args(ExplPlan& p, const float* eps, float beta, float delta) {
  const oac_sac_layout& L = p.L;
  float* w = p.ws;
  ExplFusedArgs a;
  std::memset(&a, 0, sizeof(a));
  a.obs = w + p.o_x; a.ld_obs = p.Do + p.Da;
  a.pol = p.pol; a.q[0] = p.q1; a.q[1] = p.q2;
  a.p_fc0_w = L.pol_fc0_w; a.p_fc0_b = L.pol_fc0_b; a.p_fc1_w = L.pol_fc1_w;
  a.p_fc1_b = L.pol_fc1_b; a.p_head_w = L.pol_head_w; a.p_head_b = L.pol_head_b;
  a.q_fc0_w = L.q_fc0_w; a.q_fc0_b = L.q_fc0_b; a.q_fc1_w = L.q_fc1_w; a.q_fc1_b = L.q_fc1_b;
  a.q_last_w = L.q_last_w; a.q_last_b = L.q_last_b;
  a.Do = p.Do; a.Da = p.Da; a.H = p.H; a.n = p.N;
  a.nq = p.q2 ? 2 : 1; a.K = p.K;
  a.eps = eps; a.out = w + p.o_out; a.grad = w + p.o_grad;
  a.state = p.state; a.ticket = reinterpret_cast<unsigned*>(w + p.o_cnt);
  a.fail = reinterpret_cast<unsigned*>(w + p.o_cnt + 1);
  a.seed = p.seed; a.beta_UB = beta; a.sqrt_2delta = (float)std::sqrt(2.0 * (double)delta);
  a.ub_index = p.ub_index;
  return a;
}

static int expl_launch(ExplPlan& p, const ExplFusedArgs& a, hipStream_t s) {
  for (int row0 = 0; row0 < p.N; row0 += kExplRows)
    OAC_HIP_CHECK(launch_expl_split(a, row0, std::min(kExplRows, p.N - row0), p.ws + p.o_split, s));
  return 0;
}

static int expl_sequence(ExplPlan& p, const float* eps, float beta, float delta, hipStream_t s) {
  const int Do = p.Do, Da = p.Da, N = p.N;
  float* w = p.ws;
  if (p.host_obs)   // rows [N, Do + Da]: the caller's pinned copy of the observations
    OAC_HIP_CHECK(hipMemcpyAsync(w + p.o_x, p.host_obs, sizeof(float) * N * (Do + Da),
                                 hipMemcpyHostToDevice, s));
  const ExplFusedArgs a = expl_args(p, eps, beta, delta);
  if (expl_launch(p, a, s)) return 1;
  if (p.host_out)
    OAC_HIP_CHECK(hipMemcpyAsync(p.host_out, w + p.o_out, sizeof(float) * 3 * N * Da,
                                 hipMemcpyDeviceToHost, s));
  return 0;
}

static int expl_host_alloc(ExplPlan& p) {
  if (p.hc_obs) return 0;
  const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
  OAC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p.hc_obs),
                              sizeof(float) * (size_t)p.N * (p.Do + p.Da), fl));
  OAC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p.hc_out),
                              sizeof(float) * 3 * (size_t)p.N * p.Da, fl));
  OAC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p.hc_done), 64, fl));
  OAC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p.hc_tag),
                              sizeof(unsigned long long) * 3 * (size_t)p.N * p.Da, fl));
  std::memset(p.hc_tag, 0, sizeof(unsigned long long) * 3 * (size_t)p.N * p.Da);
  std::memset(p.hc_obs, 0, sizeof(float) * (size_t)p.N * (p.Do + p.Da));
  std::memset(p.hc_out, 0, sizeof(float) * 3 * (size_t)p.N * p.Da);
  *p.hc_done = p.seq;
  return 0;
}

static inline void cpu_relax() {
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
  __builtin_ia32_pause();
#endif
}

// spin on the completion word (bits 0-30: the call's sequence number, bit 31:
// a hand-off of the call timed out); every ~4k polls ask the stream whether it
// failed (or finished without writing the word)
static int expl_wait(ExplPlan& p, unsigned seq, hipStream_t s) {
  volatile unsigned* f = p.hc_done;
  unsigned polls = 0;
  while ((*f & 0x7fffffffu) != seq) {
    cpu_relax();
    if ((++polls & 4095) == 0) {
      const hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess && (*f & 0x7fffffffu) != seq) {
        set_error("exploration: the launch finished without its completion word");
        return 1;
      }
      if (e != hipSuccess && e != hipErrorNotReady) {
        set_error("exploration: %s", hipGetErrorString(e));
        return 1;
      }
    }
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  if (*f & 0x80000000u) {
    set_error("exploration: an in-launch hand-off timed out (the workgroups of an observation's "
              "group were not co-resident); the results are NaN");
    return 1;
  }
  return 0;
}

// the single-observation call's tagged granules: spin until every one carries
// this call's sequence number (8-byte granules arrive whole, in any order),
// then unpack the values into the float outputs
static int expl_wait_tags(ExplPlan& p, unsigned seq, hipStream_t s) {
  const int n = 3 * p.Da;
  volatile unsigned long long* g = p.hc_tag;
  unsigned polls = 0;
  for (int i = 0; i < n; ++i) {
    while (((unsigned)(g[i] >> 32) & 0x7fffffffu) != seq) {
      cpu_relax();
      if ((++polls & 4095) == 0) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess && ((unsigned)(g[i] >> 32) & 0x7fffffffu) != seq) {
          set_error("exploration: the launch finished without its outputs");
          return 1;
        }
        if (e != hipSuccess && e != hipErrorNotReady) {
          set_error("exploration: %s", hipGetErrorString(e));
          return 1;
        }
      }
    }
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  bool failed = false;
  for (int i = 0; i < n; ++i) {
    const unsigned long long w = g[i];
    failed |= (w >> 63) != 0;
    const unsigned bits = (unsigned)w;
    std::memcpy(p.hc_out + i, &bits, sizeof(float));
  }
  if (failed) {
    set_error("exploration: an in-launch hand-off timed out (the workgroups of an observation's "
              "group were not co-resident); the results are NaN");
    return 1;
  }
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
  if (expl_split_lds_bytes(obs_dim, act_dim, hidden) > 64 * 1024) {
    set_error("exploration: obs_dim + 4 * hidden too large for one workgroup's LDS");
    return 1;
  }
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

int oac_expl_create_shared(int n_obs, int obs_dim, int act_dim, int hidden, int K,
                           const float* policy, const float* q, float* workspace,
                           void* step_state, uint64_t seed, oac_expl** out) {
  if (!q) { set_error("oac_expl_create_shared: null critic"); return 1; }
  if (K < 2 || K > 16) { set_error("shared-layer critic: 2 <= K <= 16 heads"); return 1; }
  // the twin-critic constructor with the second critic absent, then the heads
  if (oac_expl_create_batch(n_obs, obs_dim, act_dim, hidden, policy, q, q, workspace, step_state,
                            seed, out))
    return 1;
  ExplPlan& p = (*out)->p;
  p.q2 = nullptr;
  p.K = K;
  oac_sac_config c;
  std::memset(&c, 0, sizeof(c));
  c.kind = OAC_KIND_PARTICLE; c.obs_dim = obs_dim; c.act_dim = act_dim; c.hidden = hidden;
  c.q_out = K; c.batch = 1; c.row_stride = ((2 * obs_dim + act_dim + 2 + 3) / 4) * 4;
  c.off_obs = 0; c.off_act = obs_dim; c.off_rew = obs_dim + act_dim; c.off_term = c.off_rew + 1;
  c.off_next_obs = c.off_term + 1; c.gemm_cfg = 0; c.world_size = 1;
  if (oac_sac_query_layout(&c, &p.L)) { oac_expl_destroy(*out); *out = nullptr; return 1; }
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
  h->p.drop_graphs();
  if (h->p.cap_stream) (void)hipStreamDestroy(h->p.cap_stream);
  if (h->p.hc_obs) (void)hipHostFree(h->p.hc_obs);
  if (h->p.hc_out) (void)hipHostFree(h->p.hc_out);
  if (h->p.hc_done) (void)hipHostFree(h->p.hc_done);
  if (h->p.hc_tag) (void)hipHostFree(h->p.hc_tag);
  delete h;
  return 0;
}

float* oac_expl_obs_slot(oac_expl* h) { return h ? h->p.ws + h->p.o_x : nullptr; }

int oac_expl_action(oac_expl* h, const float* eps, float beta_UB, float delta, float* action,
                    float* mu_E, float* std_out, float* grad_out, void* stream) {
  if (!h) { set_error("null handle"); return 1; }
  ExplPlan& p = h->p;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int gi = -1;
  for (int i = 0; i < p.n_graphs && gi < 0; ++i) {
    const ExplPlan::Graph& g = p.graphs[i];
    if (g.eps == eps && g.beta == beta_UB && g.delta == delta && g.ub == p.ub_index) gi = i;
  }
  if (gi < 0) {
    if (!p.cap_stream) OAC_HIP_CHECK(hipStreamCreateWithFlags(&p.cap_stream, hipStreamNonBlocking));
    OAC_HIP_CHECK(hipStreamBeginCapture(p.cap_stream, hipStreamCaptureModeThreadLocal));
    const int rc = expl_sequence(p, eps, beta_UB, delta, p.cap_stream);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(p.cap_stream, &g);
    if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
    if (e != hipSuccess) { set_error("hipStreamEndCapture: %s", hipGetErrorString(e)); return 1; }
    hipGraphExec_t ex = nullptr;
    const hipError_t ie = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    if (ie != hipSuccess) {
      (void)hipGraphDestroy(g);
      set_error("hipGraphInstantiate: %s", hipGetErrorString(ie));
      return 1;
    }
    if (p.n_graphs < 4) {
      gi = p.n_graphs++;
    } else {   // evict round-robin
      gi = p.next_evict;
      p.next_evict = (p.next_evict + 1) % 4;
      (void)hipGraphExecDestroy(p.graphs[gi].e);
      (void)hipGraphDestroy(p.graphs[gi].g);
    }
    p.graphs[gi] = ExplPlan::Graph{g, ex, eps, beta_UB, delta, p.ub_index};
  }
  OAC_HIP_CHECK(hipGraphLaunch(p.graphs[gi].e, s));
  const size_t nb = sizeof(float) * p.Da * p.N;
  const float* o = p.ws + p.o_out;
  if (action) OAC_HIP_CHECK(hipMemcpyAsync(action, o, nb, hipMemcpyDeviceToDevice, s));
  if (mu_E) OAC_HIP_CHECK(hipMemcpyAsync(mu_E, o + p.Da * p.N, nb, hipMemcpyDeviceToDevice, s));
  if (std_out) OAC_HIP_CHECK(hipMemcpyAsync(std_out, o + 2 * p.Da * p.N, nb, hipMemcpyDeviceToDevice, s));
  if (grad_out) OAC_HIP_CHECK(hipMemcpyAsync(grad_out, p.ws + p.o_grad, nb, hipMemcpyDeviceToDevice, s));
  return 0;
}

int oac_expl_host_staging(oac_expl* h, float** obs, float** out) {
  if (!h || !obs || !out) { set_error("oac_expl_host_staging: null pointer"); return 1; }
  if (expl_host_alloc(h->p)) return 1;
  *obs = h->p.hc_obs;
  *out = h->p.hc_out;
  return 0;
}

int oac_expl_action_now(oac_expl* h, const float* eps, float beta_UB, float delta, void* stream) {
  if (!h) { set_error("null handle"); return 1; }
  ExplPlan& p = h->p;
  if (expl_host_alloc(p)) return 1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  ExplFusedArgs a = expl_args(p, eps, beta_UB, delta);
  a.obs = p.hc_obs;
  a.out = p.hc_out;
  p.seq = (p.seq + 1) & 0x7fffffffu;   // bit 31 of the word is the failure flag
  if (p.seq == 0) p.seq = 1;           // 0 is the word's initial value
  a.done = p.hc_done;
  a.done_seq = p.seq;
  if (p.N == 1 && p.Do <= kExplObsArg) {   // one observation: it travels in the arguments,
    ExplObsArg o;                            // the outputs come back as tagged granules
    std::memcpy(o.v, p.hc_obs, sizeof(float) * p.Do);
    a.tags = p.hc_tag;
    OAC_HIP_CHECK(launch_expl_split_obs(a, o, p.ws + p.o_split, s));
    return expl_wait_tags(p, a.done_seq, s);
  }
  if (expl_launch(p, a, s)) return 1;
  return expl_wait(p, a.done_seq, s);
}

const float* oac_expl_outputs(oac_expl* h) { return h ? h->p.ws + h->p.o_out : nullptr; }

int oac_expl_set_ub_index(oac_expl* h, int index) {
  if (!h) { set_error("null handle"); return 1; }
  ExplPlan& p = h->p;
  if (index < -1 || index >= p.K || (index >= 0 && p.q2)) {
    set_error("ub index %d: needs a K-head handle and -1 <= index < K (K = %d)", index, p.K);
    return 1;
  }
  p.ub_index = index;   // selects (or captures) the call graph of this bound
  return 0;
}

int oac_expl_set_host_io(oac_expl* h, const float* host_obs, float* host_out) {
  if (!h) { set_error("null handle"); return 1; }
  ExplPlan& p = h->p;
  p.host_obs = host_obs; p.host_out = host_out;
  p.drop_graphs();   // re-capture with the new staging
  return 0;
}

}  // extern "C"
