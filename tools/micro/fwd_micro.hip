// Large-batch forward GEMM launches of the B=4096 SAC step (Humanoid dims),
// run through gemm_batch_launch on the LDS-tiled kernel (cfg 1, gemm.hip; the
// small-batch kernel, cfg 0, for the batch with the width-1 head dot, which
// cfg 1 lacks) and the LDS-pipelined kernel (cfg 6, gemm_fwd.hip;
// OAC_FWD2_TILE selects its tile): outputs compared (bitwise count, and within
// 1e-5 relative), per-launch time averaged over back-to-back launches.  (The
// round-1 register-direct kernel, the reference here until round 5, is gone.)
// Build: tools/micro/Makefile (links the in-tree liboac_amd.so).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include "../../oac-explore_amd/csrc/oac_common.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

#include "../../oac-explore_amd/csrc/kernels.h"
#ifdef OAC_PIPE_CLOCK
// this TU's own gemm_fwd.hip, built with the per-stage clocks of wave 0
#include "../../oac-explore_amd/csrc/gemm_fwd.hip"
#include "pipe_clock.h"
#endif
using namespace oac;

#ifdef OAC_PIPE_CLOCK
// one clocked launch of the cfg-6 kernel: per-phase cycles averaged over workgroups
static void clocks(const GemmBatch& b0, hipStream_t s) {
  GemmBatch b = b0;
  gemm_batch_finalize(b, 6);
  CK(gemm_fwd_launch(b, 6, s));
  CK(hipStreamSynchronize(s));
  print_pipe_clocks(b.total_tiles);
}
#endif

static float* dev_rand(size_t n, unsigned seed) {
  std::vector<float> h(n + 64);
  srand(seed);
  for (auto& x : h) x = ((float)rand() / (float)RAND_MAX - 0.5f);
  float* d; CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  return d;
}
static float* dev_zero(size_t n) {
  float* d; CK(hipMalloc(&d, (n + 64) * 4)); CK(hipMemset(d, 0, (n + 64) * 4)); return d;
}

static GemmTask fwd(const float* A, long lda, int M, int K, const float* W, long ldw, int N, float* C,
                    long ldc, int epi, const float* bias) {
  GemmTask t; memset(&t, 0, sizeof(t));
  t.A = A; t.lda = lda; t.M = M; t.K = K; t.B = W; t.ldb = ldw; t.N = N; t.C = C; t.ldc = ldc;
  t.epi = epi; t.bias = bias; t.a_kc = 1; t.b_kc = 1; t.ksplit = 1;
  return t;
}

struct Out { float* p; size_t n; };

static double run(const GemmBatch& b0, int cfg, hipStream_t s, int reps) {
  GemmBatch b = b0;
  gemm_batch_finalize(b, cfg);
  CK(gemm_batch_launch(b, cfg, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) CK(gemm_batch_launch(b, cfg, s));
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3 * ms / reps;
}

static std::vector<float> snap(const std::vector<Out>& o) {
  std::vector<float> h;
  for (auto& x : o) {
    std::vector<float> t(x.n);
    CK(hipMemcpy(t.data(), x.p, x.n * 4, hipMemcpyDeviceToHost));
    h.insert(h.end(), t.begin(), t.end());
    CK(hipMemset(x.p, 0, x.n * 4));
  }
  return h;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 4096;
  const int Do = argc > 2 ? atoi(argv[2]) : 376, Da = argc > 3 ? atoi(argv[3]) : 17;
  const int H = argc > 4 ? atoi(argv[4]) : 256, Dq = Do + Da, RS = ((2 * Do + Da + 2 + 3) / 4) * 4;
  const int off_obs = 0, off_act = Do, off_next = Do + Da + 2;
  hipStream_t s; CK(hipStreamCreate(&s));
  float* X = dev_rand((size_t)B * RS, 1);
  float* Wp = dev_rand((size_t)H * Do, 2);
  float* bp = dev_rand(H, 3);
  float* Wq[4]; float* bq[4];
  for (int i = 0; i < 4; ++i) { Wq[i] = dev_rand((size_t)H * Dq, 10 + i); bq[i] = dev_rand(H, 20 + i); }
  float* W1[4]; float* b1[4]; float* wl[4];
  for (int i = 0; i < 4; ++i) {
    W1[i] = dev_rand((size_t)H * H, 30 + i); b1[i] = dev_rand(H, 40 + i); wl[i] = dev_rand(H, 50 + i);
  }
  std::vector<Out> outs;
  auto buf = [&](size_t n) { float* p = dev_zero(n); outs.push_back({p, n}); return p; };
  // layer 0: policy(obs), policy(next_obs), Q1/Q2 [obs | act] (obs projection + rank-Da
  // continuation), TQ1/TQ2 on next_obs
  GemmBatch l0; memset(&l0, 0, sizeof(l0));
  float* h1p = buf((size_t)B * H); float* h1p2 = buf((size_t)B * H);
  l0.t[l0.ntasks++] = fwd(X + off_obs, RS, B, Do, Wp, Do, H, h1p, H, EPI_BIAS_RELU, bp);
  l0.t[l0.ntasks++] = fwd(X + off_next, RS, B, Do, Wp, Do, H, h1p2, H, EPI_BIAS_RELU, bp);
  for (int i = 0; i < 2; ++i) {
    GemmTask t = fwd(X + off_obs, RS, B, Do, Wq[i], Dq, H, buf((size_t)B * H), H, EPI_BIAS_RANK_RELU, bq[i]);
    t.U = X + off_act; t.ldu = RS; t.V = Wq[i] + Do; t.ldv = Dq; t.R = Da;
    t.C2 = buf((size_t)B * H); t.ldc2 = H;
    l0.t[l0.ntasks++] = t;
  }
  for (int i = 2; i < 4; ++i)
    l0.t[l0.ntasks++] = fwd(X + off_next, RS, B, Do, Wq[i], Dq, H, buf((size_t)B * H), H, EPI_BIAS, bq[i]);
  const size_t n0 = outs.size();
  // layer 1: four critics on their hidden layer, width-1 head partials in the epilogue
  GemmBatch l1; memset(&l1, 0, sizeof(l1));
  float* hin[4];
  for (int i = 0; i < 4; ++i) hin[i] = dev_rand((size_t)B * H, 60 + i);
  for (int i = 0; i < 4; ++i) {
    GemmTask t = fwd(hin[i], H, B, H, W1[i], H, H, buf((size_t)B * H), H, EPI_BIAS_RELU_DOT, b1[i]);
    t.aux = wl[i]; t.C2 = buf((size_t)B * ((H + 31) / 32)); t.ldc2 = B;
    l1.t[l1.ntasks++] = t;
  }
  // policy layer 1 (two tasks, plain ReLU)
  GemmBatch lp; memset(&lp, 0, sizeof(lp));
  lp.t[lp.ntasks++] = fwd(h1p, H, B, H, W1[0], H, H, buf((size_t)B * H), H, EPI_BIAS_RELU, b1[0]);
  lp.t[lp.ntasks++] = fwd(h1p2, H, B, H, W1[1], H, H, buf((size_t)B * H), H, EPI_BIAS_RELU, b1[1]);

  const double fl0 = 2.0 * B * H * (2.0 * Do + 2.0 * Dq + 2.0 * Do);
  const double fl1 = 2.0 * B * H * H * 4, flp = 2.0 * B * H * H * 2;
  const GemmBatch* bs[3] = {&l0, &l1, &lp};
  const double fls[3] = {fl0, fl1, flp};
  const char* names[3] = {"layer0 (6 tasks)", "critic layer1 + dot (4)", "policy layer1 (2)"};
  int bad = 0;
  for (int k = 0; k < 3; ++k) {
    // reference: cfg 1, or cfg 0 for the batch with the head dot; the layer-1
    // inputs of `lp` are l0's outputs, so run l0 first to give both kernels the
    // same inputs
    const int rc = k == 1 ? 0 : 1;
    if (k == 2) { GemmBatch b = l0; gemm_batch_finalize(b, 1); CK(gemm_batch_launch(b, 1, s)); CK(hipStreamSynchronize(s)); }
    const double t2 = run(*bs[k], rc, s, 50);
    std::vector<float> r2 = snap(outs);
    if (k == 2) { GemmBatch b = l0; gemm_batch_finalize(b, 1); CK(gemm_batch_launch(b, 1, s)); CK(hipStreamSynchronize(s)); }
    const double t6 = run(*bs[k], 6, s, 50);
    std::vector<float> r6 = snap(outs);
    size_t diff = 0, far = 0, first = (size_t)-1;
    for (size_t i = 0; i < r2.size(); ++i) {
      if (memcmp(&r2[i], &r6[i], 4) != 0) { if (first == (size_t)-1) first = i; ++diff; }
      if (!(std::fabs(r2[i] - r6[i]) <= 1e-5f * std::max(1.f, std::fabs(r2[i])))) ++far;
    }
    printf("%-26s cfg%d %7.2f us (%5.1f TF)  cfg6 %7.2f us (%5.1f TF)  bitwise-diff %zu/%zu, past 1e-5 %zu",
           names[k], rc, t2, fls[k] / t2 * 1e-6, t6, fls[k] / t6 * 1e-6, diff, r2.size(), far);
    if (diff) printf("  first @%zu: %.9g vs %.9g", first, r2[first], r6[first]);
    printf("\n");
    bad += far != 0;
#ifdef OAC_PIPE_CLOCK
    clocks(*bs[k], s);
    snap(outs);
#endif
  }
  (void)n0;
  return bad ? 1 : 0;
}
