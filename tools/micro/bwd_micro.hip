// Large-batch backward GEMM launches of the B=4096 SAC step (Humanoid dims:
// critic layer 1 dW + last-layer dW + rank-1-seeded dX, critic layer 0 dW,
// the -min Q dX pair, policy layer 1 dW + dX, policy layer 0 dW) through
// gemm_batch_launch on the LDS-DMA pipelined
// gemm_bwdp.hip (cfg 9 / 10 / 11 or OAC_BWDP_CFG): per-launch time and the
// largest norm-relative difference of every output.  Build: tools/micro/Makefile.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../oac-explore_amd/csrc/oac_common.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

#include "../../oac-explore_amd/csrc/kernels.h"
#ifdef OAC_PIPE_CLOCK
#include "../../oac-explore_amd/csrc/gemm_bwdp.hip"
#endif
using namespace oac;
#ifdef OAC_PIPE_CLOCK
#include "pipe_clock.h"
static void clocks(const GemmBatch& b0, int cfg, hipStream_t s) {
  GemmBatch b = b0;
  gemm_batch_finalize(b, cfg);
  CK(gemm_bwdp_launch(b, cfg, s));
  CK(hipStreamSynchronize(s));
  print_pipe_clocks(b.total_tiles);
}
#endif

static float* dev_rand(size_t n, unsigned seed, float lo = -0.5f) {
  std::vector<float> h(n + 64);
  srand(seed);
  for (auto& x : h) x = ((float)rand() / (float)RAND_MAX + lo);
  float* d; CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  return d;
}
struct Out { float* p; size_t n; };
static std::vector<Out> outs;
static float* buf(size_t n) {
  float* d; CK(hipMalloc(&d, (n + 64) * 4)); CK(hipMemset(d, 0, (n + 64) * 4));
  outs.push_back({d, n});
  return d;
}
static GemmTask task0() { GemmTask t; memset(&t, 0, sizeof(t)); t.ksplit = 1; return t; }
static GemmTask t_dx(const float* dY, long lddy, int M, int K, const float* W, long ldw, int N, float* C,
                     const float* mask) {
  GemmTask t = task0();
  t.A = dY; t.lda = lddy; t.a_kc = 1; t.B = W; t.ldb = ldw; t.C = C; t.ldc = N;
  t.M = M; t.N = N; t.K = K; t.epi = mask ? EPI_MASK : EPI_STORE; t.aux = mask; t.ld_aux = N;
  return t;
}
static GemmTask t_dw(const float* dY, long lddy, int M, int Bn, const float* X, long ldx, int Kin, int S) {
  GemmTask t = task0();
  int kc = (Bn + S - 1) / S; kc = (kc + 31) / 32 * 32; S = (Bn + kc - 1) / kc;
  const long slab = (long)M * (Kin + 1);
  float* g = buf(slab * S);
  t.A = dY; t.lda = lddy; t.B = X; t.ldb = ldx; t.b_ones = 1; t.M = M; t.N = Kin + 1; t.K = Bn;
  t.C = g; t.ldc = Kin; t.bias_grad = g + (long)M * Kin; t.epi = EPI_GRAD;
  t.ksplit = S; t.kchunk = kc; t.slab_stride = slab;
  return t;
}
static void rank1(GemmTask& t, const float* s, const float* v, const float* mask, long ldm) {
  t.a_mode = A_RANK1_MASK; t.a_s = s; t.a_v = v; t.a_mask = mask; t.ld_mask = ldm;
}

// OAC_MICRO_DEVREC=1: the launch records in device memory (kernels.h
// BatchCache), as the trainers' plans pass them (gemm_bwdp_kernel_dev)
static BatchCache g_bc;
static int g_pos = 0;
static const bool g_devrec = getenv("OAC_MICRO_DEVREC") != nullptr;
static double run(const GemmBatch& b0, int cfg, hipStream_t s, int reps) {
  GemmBatch b = b0;
  gemm_batch_finalize(b, cfg);
  const int pos = g_pos++;
  BatchCache* bc = g_devrec ? &g_bc : nullptr;
  CK(gemm_batch_launch(b, cfg, s, bc, pos));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) CK(gemm_batch_launch(b, cfg, s, bc, pos));
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3 * ms / reps;
}
static std::vector<std::vector<float>> snap() {
  std::vector<std::vector<float>> h;
  for (auto& x : outs) {
    std::vector<float> t(x.n);
    CK(hipMemcpy(t.data(), x.p, x.n * 4, hipMemcpyDeviceToHost));
    h.push_back(t);
    CK(hipMemset(x.p, 0, x.n * 4));
  }
  return h;
}

int main(int argc, char** argv) {
  const int cfg_new = argc > 1 ? atoi(argv[1]) : 9;
  const int cfg_ref = argc > 2 ? atoi(argv[2]) : 3;   // reference kernel (outputs and time)
  const int B = 4096, Do = 376, Da = 17, H = 256, Dq = Do + Da, RS = 772;
  hipStream_t s; CK(hipStreamCreate(&s));
  float* X = dev_rand((size_t)B * RS, 1);
  float* h1 = dev_rand((size_t)B * H, 2), *h2 = dev_rand((size_t)B * H, 3);
  float* dq = dev_rand(B, 4), *wl = dev_rand(H, 5), *W1 = dev_rand((size_t)H * H, 6);
  float* dh1 = dev_rand((size_t)B * H, 7), *dh2 = dev_rand((size_t)B * H, 8);
  std::vector<GemmBatch> bs;
  std::vector<const char*> names;
  std::vector<double> fl;
  {  // critic backward layer 1: dW (rank-1 seed), last-layer dW, dX (rank-1 seed, masked)
    GemmBatch g; memset(&g, 0, sizeof(g));
    for (int i = 0; i < 2; ++i) {
      GemmTask t = t_dw(nullptr, 0, H, B, h1, H, H, 16); rank1(t, dq, wl, h2, H); g.t[g.ntasks++] = t;
      g.t[g.ntasks++] = t_dw(dq, 1, 1, B, h2, H, H, 16);
      GemmTask d = t_dx(nullptr, 0, B, H, W1, H, H, buf((size_t)B * H), h1); rank1(d, dq, wl, h2, H);
      g.t[g.ntasks++] = d;
    }
    bs.push_back(g); names.push_back("critic bwd L1 (dW+dWlast+dX)x2");
    fl.push_back(2.0 * (2.0 * H * (H + 1) * B + 2.0 * (H + 1) * B + 2.0 * B * H * H));
  }
  {  // critic backward layer 0: dW over [obs | act]
    GemmBatch g; memset(&g, 0, sizeof(g));
    for (int i = 0; i < 2; ++i) g.t[g.ntasks++] = t_dw(dh1, H, H, B, X, RS, Dq, 19);
    bs.push_back(g); names.push_back("critic bwd L0 dW x2");
    fl.push_back(2.0 * 2.0 * H * (Dq + 1) * B);
  }
  {  // -min Q backward to layer 1: dX x2 (rank-1 seed, masked)
    GemmBatch g; memset(&g, 0, sizeof(g));
    for (int i = 0; i < 2; ++i) {
      GemmTask d = t_dx(nullptr, 0, B, H, W1, H, H, buf((size_t)B * H), h1); rank1(d, dq, wl, h2, H);
      g.t[g.ntasks++] = d;
    }
    bs.push_back(g); names.push_back("minQ dX x2");
    fl.push_back(2.0 * 2.0 * B * H * H);
  }
  {  // policy layer 1: dW + dX (masked)
    GemmBatch g; memset(&g, 0, sizeof(g));
    g.t[g.ntasks++] = t_dw(dh2, H, H, B, h1, H, H, 32);
    g.t[g.ntasks++] = t_dx(dh2, H, B, H, W1, H, H, buf((size_t)B * H), h1);
    bs.push_back(g); names.push_back("policy L1 dW + dX");
    fl.push_back(2.0 * H * (H + 1) * B + 2.0 * B * H * H);
  }
  {  // policy layer 0: dW over obs
    GemmBatch g; memset(&g, 0, sizeof(g));
    g.t[g.ntasks++] = t_dw(dh1, H, H, B, X, RS, Do, 32);
    bs.push_back(g); names.push_back("policy L0 dW");
    fl.push_back(2.0 * H * (Do + 1) * B);
  }
  {  // configs[4] (P-OAC, Ant dims, K = 10 heads): critic layer-0 dW over [obs | act]
     // beside the K-head last layer's dW (its 10 rows in one 64-row tile)
    const int Do4 = 111, Da4 = 8, K4 = 10, RS4 = 240;
    GemmBatch g; memset(&g, 0, sizeof(g));
    g.t[g.ntasks++] = t_dw(dh1, H, H, B, X, RS4, Do4 + Da4, 32);
    g.t[g.ntasks++] = t_dw(dh2, K4, K4, B, h2, H, H, 16);
    bs.push_back(g); names.push_back("poac L0 dW + K-head dW");
    fl.push_back(2.0 * H * (Do4 + Da4 + 1) * B + 2.0 * K4 * (H + 1) * B);
  }
  // concurrency probe: the critic layer-1 dW (rank-1 seeded, 16 K chunks)
  // alone at 1 / 2 / 3 / 4 copies = 256 / 512 / 768 / 1,024 workgroups, so
  // one launch fills 1 / 2 / 3 / 4 workgroups per CU: the per-stage cycles
  // show whether a stage is bound by the workgroup's own latency chain (flat)
  // or by a resource the co-resident workgroups share (growing with them)
  static char nm[8][48];
  for (int copies : {1, 2, 3, 4, 6, 8}) {
    GemmBatch g; memset(&g, 0, sizeof(g));
    for (int i = 0; i < copies; ++i) {
      GemmTask t = t_dw(nullptr, 0, H, B, h1, H, H, 16); rank1(t, dq, wl, h2, H); g.t[g.ntasks++] = t;
    }
    snprintf(nm[copies - 1], 48, "occupancy: dW1 x%d (%d wgs)", copies, 256 * copies);
    bs.push_back(g); names.push_back(nm[copies - 1]);   // (x6 / x8: 1.5 / 2 rounds)
    fl.push_back(copies * 2.0 * H * (H + 1) * B);
  }
  int bad = 0;
  for (size_t k = 0; k < bs.size(); ++k) {
    const double t5 = run(bs[k], cfg_ref, s, 30);
    auto r5 = snap();
    const double tn = run(bs[k], cfg_new, s, 30);
    auto rn = snap();
    double worst = 0;
    for (size_t o = 0; o < r5.size(); ++o) {
      double num = 0, den = 0;
      for (size_t i = 0; i < r5[o].size(); ++i) {
        const double d = (double)r5[o][i] - rn[o][i];
        num += d * d; den += (double)r5[o][i] * r5[o][i];
      }
      if (den > 0) worst = std::max(worst, std::sqrt(num / den));
    }
    printf("%-34s cfg%d %7.2f us (%5.1f TF)  cfg%d %7.2f us (%5.1f TF)  max rel diff %.2e\n", names[k],
           cfg_ref, t5, fl[k] / t5 * 1e-6, cfg_new, tn, fl[k] / tn * 1e-6, worst);
    bad += worst > 1e-5;
#ifdef OAC_PIPE_CLOCK
    clocks(bs[k], cfg_new, s);
    snap();
#endif
  }
  return bad ? 1 : 0;
}
