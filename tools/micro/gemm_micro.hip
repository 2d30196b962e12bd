// Small-GEMM launch cost inside a hipGraph chain (the regime of the B=256
// step): per-launch time of 50 dependent launches of one stage's GemmBatch,
// by geometry, against an empty-kernel chain.  Build: tools/micro/Makefile.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "../../oac-explore_amd/csrc/plan_common.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

#include "../../oac-explore_amd/csrc/gemm_small.hip"   // one TU: the stage-clock symbol is visible here
namespace oac {
void set_error(const char*, ...) {}
thread_local ExtTiming g_ext_timing;
}
using namespace oac;

static float* dev_rand(size_t n) {
  std::vector<float> h(n + 64);
  for (auto& x : h) x = ((float)rand() / (float)RAND_MAX - 0.5f);
  float* d; CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  return d;
}
__global__ void k_empty() {}

// per-stage spans of one launch (gemm_small.hip built with -DOAC_STAGE_CLOCK)
static void stages(hipStream_t s, const GemmBatch& b) {
  CK(gemm_small_launch(b, s));
  CK(hipStreamSynchronize(s));
  const int n = std::min(b.total_tiles, 4096);
  std::vector<long long> c(n * 8);
  CK(hipMemcpyFromSymbol(c.data(), HIP_SYMBOL(g_gs_clock), n * 8 * 8));
  int khz = 0; CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const double us = 1e3 / khz;
  long long t0 = c[0], tend = 0;
  double d[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    t0 = std::min(t0, c[i * 8]);
    tend = std::max(tend, c[i * 8 + 4]);
    for (int k = 0; k < 4; ++k) d[k] += (c[i * 8 + k + 1] - c[i * 8 + k]) * us / n;
  }
  long long first_end = c[4];
  for (int i = 0; i < n; ++i) first_end = std::min(first_end, c[i * 8 + 4]);
  printf("    stages (avg per block, us): lookup %.2f  loads+mfma %.2f  lds-reduce %.2f  epilogue %.2f | "
         "first-entry->last-exit %.2f  first-entry->first-exit %.2f\n", d[0], d[1], d[2], d[3],
         (tend - t0) * us, (first_end - t0) * us);
}

static double chain_us(hipStream_t s, const GemmBatch* b, int n = 50) {
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < n; ++i) {
    if (b) CK(gemm_small_launch(*b, s));
    else hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s);
  }
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t c, d; CK(hipEventCreate(&c)); CK(hipEventCreate(&d));
  const int reps = 20;
  CK(hipEventRecord(c, s));
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(d, s)); CK(hipEventSynchronize(d));
  float ms; CK(hipEventElapsedTime(&ms, c, d));
  CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  return 1e3 * ms / (reps * n);
}

int main(int argc, char** argv) {
  hipStream_t s; CK(hipStreamCreate(&s));
  const int B = 256, H = 256, Do = 376, Dq = 393, RS = 772;
  float* X = dev_rand((size_t)B * RS);
  float* W0 = dev_rand((size_t)H * Dq);
  float* W1 = dev_rand((size_t)H * H);
  float* bias = dev_rand(H);
  float* h[8];
  for (auto& p : h) p = dev_rand((size_t)B * H);
  float* gw = dev_rand((size_t)4 * H * (Dq + 1));
  printf("empty-kernel chain: %.2f us/launch\n", chain_us(s, nullptr));
  struct Case { const char* name; int kind, ntasks; };
  const Case cases[] = {
    {"fwd 256x256 K=256 x1", 0, 1}, {"fwd 256x256 K=256 x4", 0, 4}, {"fwd 256x256 K=376 x6", 1, 6},
    {"dW 256x257 K=B=256 x2", 2, 2}, {"dX 256x256 K=256 x2 (mask)", 3, 2}, {"fwd 32x32 K=256 x1 (1 tile)", 4, 1},
    {"dW 256x257 x2 + fused Adam", 5, 2},
  };
  // fused-Adam operands for case 5 (the critic group layout: the dW tiles' gradient
  // addresses index p / m / v / target)
  const long ng = (long)4 * H * (H + 1);
  float* ap = dev_rand(ng); float* am = dev_rand(ng); float* at = dev_rand(ng);
  float* av = dev_rand(ng);
  StepState* st; CK(hipMalloc(&st, sizeof(StepState))); CK(hipMemset(st, 0, sizeof(StepState)));
  for (const Case& c : cases) {
    for (int nw : {0, 4, 8, 16}) for (int gpw : {0, 3, 5, 6}) {
      if (nw == 0 && gpw) continue;
      if (nw && !gpw) continue;
      if (nw == 16 && gpw == 6) continue;
      if (nw && nw < 16 && gpw == 3 && nw != 8 && nw != 4) continue;
      GemmBatch gb{};
      for (int i = 0; i < c.ntasks; ++i) {
        GemmTask t;
        switch (c.kind) {
          case 0: t = t_fwd(h[i], H, B, H, W1, H, H, h[4 + (i & 3)], H, EPI_BIAS_RELU, bias); break;
          case 1: t = t_fwd(X, RS, B, Do, W0, Dq, H, h[i], H, EPI_BIAS_RELU, bias); break;
          case 2: t = t_dw(h[i], H, H, B, h[2 + i], H, H, gw + (long)i * H * (H + 1), gw + (long)i * H * (H + 1) + H * H,
                           0, Split{1, B}); break;
          case 3: t = t_dx(h[i], H, B, H, W1, H, H, h[4 + i], H, h[2 + i], H); break;
          case 5: t = t_dw(h[i], H, H, B, h[2 + i], H, H, gw + (long)i * H * (H + 1), gw + (long)i * H * (H + 1) + H * H,
                           0, Split{1, B}); break;
          default: t = t_fwd(h[i], H, 32, H, W1, H, 32, h[4], H, EPI_BIAS_RELU, bias); break;
        }
        add(gb, t);
      }
      if (c.kind == 5) {   // v >= 0 (sqrt), the step's constants unpublished (computed per block)
        CK(hipMemset(av, 0, ng * 4));
        AdamArgs a{}; a.p = ap; a.g = gw; a.m = am; a.v = av; a.n = ng; a.gslab = gw; a.S = 1;
        a.slab_stride = ng; a.target = at; a.tau = 0.005f; a.period = 1;
        a.lr = 3e-4; a.beta1 = 0.9; a.beta2 = 0.999; a.eps = 1e-8; a.state = st; a.no_book = 1;
        gb.fuse_adam = 1; gb.adam = a; gb.nseg = 0;
      }
      gemm_small_finalize(gb);
      gb.force_nw = nw; gb.force_gpw = gpw;
      printf("%-30s tiles %4d nw %2d gpw %d : %6.2f us/launch\n", c.name, gb.total_tiles, nw, gpw, chain_us(s, &gb));
      if (nw == 0) stages(s, gb);
    }
  }
  return 0;
}
