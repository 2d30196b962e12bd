// Micro-benchmark of policy_head_kernel (csrc/head.hip) at Humanoid SAC sizes:
// average launch time over back-to-back launches and a per-stage wall-clock
// breakdown (head.hip built with -DOAC_STAGE_CLOCK).  Build: tools/micro/Makefile.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../oac-explore_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

namespace oac { void set_error(const char*, ...) {} thread_local ExtTiming g_ext_timing; }
using namespace oac;

static float* dev_rand(size_t n, float scale) {
  std::vector<float> h(n);
  for (auto& x : h) x = scale * ((float)rand() / RAND_MAX - 0.5f);
  float* d; CK(hipMalloc(&d, (n + 64) * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256, H = 256, Da = 17, Do = 376, Dq = Do + Da;
  const int cc = argc > 2 ? atoi(argv[2]) : 4;
  HeadArgs a{};
  a.wh = dev_rand(2 * Da * H, 0.1f); a.bh = dev_rand(2 * Da, 0.1f); a.ld_wa = Dq;
  a.B = B; a.H = H; a.Da = Da; a.col_chunks = cc;
  for (int s = 0; s < 2; ++s) {
    HeadSeg& g = a.seg[s];
    g.h2 = dev_rand((size_t)B * H, 1.f); g.eps = dev_rand((size_t)B * Da, 2.f);
    g.head = dev_rand((size_t)B * 2 * Da, 0); g.act = dev_rand((size_t)B * Da, 0);
    g.stdv = dev_rand((size_t)B * Da, 0); g.u = dev_rand((size_t)B * Da, 0); g.logp = dev_rand(B, 0);
    g.n_nets = 2;
    for (int i = 0; i < 2; ++i) {
      g.wa[i] = dev_rand((size_t)H * Dq, 0.1f); g.pre[i] = dev_rand((size_t)B * H, 1.f);
      g.h1[i] = dev_rand((size_t)B * H, 0);
    }
  }
  const int nblk = ((B + 15) / 16) * cc * 2;
  CK(hipMalloc(&a.stage_clock, nblk * 8 * sizeof(long long)));
  hipStream_t st; CK(hipStreamCreate(&st));
  for (int i = 0; i < 20; ++i) CK(launch_policy_head(a, 2, st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int reps = 200;
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) CK(launch_policy_head(a, 2, st));
  CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("policy_head B=%d cc=%d blocks=%d: %.2f us/launch (back-to-back)\n", B, cc, nblk, 1e3 * ms / reps);
  int khz = 0; CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const double us_per_tick = 1e3 / khz;
  std::vector<long long> clk(nblk * 8);
  CK(hipMemcpy(clk.data(), a.stage_clock, clk.size() * 8, hipMemcpyDeviceToHost));
  long long t0 = clk[0], tend = 0;
  double st_sum[5] = {0};
  for (int b = 0; b < nblk; ++b) {
    t0 = std::min(t0, clk[b * 8]);
    tend = std::max(tend, clk[b * 8 + 4]);
    for (int i = 1; i < 5; ++i) st_sum[i] += (clk[b * 8 + i] - clk[b * 8 + i - 1]) * us_per_tick;
  }
  double pf = 0;
  for (int b = 0; b < nblk; ++b) pf += (clk[b * 8 + 5] - clk[b * 8]) * us_per_tick;
  double hl = 0;
  for (int b = 0; b < nblk; ++b) hl += (clk[b * 8 + 6] - clk[b * 8 + 5]) * us_per_tick;
  printf("prefetch-drain %.2f us (from start), head-operand loads %.2f us after that\n", pf / nblk, hl / nblk);
  printf("stage means (us): heads %.2f  reduce %.2f  sample %.2f  critic-cols %.2f ; first start -> last end %.2f us\n",
         st_sum[1] / nblk, st_sum[2] / nblk, st_sum[3] / nblk, st_sum[4] / nblk, (tend - t0) * us_per_tick);
  return 0;
}
