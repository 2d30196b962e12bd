// configs[4]'s single-product launches (one 4096 x 256 x 256 product: the
// target critic's / post-step critic's layer 1 forward, the post-step
// critic's dX into its first hidden layer) on every kernel that takes them:
// the per-launch time of back-to-back launches, and each output against the
// small kernel's within 1e-5.  usage: tools/micro/single_micro [B] [H]
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
using namespace oac;

static float* dev_rand(size_t n, unsigned seed) {
  std::vector<float> h(n + 64);
  srand(seed);
  for (auto& x : h) x = ((float)rand() / (float)RAND_MAX - 0.5f);
  float* d; CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  return d;
}

static double run(const GemmBatch& b0, int cfg, hipStream_t s, int reps) {
  GemmBatch b = b0;
  gemm_batch_finalize(b, cfg);
  hipError_t e = gemm_batch_launch(b, cfg, s);
  if (e != hipSuccess) return -1.0;
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) CK(gemm_batch_launch(b, cfg, s));
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3 * ms / reps;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 4096, H = argc > 2 ? atoi(argv[2]) : 256;
  hipStream_t s; CK(hipStreamCreate(&s));
  float* X = dev_rand((size_t)B * H, 1);
  float* W = dev_rand((size_t)H * H, 2);
  float* bias = dev_rand(H, 3);
  float* aux = dev_rand((size_t)B * H, 4);
  float* C; CK(hipMalloc(&C, (size_t)B * H * 4));
  const size_t n = (size_t)B * H;
  for (int kind = 0; kind < 2; ++kind) {
    GemmBatch b; memset(&b, 0, sizeof(b));
    GemmTask& t = b.t[0];
    t.A = X; t.lda = H; t.M = B; t.K = H; t.B = W; t.ldb = H; t.N = H; t.C = C; t.ldc = H; t.ksplit = 1;
    if (kind == 0) { t.a_kc = 1; t.b_kc = 1; t.epi = EPI_BIAS_RELU; t.bias = bias; }   // Y = relu(X W^T + b)
    else { t.a_kc = 1; t.b_kc = 0; t.epi = EPI_MASK; t.aux = aux; t.ld_aux = H; }      // dX = dY W, masked
    b.ntasks = 1;
    std::vector<float> ref(n), got(n);
    const int cfgs[2][6] = {{0, 1, 6, 7, 8, -1}, {0, 1, 9, 10, 11, 12}};
    for (int c : cfgs[kind]) {
      if (c < 0) continue;
      CK(hipMemset(C, 0, n * 4));
      const double us = run(b, c, s, 50);
      if (us < 0) { printf("%s cfg %2d: not taken\n", kind ? "dX " : "fwd", c); continue; }
      CK(hipMemcpy(got.data(), C, n * 4, hipMemcpyDeviceToHost));
      if (c == 0) ref = got;
      size_t far = 0;
      for (size_t i = 0; i < n; ++i)
        if (!(std::fabs(got[i] - ref[i]) <= 1e-5f * std::max(1.f, std::fabs(ref[i])))) ++far;
      printf("%s cfg %2d: %7.2f us/launch (%5.1f TF), past 1e-5 of cfg 0: %zu\n", kind ? "dX " : "fwd",
             c, us, 2.0 * B * H * H / us * 1e-6, far);
    }
  }
  return 0;
}
