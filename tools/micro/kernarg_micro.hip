// Where a launch's task record should live: a chain of small kernels (the
// B=256 step's shape: 11 dependent launches of 256 workgroups) whose waves
// first read a 304-byte record -- the GemmTask size -- and then one operand
// through a pointer taken from it.  (a) the record by value in the kernel
// arguments (written by the host for every launch, as the plans pass their
// GemmBatch today); (b) the same record in device memory written once, read
// through a pointer (held in a preloaded kernel argument).  Per-launch time
// from events around 1,000 chains, and the in-kernel clock from wave start to
// the record's arrival.
// usage: tools/micro/kernarg_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

struct Rec { const float* p[16]; long v[22]; };   // 304 bytes
static_assert(sizeof(Rec) == 304, "record size");

__device__ long long g_clk[2][256];

__global__ void __launch_bounds__(256) k_val(float* out, int idx, int rec_clk, const Rec r) {
  const long long t0 = __builtin_readcyclecounter();
  const float* src = r.p[idx & 15] + r.v[idx % 22];
  const long long t1 = __builtin_readcyclecounter();
  float x = src[threadIdx.x];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (rec_clk && threadIdx.x == 0) { g_clk[0][blockIdx.x] = t0; g_clk[1][blockIdx.x] = t1; }
}

__global__ void __launch_bounds__(256) k_ptr(float* out, int idx, int rec_clk, const Rec* __restrict__ rp) {
  const long long t0 = __builtin_readcyclecounter();
  const Rec& r = *rp;
  const float* src = r.p[idx & 15] + r.v[idx % 22];
  const long long t1 = __builtin_readcyclecounter();
  float x = ((const __attribute__((address_space(1))) float*)src)[threadIdx.x];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (rec_clk && threadIdx.x == 0) { g_clk[0][blockIdx.x] = t0; g_clk[1][blockIdx.x] = t1; }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  float *buf, *out;
  CK(hipMalloc(&buf, 64 << 20));
  CK(hipMalloc(&out, 256 * 256 * 4));
  CK(hipMemset(buf, 0, 64 << 20));
  Rec r;
  for (int i = 0; i < 16; ++i) r.p[i] = buf + (long)i * (1 << 20);
  for (int i = 0; i < 22; ++i) r.v[i] = i * 64;
  Rec* dr;
  CK(hipMalloc(&dr, sizeof(Rec) * 11));
  for (int i = 0; i < 11; ++i) CK(hipMemcpy(dr + i, &r, sizeof(Rec), hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int chains = 1000;
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      for (int w = 0; w < 50; ++w)
        for (int k = 0; k < 11; ++k) {
          if (mode == 0) k_val<<<256, 256, 0, s>>>(out, k, 0, r);
          else k_ptr<<<256, 256, 0, s>>>(out, k, 0, dr + k);
        }
      CK(hipEventRecord(e0, s));
      for (int c = 0; c < chains; ++c)
        for (int k = 0; k < 11; ++k) {
          if (mode == 0) k_val<<<256, 256, 0, s>>>(out, k, 0, r);
          else k_ptr<<<256, 256, 0, s>>>(out, k, 0, dr + k);
        }
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      // in-kernel: one clocked launch after a chain
      if (mode == 0) k_val<<<256, 256, 0, s>>>(out, 3, 1, r);
      else k_ptr<<<256, 256, 0, s>>>(out, 3, 1, dr + 3);
      CK(hipStreamSynchronize(s));
      long long c0[256], c1[256];
      CK(hipMemcpyFromSymbol(c0, HIP_SYMBOL(g_clk), sizeof(c0), 0));
      CK(hipMemcpyFromSymbol(c1, HIP_SYMBOL(g_clk), sizeof(c1), sizeof(c0)));
      std::vector<long long> d(256);
      for (int i = 0; i < 256; ++i) d[i] = c1[i] - c0[i];
      std::sort(d.begin(), d.end());
      printf("%s: %.3f us per launch (chains of 11, %d chains); record wait median %lld cycles, p90 %lld\n",
             mode == 0 ? "record in kernel arguments" : "record in device memory   ",
             1e3 * ms / (chains * 11), chains, d[128], d[230]);
    }
  }
  return 0;
}
