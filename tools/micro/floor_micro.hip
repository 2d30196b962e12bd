// Kernel-duration floor on MI355X: what a launch costs before any real work.
// Each case is timed with hipExtLaunchKernelGGL start/stop events (the
// dispatch's own begin/end, as rocprofv3 reports it), averaged over reps.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

struct Big { long v[300]; };   // ~2.4 KB kernarg, like GemmBatch

__global__ void k_empty() {}
__global__ void k_big(Big b, float* out) {
  if (threadIdx.x == 0 && b.v[blockIdx.x % 300] == -12345) out[0] = 1.f;
}
__global__ void k_big_chain(Big b, float* out) {   // dependent kernarg reads
  long i = blockIdx.x % 8;
  for (int r = 0; r < 4; ++r) i = (b.v[i] + i) % 300;
  if (threadIdx.x == 0 && i == -1) out[0] = 1.f;
}
__global__ void k_copy(const float* in, float* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i] * 2.f;
}
__global__ void k_copy_chain(const float* in, float* out, int n) {   // 2 dependent loads
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { int j = (int)in[i] % n; out[i] = in[j < 0 ? 0 : j] * 2.f; }
}

__global__ void k_ptr(const Big* b, float* out) {   // the same struct, device-resident
  if (threadIdx.x == 0 && b->v[blockIdx.x % 300] == -12345) out[0] = 1.f;
}

// per-launch time of a chain of `n` launches captured into one hipGraph
template <typename F>
static void graphit(const char* name, F launch, hipStream_t s, int n = 100) {
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < n; ++i) launch();
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t c, d; CK(hipEventCreate(&c)); CK(hipEventCreate(&d));
  const int reps = 20;
  CK(hipEventRecord(c, s));
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(d, s)); CK(hipEventSynchronize(d));
  float ms; CK(hipEventElapsedTime(&ms, c, d));
  printf("graph %-38s %6.2f us/launch\n", name, 1e3 * ms / (reps * n));
}

template <typename F>
static void timeit(const char* name, F launch, hipStream_t s) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) launch(nullptr, nullptr);
  const int reps = 200;
  double tot = 0;
  for (int i = 0; i < reps; ++i) {
    launch(a, b);
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  hipEvent_t c, d; CK(hipEventCreate(&c)); CK(hipEventCreate(&d));
  CK(hipEventRecord(c, s));
  for (int i = 0; i < reps; ++i) launch(nullptr, nullptr);
  CK(hipEventRecord(d, s)); CK(hipEventSynchronize(d));
  float ms2; CK(hipEventElapsedTime(&ms2, c, d));
  printf("%-44s kernel %6.2f us   back-to-back %6.2f us/launch\n", name, 1e3 * tot / reps, 1e3 * ms2 / reps);
}

int main() {
  hipStream_t s; CK(hipStreamCreate(&s));
  Big big; for (int i = 0; i < 300; ++i) big.v[i] = i;
  float *in, *out; const int n = 1 << 20;
  CK(hipMalloc(&in, n * 4)); CK(hipMalloc(&out, n * 4)); CK(hipMemset(in, 0, n * 4));
  const char* e = getenv("HIP_FORCE_DEV_KERNARG");
  printf("HIP_FORCE_DEV_KERNARG=%s\n", e ? e : "(unset)");
  Big* dbig; CK(hipMalloc(&dbig, sizeof(Big)));
  CK(hipMemcpy(dbig, &big, sizeof(Big), hipMemcpyHostToDevice));
  for (int g : {1, 256, 512}) {
    char nm[96];
    snprintf(nm, 96, "empty %d x 256", g);
    graphit(nm, [&]() { hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, s); }, s);
    snprintf(nm, 96, "2.4KB kernarg %d x 256", g);
    graphit(nm, [&]() { hipLaunchKernelGGL(k_big, dim3(g), dim3(256), 0, s, big, out); }, s);
    snprintf(nm, 96, "device struct ptr %d x 256", g);
    graphit(nm, [&]() { hipLaunchKernelGGL(k_ptr, dim3(g), dim3(256), 0, s, (const Big*)dbig, out); }, s);
    snprintf(nm, 96, "copy 262144 floats");
    graphit(nm, [&]() { hipLaunchKernelGGL(k_copy, dim3(256), dim3(1024), 0, s, (const float*)in, out, 262144); }, s);
  }
  int grids[3] = {1, 256, 1024};
  for (int g : grids) for (int t : {64, 1024}) {
    char nm[96];
    snprintf(nm, 96, "empty grid %d x %d", g, t);
    timeit(nm, [&](hipEvent_t a, hipEvent_t b) { hipExtLaunchKernelGGL(k_empty, dim3(g), dim3(t), 0, s, a, b, 0); }, s);
    snprintf(nm, 96, "2.4KB kernarg grid %d x %d", g, t);
    timeit(nm, [&](hipEvent_t a, hipEvent_t b) { hipExtLaunchKernelGGL(k_big, dim3(g), dim3(t), 0, s, a, b, 0, big, out); }, s);
    snprintf(nm, 96, "2.4KB kernarg, 4 dep reads grid %d x %d", g, t);
    timeit(nm, [&](hipEvent_t a, hipEvent_t b) { hipExtLaunchKernelGGL(k_big_chain, dim3(g), dim3(t), 0, s, a, b, 0, big, out); }, s);
  }
  for (int m : {65536, 262144, 1 << 20}) {
    char nm[96];
    snprintf(nm, 96, "copy %d floats (1024-thr WGs)", m);
    timeit(nm, [&](hipEvent_t a, hipEvent_t b) { hipExtLaunchKernelGGL(k_copy, dim3(m / 1024), dim3(1024), 0, s, a, b, 0, (const float*)in, out, m); }, s);
    snprintf(nm, 96, "copy-chain %d floats", m);
    timeit(nm, [&](hipEvent_t a, hipEvent_t b) { hipExtLaunchKernelGGL(k_copy_chain, dim3(m / 1024), dim3(1024), 0, s, a, b, 0, (const float*)in, out, m); }, s);
  }
  return 0;
}
