// Persistent-kernel prototype for the B=256 critic branch:
// three dependent stages with the shapes of the step's critic launches --
//   S1 critic layer 1 on the fresh actions  (4 x fwd 256x256, K=256)
//   S2 critic backward layer 1               (2 x dW 256x257 K=B + 2 x dX 256x256 masked)
//   S3 critic backward layer 0               (2 x dW 256x394 K=B)
// run (a) as three launches per step in a hipGraph, and (b) as ONE persistent
// launch per step (256 workgroups of 1024 threads, one per CU) running the
// same gemm_small_block code per stage with a grid barrier between stages:
// flat (one counter) or two-level (8 groups by blockIdx % 8, the group's last
// arriver forwards to a top counter and releases its group).  Every barrier
// is the agent-scope release -> counter -> relaxed poll -> acquire form; the
// last workgroup to leave resets the counters for the next replay.
// Outputs of (a) and (b) are compared bitwise.
// Build: make -C tools/micro persist_micro; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include "../../oac-explore_amd/csrc/plan_common.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

#include "../../oac-explore_amd/csrc/gemm_small.hip"
namespace oac {
void set_error(const char*, ...) {}
thread_local ExtTiming g_ext_timing;
}
using namespace oac;

constexpr int kLine = 32;   // counters on separate 128-B lines (unsigned words)

__device__ __forceinline__ void drain_and_meet() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}
__device__ __forceinline__ void rel() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void acq() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ unsigned ld(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned add(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool spin_until(unsigned* p, unsigned target) {
  for (unsigned i = 0; ld(p) < target; ++i) {
    __builtin_amdgcn_s_sleep(1);
    if (i > (1u << 26)) return false;   // bounded: a stuck barrier gives up (results then differ)
  }
  return true;
}

// epoch e = 1, 2, ...: every workgroup has arrived e times when it returns
template <bool HIER>
__device__ void grid_sync(unsigned* bar, unsigned e) {
  drain_and_meet();
  if (threadIdx.x == 0) {
    rel();
    if (!HIER) {
      add(bar, 1u);
      spin_until(bar, e * gridDim.x);
    } else {
      const unsigned grp = blockIdx.x & 7, per = gridDim.x >> 3;
      unsigned* gc = bar + (1 + grp) * kLine;    // group arrivals
      unsigned* gg = bar + (9 + grp) * kLine;    // group generation
      unsigned* top = bar + 17 * kLine;
      if (add(gc, 1u) == e * per - 1) {          // the group's last arriver
        acq(); rel();
        add(top, 1u);
        spin_until(top, e * 8);
        acq(); rel();
        __hip_atomic_store(gg, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        spin_until(gg, e);
      }
    }
    acq();
  }
  __syncthreads();
}

template <int NW, int GPW, bool HIER>
__global__ void __launch_bounds__(64 * NW)
chain_kernel(const GemmBatch* bs, const GemmHead* hs, int nst, unsigned* bar) {
  __shared__ __attribute__((aligned(16))) float red[SmallLds<NW>::N];
  for (int st = 0; st < nst; ++st) {
    const GemmHead h = hs[st];
    const int grid = h.total_tiles + bs[st].adam_blocks;
    for (int vb = blockIdx.x; vb < grid; vb += gridDim.x) {
      gemm_small_block<NW, GPW>(vb, h.total_tiles, h.publish, h.tb1, h.tb2, h.tb3, h.tb4, h.tb5,
                                h.tb6, h.tb7, bs[st], red);
      __syncthreads();
    }
    if (st + 1 < nst) grid_sync<HIER>(bar, st + 1);
  }
  // exit: the last workgroup out resets every counter for the next replay
  drain_and_meet();
  if (threadIdx.x == 0) {
    unsigned* ex = bar + 18 * kLine;
    if (add(ex, 1u) == gridDim.x - 1) {
      for (int i = 0; i < 19; ++i) __hip_atomic_store(bar + i * kLine, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

static float* dev_rand(size_t n, unsigned seed) {
  std::vector<float> h(n + 64);
  srand(seed);
  for (auto& x : h) x = ((float)rand() / (float)RAND_MAX - 0.5f);
  float* d; CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  return d;
}

template <typename F>
static double per_step_us(hipStream_t s, F issue, int steps = 50) {
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < steps; ++i) issue();
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
  return 1e3 * ms / (reps * steps);
}

int main() {
  hipStream_t s; CK(hipStreamCreate(&s));
  const int B = 256, H = 256, Dq = 393, RS = 772;
  float* X = dev_rand((size_t)B * RS, 1);
  float* W1[2] = {dev_rand((size_t)H * H, 2), dev_rand((size_t)H * H, 3)};
  float* bias = dev_rand(H, 4);
  float* h1[4]; float* h2[4];
  for (int i = 0; i < 4; ++i) { h1[i] = dev_rand((size_t)B * H, 10 + i); h2[i] = dev_rand((size_t)B * H, 20 + i); }
  float* dq[2] = {dev_rand(B, 30), dev_rand(B, 31)};
  float* wl = dev_rand(H, 32);
  float* dh1[2] = {dev_rand((size_t)B * H, 40), dev_rand((size_t)B * H, 41)};
  const long gsz = (long)H * (Dq + 1) + (long)H * (H + 1) + 2 * H;
  float* gq = dev_rand(2 * gsz, 50);

  GemmBatch st[3];
  for (auto& b : st) std::memset(&b, 0, sizeof(b));
  for (int i = 0; i < 4; ++i)   // S1: critic layer 1 of four nets
    add(st[0], t_fwd(h1[i], H, B, H, W1[i & 1], H, H, h2[i], H, EPI_BIAS_RELU, bias));
  for (int i = 0; i < 2; ++i) {  // S2: dW1 (rank-1 seed through the layer-1 mask) + dh1
    float* g = gq + i * gsz;
    GemmTask t = t_dw(nullptr, 0, H, B, h1[i], H, H, g + (long)H * (Dq + 1), g + (long)H * (Dq + 1) + H * H, 0, Split{1, B});
    set_rank1(t, dq[i], wl, h2[i], H);
    add(st[1], t);
    GemmTask d = t_dx(nullptr, 0, B, H, W1[i], H, H, dh1[i], H, h1[i], H);
    set_rank1(d, dq[i], wl, h2[i], H);
    add(st[1], d);
  }
  for (int i = 0; i < 2; ++i) {  // S3: dW0 over [obs | act]
    float* g = gq + i * gsz;
    add(st[2], t_dw(dh1[i], H, H, B, X, RS, Dq, g, g + (long)H * Dq, 0, Split{1, B}));
  }
  for (auto& b : st) gemm_small_finalize(b);
  GemmHead hh[3];
  for (int i = 0; i < 3; ++i) hh[i] = gemm_head(st[i]);
  GemmBatch* d_st; GemmHead* d_hh; unsigned* bar;
  CK(hipMalloc(&d_st, sizeof(st))); CK(hipMalloc(&d_hh, sizeof(hh)));
  CK(hipMalloc(&bar, 19 * kLine * 4));
  CK(hipMemcpy(d_st, st, sizeof(st), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_hh, hh, sizeof(hh), hipMemcpyHostToDevice));
  CK(hipMemset(bar, 0, 19 * kLine * 4));
  printf("tiles per stage: %d %d %d\n", st[0].total_tiles, st[1].total_tiles, st[2].total_tiles);

  // the outputs of one step (for the bitwise comparison)
  auto snapshot = [&]() {
    std::vector<float> o;
    auto grab = [&](const float* p, size_t n) {
      size_t k = o.size(); o.resize(k + n);
      CK(hipMemcpy(o.data() + k, p, n * 4, hipMemcpyDeviceToHost));
    };
    for (int i = 0; i < 4; ++i) grab(h2[i], (size_t)B * H);
    for (int i = 0; i < 2; ++i) grab(dh1[i], (size_t)B * H);
    grab(gq, 2 * gsz);
    return o;
  };
  auto launches = [&](int nw) {
    for (int i = 0; i < 3; ++i) {
      GemmBatch b = st[i];
      b.force_nw = nw;
      CK(gemm_small_launch(b, s));
    }
  };
  auto persist = [&](bool hier) {
    if (hier) hipLaunchKernelGGL((chain_kernel<16, 4, true>), dim3(256), dim3(1024), 0, s, d_st, d_hh, 3, bar);
    else hipLaunchKernelGGL((chain_kernel<16, 4, false>), dim3(256), dim3(1024), 0, s, d_st, d_hh, 3, bar);
  };
  // reference: the same stages as separate launches with the persistent
  // kernel's geometry (16 waves: the same K split, so the same summation order)
  launches(16); CK(hipStreamSynchronize(s));
  const std::vector<float> ref = snapshot();
  for (int hier = 0; hier < 2; ++hier) {
    persist(hier); CK(hipStreamSynchronize(s));
    const std::vector<float> got = snapshot();
    size_t bad = 0;
    for (size_t i = 0; i < ref.size(); ++i) bad += std::memcmp(&ref[i], &got[i], 4) != 0;
    printf("persistent (%s barrier) vs 16-wave launches: %zu of %zu words differ\n", hier ? "two-level" : "flat",
           bad, ref.size());
  }
  printf("3 launches per step (default waves)      : %7.2f us/step\n", per_step_us(s, [&] { launches(0); }));
  printf("3 launches per step (16 waves)           : %7.2f us/step\n", per_step_us(s, [&] { launches(16); }));
  printf("1 persistent launch, flat barrier        : %7.2f us/step\n", per_step_us(s, [&] { persist(false); }));
  printf("1 persistent launch, two-level barrier   : %7.2f us/step\n", per_step_us(s, [&] { persist(true); }));
  // barrier cost alone: the same persistent launch with empty stages
  GemmBatch empty[3];
  for (auto& b : empty) { std::memset(&b, 0, sizeof(b)); gemm_small_finalize(b); }
  GemmHead eh[3];
  for (int i = 0; i < 3; ++i) eh[i] = gemm_head(empty[i]);
  CK(hipMemcpy(d_st, empty, sizeof(empty), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_hh, eh, sizeof(eh), hipMemcpyHostToDevice));
  printf("persistent, empty stages, flat barrier   : %7.2f us/step (2 barriers)\n",
         per_step_us(s, [&] { persist(false); }));
  printf("persistent, empty stages, two-level      : %7.2f us/step (2 barriers)\n",
         per_step_us(s, [&] { persist(true); }));
  return 0;
}
