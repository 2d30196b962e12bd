// Row-block DATAFLOW form of the B=256 critic branch,
// measured against the three launches it would replace:
//   S1 critic layer 1 on the fresh actions   4 x fwd 256x256, K=256  (256 tiles)
//   S2 critic backward layer 1               2 x dW1 256x257 + 2 x dh1 256x256 (272 tiles)
//   S3 critic backward layer 0               2 x dW0 256x394 (208 tiles)
// One launch of 256 workgroups (one per CU) runs the same gemm_small_block
// code per tile as the launches do, but instead of a grid barrier between
// stages each tile waits only for the tiles it reads:
//   dh1 tile (net i, row block m)     <- the 8 S1 tiles of (i, row block m)
//                                        (the ReLU mask / seed of its rows)
//   dW1 tile (net i, unit block n)    <- the 8 S1 tiles of (i, column block n)
//   dW0 tile (net i, unit block n')   <- the 8 dh1 tiles of (i, column block n')
// i.e. fan-ins of 8 producers per edge, counted on per-(net, block) counters
// (each on its own 128-byte line).  A producer drains its stores, meets its
// workgroup and adds 1 to each counter its tile feeds; a consumer's lane 0
// spins on its counter (relaxed, agent scope, bounded) and the workgroup
// meets again.  Two hand-off forms:
//   FENCE   activations in ordinary memory: agent-scope release before the
//           add, acquire after the spin (L2 write-back / invalidate: the
//           XCDs' L2s are not coherent with each other);
//   UNCACHED the handed-off activations (h2, dh1) in uncached device memory
//           (hipDeviceMallocUncached): stores and loads go past the L2s, so
//           the hand-off needs only the drain and the counter.
// PREFETCH (round 5): before a tile waits, each wave
// issues the loads of its first k-groups of the operand that is not handed
// off (B: W1 for dh1, h1 for dW1, the batch rows X for dW0) and keeps the
// values live, so the tile's own loads of those lines after the wait hit the
// CU's L1 instead of L2 / MALL -- the one overlap a launch boundary cannot
// have.
// Per-workgroup wall clocks (s_memrealtime, 100 MHz) at every stage edge give
// the edge waits; outputs are compared bitwise with the launches (the same
// 16-wave geometry, so the same summation order).  The last workgroup out
// resets the counters for the next replay.
// Build: make -C tools/micro dataflow_micro; run on the GPU box.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
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

constexpr int kLine = 32;        // counter stride (words): one 128-B line each
constexpr int kCounters = 81;    // C1rb[4][8] | C1ct[4][8] | C2ct[2][8] | exit
constexpr int kEdges = 7;        // clock marks per workgroup

struct TileDep { int wait, target, sig0, sig1; };   // counter ids (-1: none)

__device__ __forceinline__ unsigned ld(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add1(unsigned* p) {
  __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool FENCE>
__device__ __forceinline__ void wait_dep(unsigned* ctr, const TileDep& d) {
  if (d.wait >= 0 && threadIdx.x == 0) {
    unsigned* c = ctr + d.wait * kLine;
    const unsigned long long t0 = wall_clock64();
    while (ld(c) < (unsigned)d.target) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > 20000000ull) break;   // 0.2 s: a stuck edge gives up (outputs differ)
    }
    if constexpr (FENCE) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
}

template <bool FENCE>
__device__ __forceinline__ void signal_dep(unsigned* ctr, const TileDep& d) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && (d.sig0 >= 0 || d.sig1 >= 0)) {
    if constexpr (FENCE) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (d.sig0 >= 0) add1(ctr + d.sig0 * kLine);
    if (d.sig1 >= 0) add1(ctr + d.sig1 * kLine);
  }
}

// the loads k_loop will issue first for this tile's B operand (its first GPW
// k-groups per wave), summed into a register the caller keeps live
template <int NW, int GPW>
__device__ __forceinline__ float warm_b(int bid, const GemmHead& h, const GemmBatch& batch) {
  int ti = 0;
  ti = bid >= h.tb1 ? 1 : ti; ti = bid >= h.tb2 ? 2 : ti; ti = bid >= h.tb3 ? 3 : ti;
  ti = bid >= h.tb4 ? 4 : ti; ti = bid >= h.tb5 ? 5 : ti; ti = bid >= h.tb6 ? 6 : ti;
  ti = bid >= h.tb7 ? 7 : ti;
  ti = __builtin_amdgcn_readfirstlane(ti);
  const GemmTask& t = batch.t[ti];
  const int local = bid - t.tile_begin;   // (ksplit == 1 in this branch)
  const int n0 = (local % t.tiles_n) * 32;
  const int lane = threadIdx.x & 63, l32 = lane & 31, half = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g_hi = (t.K + 7) >> 3, kmax = t.K - 1;
  float s = 0.f, x[4], y[4];
  if (t.b_kc) {
    const Lane lb = lane_init<OP_KC>(n0 + l32, t.N, false, t.B, t.ldb, nullptr, nullptr);
#pragma unroll
    for (int j = 0; j < GPW; ++j)
      if (wave + j * NW < g_hi) {
        load4<OP_KC>(lb, 8 * (wave + j * NW) + 4 * half, kmax, x, y);
        s += (x[0] + x[1]) + (x[2] + x[3]);
      }
  } else {
    const Lane lb = lane_init<OP_MN>(n0 + l32, t.b_ones ? t.N - 1 : t.N, t.b_ones != 0, t.B, t.ldb,
                                     nullptr, nullptr);
#pragma unroll
    for (int j = 0; j < GPW; ++j)
      if (wave + j * NW < g_hi) {
        load4<OP_MN>(lb, 8 * (wave + j * NW) + 4 * half, kmax, x, y);
        s += (x[0] + x[1]) + (x[2] + x[3]);
      }
  }
  return s;
}

// the three stages' batches travel in the kernel arguments (as a launch's
// batch does): pointers loaded from the argument segment are known to be
// global, so the tiles' operand accesses are global loads -- from a batch in
// global memory they were flat loads (generic pointers), which also count
// against lgkmcnt and serialise with the LDS reduction
struct Stages { GemmBatch st[3]; GemmHead hh[3]; };

template <int NW, int GPW, bool FENCE, bool PF = false>
__global__ void __launch_bounds__(64 * NW)
dataflow_kernel(const Stages sg, const TileDep* __restrict__ deps, int nst,
                unsigned* ctr, unsigned long long* clk) {
  const GemmBatch* bs = sg.st;
  const GemmHead* hs = sg.hh;
  __shared__ __attribute__((aligned(16))) float red[SmallLds<NW>::N];
  unsigned long long* my = clk + (long)blockIdx.x * kEdges;
  if (threadIdx.x == 0) my[0] = wall_clock64();
  int off = 0, extra = 0;   // extra: workgroups [0, extra) took a second tile last stage
  for (int st = 0; st < nst; ++st) {
    const GemmHead h = hs[st];
    // this stage's tiles start past the workgroups still busy with a second
    // tile of the last stage (tile (w - extra) mod grid for workgroup w)
    const int w0 = ((int)blockIdx.x - extra + (int)gridDim.x) % (int)gridDim.x;
    for (int vb = w0; vb < h.total_tiles; vb += gridDim.x) {
      const TileDep d = deps[off + vb];
      float warm = 0.f;
      if (PF && d.wait >= 0) warm = warm_b<NW, GPW>(vb, h, bs[st]);
      wait_dep<FENCE>(ctr, d);
      asm volatile("" ::"v"(warm));
      if (threadIdx.x == 0 && vb == w0 && st > 0) my[2 * st] = wall_clock64();
      gemm_small_block<NW, GPW>(vb, h.total_tiles, h.publish, h.tb1, h.tb2, h.tb3, h.tb4, h.tb5,
                                h.tb6, h.tb7, bs[st], red);
      signal_dep<FENCE>(ctr, d);
    }
    if (threadIdx.x == 0) my[2 * st + 1] = wall_clock64();
    off += h.total_tiles;
    extra = h.total_tiles > (int)gridDim.x ? h.total_tiles - (int)gridDim.x : 0;
  }
  // exit: the last workgroup out resets every counter for the next replay
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* ex = ctr + (kCounters - 1) * kLine;
    if (__hip_atomic_fetch_add(ex, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1)
      for (int i = 0; i < kCounters; ++i)
        __hip_atomic_store(ctr + i * kLine, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static float* dev_rand(size_t n, unsigned seed, bool uncached = false) {
  std::vector<float> h(n + 64);
  srand(seed);
  for (auto& x : h) x = ((float)rand() / (float)RAND_MAX - 0.5f);
  float* d;
  if (uncached) CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&d), h.size() * 4, hipDeviceMallocUncached));
  else CK(hipMalloc(&d, h.size() * 4));
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

struct Branch {
  GemmBatch st[3];
  float *h2[4], *dh1[2], *gq;
  long gsz;
};

static Branch make_branch(bool uncached) {
  const int B = 256, H = 256, Dq = 393, RS = 772;
  Branch br;
  float* X = dev_rand((size_t)B * RS, 1);
  float* W1[2] = {dev_rand((size_t)H * H, 2), dev_rand((size_t)H * H, 3)};
  float* bias = dev_rand(H, 4);
  float* h1[4];
  for (int i = 0; i < 4; ++i) { h1[i] = dev_rand((size_t)B * H, 10 + i); br.h2[i] = dev_rand((size_t)B * H, 20 + i, uncached); }
  float* dq[2] = {dev_rand(B, 30), dev_rand(B, 31)};
  float* wl = dev_rand(H, 32);
  for (int i = 0; i < 2; ++i) br.dh1[i] = dev_rand((size_t)B * H, 40 + i, uncached);
  br.gsz = (long)H * (Dq + 1) + (long)H * (H + 1) + 2 * H;
  br.gq = dev_rand(2 * br.gsz, 50);
  for (auto& b : br.st) std::memset(&b, 0, sizeof(b));
  for (int i = 0; i < 4; ++i)   // S1: critic layer 1 of four nets
    add(br.st[0], t_fwd(h1[i], H, B, H, W1[i & 1], H, H, br.h2[i], H, EPI_BIAS_RELU, bias));
  // S2: dh1 of both nets first, then dW1 (rank-1 seeds through the layer-1
  // mask): the 16 tiles past one round (272 > 256 workgroups) are dW1 tiles,
  // which no later tile waits for
  for (int i = 0; i < 2; ++i) {
    GemmTask d = t_dx(nullptr, 0, B, H, W1[i], H, H, br.dh1[i], H, h1[i], H);
    set_rank1(d, dq[i], wl, br.h2[i], H);
    add(br.st[1], d);
  }
  for (int i = 0; i < 2; ++i) {
    float* g = br.gq + i * br.gsz;
    GemmTask t = t_dw(nullptr, 0, H, B, h1[i], H, H, g + (long)H * (Dq + 1), g + (long)H * (Dq + 1) + H * H, 0, Split{1, B});
    set_rank1(t, dq[i], wl, br.h2[i], H);
    add(br.st[1], t);
  }
  for (int i = 0; i < 2; ++i) {  // S3: dW0 over [obs | act]
    float* g = br.gq + i * br.gsz;
    add(br.st[2], t_dw(br.dh1[i], H, H, B, X, RS, Dq, g, g + (long)H * Dq, 0, Split{1, B}));
  }
  for (auto& b : br.st) gemm_small_finalize(b);
  return br;
}

// counters: C1rb(i, m) = i * 8 + m, C1ct(i, n) = 32 + i * 8 + n, C2ct(i, n) = 64 + i * 8 + n
static std::vector<TileDep> make_deps(const Branch& br) {
  std::vector<TileDep> dep;
  for (int s = 0; s < 3; ++s) {
    const GemmBatch& b = br.st[s];
    for (int ti = 0; ti < b.ntasks; ++ti) {
      const GemmTask& t = b.t[ti];
      const int tiles = ((t.M + 31) / 32) * t.tiles_n;
      for (int l = 0; l < tiles; ++l) {
        const int mb = l / t.tiles_n, nb = l % t.tiles_n;
        TileDep d{-1, 0, -1, -1};
        if (s == 0) {            // S1 net ti: rows mb, columns nb
          d.sig0 = ti * 8 + mb; d.sig1 = 32 + ti * 8 + nb;
        } else if (s == 1) {     // tasks dX(0), dX(1), dW(0), dW(1)
          const int i = ti & 1;
          if (ti >= 2) { d.wait = 32 + i * 8 + mb; d.target = 8; }   // dW1 units mb
          else { d.wait = i * 8 + mb; d.target = 8; d.sig0 = 64 + i * 8 + nb; }   // dh1 rows mb
        } else {                 // dW0 net ti, units mb
          d.wait = 64 + ti * 8 + mb; d.target = 8;
        }
        dep.push_back(d);
      }
    }
  }
  return dep;
}

int main() {
  hipStream_t s; CK(hipStreamCreate(&s));
  for (int form = 0; form < 2; ++form) {
    const bool uncached = form == 1;
    Branch br = make_branch(uncached);
    GemmHead hh[3];
    for (int i = 0; i < 3; ++i) hh[i] = gemm_head(br.st[i]);
    const std::vector<TileDep> dep = make_deps(br);
    GemmBatch* d_st; GemmHead* d_hh; TileDep* d_dep; unsigned* ctr; unsigned long long* clk;
    CK(hipMalloc(&d_st, sizeof(br.st))); CK(hipMalloc(&d_hh, sizeof(hh)));
    CK(hipMalloc(&d_dep, dep.size() * sizeof(TileDep)));
    CK(hipMalloc(&ctr, kCounters * kLine * 4)); CK(hipMalloc(&clk, 256 * kEdges * 8));
    CK(hipMemcpy(d_st, br.st, sizeof(br.st), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_hh, hh, sizeof(hh), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_dep, dep.data(), dep.size() * sizeof(TileDep), hipMemcpyHostToDevice));
    CK(hipMemset(ctr, 0, kCounters * kLine * 4));
    printf("== %s hand-off: tiles per stage %d %d %d\n", uncached ? "uncached-activation" : "fenced",
           br.st[0].total_tiles, br.st[1].total_tiles, br.st[2].total_tiles);
    auto snapshot = [&]() {
      std::vector<float> o;
      auto grab = [&](const float* p, size_t n) {
        size_t k = o.size(); o.resize(k + n);
        CK(hipMemcpy(o.data() + k, p, n * 4, hipMemcpyDeviceToHost));
      };
      for (int i = 0; i < 4; ++i) grab(br.h2[i], (size_t)256 * 256);
      for (int i = 0; i < 2; ++i) grab(br.dh1[i], (size_t)256 * 256);
      grab(br.gq, 2 * br.gsz);
      return o;
    };
    auto launches = [&](int nw) {
      for (int i = 0; i < 3; ++i) {
        GemmBatch b = br.st[i];
        b.force_nw = nw;
        CK(gemm_small_launch(b, s));
      }
    };
    Stages sg;
    for (int i = 0; i < 3; ++i) { sg.st[i] = br.st[i]; sg.hh[i] = hh[i]; }
    bool pf = false;
    auto dataflow = [&]() {
      if (uncached && pf)
        hipLaunchKernelGGL((dataflow_kernel<16, 4, false, true>), dim3(256), dim3(1024), 0, s, sg, d_dep, 3, ctr, clk);
      else if (uncached)
        hipLaunchKernelGGL((dataflow_kernel<16, 4, false>), dim3(256), dim3(1024), 0, s, sg, d_dep, 3, ctr, clk);
      else if (pf)
        hipLaunchKernelGGL((dataflow_kernel<16, 4, true, true>), dim3(256), dim3(1024), 0, s, sg, d_dep, 3, ctr, clk);
      else
        hipLaunchKernelGGL((dataflow_kernel<16, 4, true>), dim3(256), dim3(1024), 0, s, sg, d_dep, 3, ctr, clk);
      CK(hipGetLastError());
    };
    launches(16); CK(hipStreamSynchronize(s));
    const std::vector<float> ref = snapshot();
    for (int pass = 0; pass < 2; ++pass) {
    pf = pass == 1;
    printf("-- %s\n", pf ? "PREFETCH: non-handed-off operand loaded before the wait" : "no prefetch");
    dataflow(); CK(hipStreamSynchronize(s));
    const std::vector<float> got = snapshot();
    size_t bad = 0;
    for (size_t i = 0; i < ref.size(); ++i) bad += std::memcmp(&ref[i], &got[i], 4) != 0;
    printf("dataflow vs 16-wave launches: %zu of %zu words differ\n", bad, ref.size());
    // per-edge clocks of one replay (median and max over the 256 workgroups,
    // us from the earliest workgroup start)
    std::vector<unsigned long long> c(256 * kEdges);
    for (int rep = 0; rep < 4; ++rep) { dataflow(); }
    CK(hipMemsetAsync(clk, 0, 256 * kEdges * 8, s));   // (a workgroup without an S3 tile leaves its mark 0)
    dataflow();
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull;
    for (int w = 0; w < 256; ++w) t0 = std::min(t0, c[w * kEdges]);
    const char* names[kEdges] = {"start", "S1 done", "S2 first tile may start", "S2 done",
                                 "S3 first tile may start", "S3 done", ""};
    for (int e = 0; e < 6; ++e) {
      std::vector<double> v;
      for (int w = 0; w < 256; ++w)
        if (c[w * kEdges + e]) v.push_back((c[w * kEdges + e] - t0) * 0.01);
      std::sort(v.begin(), v.end());
      const size_t n = v.size();
      printf("  %-26s median %6.2f us  p90 %6.2f  max %6.2f  (%zu workgroups)\n", names[e], v[n / 2],
             v[(9 * n) / 10], v[n - 1], n);
    }
    printf("3 launches per step (default waves) : %7.2f us/step\n", per_step_us(s, [&] { launches(0); }));
    printf("3 launches per step (16 waves)      : %7.2f us/step\n", per_step_us(s, [&] { launches(16); }));
    printf("1 dataflow launch                   : %7.2f us/step\n", per_step_us(s, [&] { dataflow(); }));
    }
  }
  return 0;
}
