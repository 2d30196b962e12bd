// Stage clocks of the exploration kernel (expl_split.hip built with
// -DOAC_EXPL_CLOCK): one Humanoid-dim observation (obs 376, act 17, 2x256,
// twin critics), the launch shape of oac_expl_action_now (observation and
// outputs in host-coherent memory, the host polling the completion word).
// Prints the per-stage wall clock of the group's first and last workgroup
// (100 MHz counter, median over the calls) and the host wall per call.
// Build: tools/micro/Makefile.  Run: tools/micro/expl_micro [calls] [obs in arguments 0|1]
//   [split kernel 0|1: the four-hand-off kernel instead of the twin-critic one] [group cap]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../oac-explore_amd/csrc/expl_split.hip"

namespace oac { thread_local ExtTiming g_ext_timing; extern bool g_expl_twin_off; extern int g_expl_group_cap; }
using namespace oac;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

static float* dev_rand(size_t n, unsigned seed, float scale) {
  std::vector<float> h(n + 64);
  srand(seed);
  for (auto& x : h) x = scale * ((float)rand() / (float)RAND_MAX - 0.5f);
  float* d; CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 200;
  const bool obs_arg = argc > 2 && atoi(argv[2]) != 0;   // the observation in the arguments
  const bool split = argc > 3 && atoi(argv[3]) != 0;     // the four-hand-off kernel
  g_expl_twin_off = split;
  if (argc > 4) g_expl_group_cap = atoi(argv[4]);   // group-size sweep
  const int Do = 376, Da = 17, H = 256, Dq = Do + Da;
  // parameter blocks: policy [fc0 | fc1 | head], critics [fc0 | fc1 | last]
  const long p0w = 0, p0b = p0w + (long)H * Do, p1w = p0b + H, p1b = p1w + (long)H * H,
             phw = p1b + H, phb = phw + 2L * Da * H, psz = phb + 2 * Da + 64;
  const long q0w = 0, q0b = q0w + (long)H * Dq, q1w = q0b + H, q1b = q1w + (long)H * H,
             qlw = q1b + H, qlb = qlw + H, qsz = qlb + 64;
  float* pol = dev_rand(psz, 1, 0.1f);
  float* q1 = dev_rand(qsz, 2, 0.1f);
  float* q2 = dev_rand(qsz, 3, 0.1f);
  float *obs, *out; unsigned* done;
  const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
  CK(hipHostMalloc((void**)&obs, sizeof(float) * (Do + Da), fl));
  CK(hipHostMalloc((void**)&out, sizeof(float) * 3 * Da, fl));
  CK(hipHostMalloc((void**)&done, 64, fl));
  unsigned long long* tags;   // the single call's outputs as tagged granules (oac_expl_action_now)
  CK(hipHostMalloc((void**)&tags, sizeof(unsigned long long) * 3 * Da, fl));
  memset(tags, 0, sizeof(unsigned long long) * 3 * Da);
  for (int k = 0; k < Do; ++k) obs[k] = (float)((k * 37) % 101) / 101.f - 0.5f;
  *done = 0;
  const long scr = expl_split_scratch_floats(H);
  float* ws; CK(hipMalloc(&ws, sizeof(float) * (scr + 4096)));
  CK(hipMemset(ws, 0, sizeof(float) * (scr + 4096)));
  float* grad; CK(hipMalloc(&grad, sizeof(float) * 64));
  StepState* st; CK(hipMalloc(&st, 256)); CK(hipMemset(st, 0, 256));
  unsigned* words; CK(hipMalloc(&words, 64)); CK(hipMemset(words, 0, 64));
  ExplFusedArgs a;
  memset(&a, 0, sizeof(a));
  a.obs = obs; a.ld_obs = Do + Da; a.pol = pol; a.q[0] = q1; a.q[1] = q2;
  a.p_fc0_w = p0w; a.p_fc0_b = p0b; a.p_fc1_w = p1w; a.p_fc1_b = p1b; a.p_head_w = phw; a.p_head_b = phb;
  a.q_fc0_w = q0w; a.q_fc0_b = q0b; a.q_fc1_w = q1w; a.q_fc1_b = q1b; a.q_last_w = qlw; a.q_last_b = qlb;
  a.Do = Do; a.Da = Da; a.H = H; a.n = 1; a.nq = 2; a.K = 1;
  a.eps = nullptr; a.out = out; a.grad = grad; a.state = st; a.ticket = words; a.fail = words + 1;
  a.seed = 7; a.beta_UB = 4.66f; a.sqrt_2delta = 6.86f; a.ub_index = -1; a.done = done; a.tags = tags;
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int G = expl_split_group(1);
  std::vector<std::vector<long long>> clk(64);
  std::vector<double> wall;
  for (int c = 0; c < calls; ++c) {
    a.done_seq = (unsigned)(c + 1);
    const auto t0 = std::chrono::steady_clock::now();
    if (obs_arg) {
      ExplObsArg o;
      memcpy(o.v, obs, sizeof(float) * Do);
      CK(launch_expl_split_obs(a, o, ws + 4096, s));
    } else {
      CK(launch_expl_split(a, 0, 1, ws + 4096, s));
    }
    // bounded: a failed call (bit 31) or a faulted launch ends the run
    for (int i = 0; i < 3 * Da; ++i) {
      volatile unsigned long long* g = tags + i;
      while (((unsigned)(*g >> 32) & 0x7fffffffu) != a.done_seq) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2) ||
            hipStreamQuery(s) != hipErrorNotReady) {
          if (((unsigned)(*g >> 32) & 0x7fffffffu) == a.done_seq) break;
          printf("call %d: no completion (stream %s)\n", c, hipGetErrorString(hipStreamQuery(s)));
          return 1;
        }
      }
      if (*g >> 63) { printf("call %d: hand-off timed out\n", c); return 1; }
    }
    const auto t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(s));
    wall.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    long long h[64];
    CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_expl_clock), sizeof(h)));
    if (c >= 20)
      for (int i = 0; i < 64; ++i) clk[i].push_back(h[i]);
  }
  auto med = [](std::vector<long long> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  auto medd = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  const char* names_split[13] = {"start", "obs read", "S1 compute", "hand-off 0", "S2 compute", "hand-off 1",
                                 "heads+tanh", "S3 rest", "hand-off 2", "S4 compute", "hand-off 3",
                                 "S5 da", "S5 rest"};
  const char* names_twin[13] = {"start", "obs read", "S1 + z", "hand-off A", "h2 sums", "heads+tanh",
                                "critic L0", "critic L1+u", "arrival B", "S3 sums", "S3 da", "S3 rest", "-"};
  const char* const* names = split ? names_split : names_twin;
  const int last_both = split ? 9 : 7, n_st = split ? 12 : 11;
  printf("%s kernel; obs %s; group of %d workgroups; host wall per call %.1f us (median of %d)\n",
         split ? "split" : "twin", obs_arg ? "in arguments" : "host row", G, medd(wall), calls);
  printf("stage (us, from workgroup 0's start; median): wg0 / last wg\n");
  std::vector<long long> base = clk[0];
  {
    std::vector<long long> d1;
    for (size_t c = 0; c < base.size(); ++c) d1.push_back(clk[32][c] - base[c]);
    printf("  %-12s %6.2f  %6.2f\n", "start", 0.0, med(d1) / 100.0);
  }
  for (int i = 1; i <= n_st; ++i) {
    std::vector<long long> d0, d1;
    for (size_t c = 0; c < base.size(); ++c) {
      d0.push_back(clk[i][c] - base[c]);
      d1.push_back(clk[32 + i][c] - base[c]);
    }
    printf("  %-12s %6.2f  %6.2f\n", names[i], med(d0) / 100.0,
           (i <= last_both ? med(d1) / 100.0 : 0.0));
  }
  return 0;
}
