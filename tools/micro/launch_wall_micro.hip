// Host wall per call of the exploration launch shape, without its work:
// what launching 32 workgroups of 1024 threads and seeing a completion word in
// host memory costs, against a resident group that polls a request word in
// host memory (the floor of a persistent exploration server).
//   launch_sys   : launch, the last block's lane 0 writes the word behind a
//                  system-scope release (expl_split.hip's completion)
//   launch_vm    : the same behind s_waitcnt vmcnt(0) only
//   resident     : 32 resident blocks poll the request word; block 0 answers
// Every resident block exits on the stop word or after ~2 s without a request.
// Build: tools/micro/Makefile.  Run: tools/micro/launch_wall_micro [calls]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

template <bool SYS>
__global__ void __launch_bounds__(1024) k_done(unsigned* done, unsigned seq) {
  __shared__ float pad[21 * 1024];   // one block per CU, as the exploration kernel
  pad[threadIdx.x] = (float)seq;
  __syncthreads();
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    if (SYS) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(done, seq + (pad[1] > 1e30f ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// req[0]: request sequence (0xffffffff = stop); done[0]: answered sequence
__global__ void __launch_bounds__(1024) k_resident(const unsigned* req, unsigned* done) {
  __shared__ float pad[21 * 1024];
  __shared__ unsigned cmd;
  unsigned last = 0;
  pad[threadIdx.x] = 0.f;
  for (;;) {
    if (threadIdx.x == 0) {
      unsigned v = last, spins = 0;
      while (v == last) {
        v = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v != last) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 24)) { v = 0xffffffffu; break; }   // idle: ~2 s
      }
      cmd = v;
    }
    __syncthreads();
    const unsigned v = cmd;
    __syncthreads();
    if (v == 0xffffffffu) return;
    last = v;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(done, v + (pad[1] > 1e30f ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 500;
  unsigned *req, *done;
  const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
  CK(hipHostMalloc((void**)&req, 64, fl));
  CK(hipHostMalloc((void**)&done, 64, fl));
  *req = 0; *done = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto wait_done = [&](unsigned seq, std::chrono::steady_clock::time_point t0) {
    while (*(volatile unsigned*)done != seq)
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        printf("no completion for %u\n", seq);
        exit(1);
      }
  };
  unsigned seq = 0;
  for (int mode = 0; mode < 2; ++mode) {
    std::vector<double> w;
    for (int c = 0; c < calls; ++c) {
      ++seq;
      const auto t0 = std::chrono::steady_clock::now();
      if (mode == 0) k_done<true><<<32, 1024, 0, s>>>(done, seq);
      else k_done<false><<<32, 1024, 0, s>>>(done, seq);
      wait_done(seq, t0);
      w.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
      CK(hipStreamSynchronize(s));
    }
    printf("%-10s host wall per call %.1f us (median of %d)\n", mode == 0 ? "launch_sys" : "launch_vm",
           med(w), calls);
  }
  *done = 0;
  *req = 0;
  seq = 0;
  k_resident<<<32, 1024, 0, s>>>(req, done);
  CK(hipGetLastError());
  std::vector<double> w;
  for (int c = 0; c < calls; ++c) {
    ++seq;
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(req, seq, __ATOMIC_RELEASE);
    wait_done(seq, t0);
    w.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  __atomic_store_n(req, 0xffffffffu, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(s));
  printf("%-10s host wall per call %.1f us (median of %d)\n", "resident", med(w), calls);
  return 0;
}
