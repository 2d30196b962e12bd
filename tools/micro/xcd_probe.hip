// Which XCD (and CU) runs each workgroup of an exploration-shaped launch
// (1024 threads, 84 KB of LDS: one workgroup per CU)?  Prints, per launch, the
// XCC id of every block, and whether block b runs on XCD b % 8.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(1024) probe(int* out, int work) {
  __shared__ float pad[21 * 1024];
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  pad[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  float acc = pad[(threadIdx.x * 7) & 1023];
  for (int i = 0; i < work; ++i) acc = acc * 1.0000001f + 1e-7f;
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = (int)(xcc & 0xf);
    out[2 * blockIdx.x + 1] = (int)hw;
  }
  if (acc == -1.f) out[0] = 7;
}

int pingpong_main(int n);
int main(int argc, char** argv) {
  if (argc > 2) return pingpong_main(atoi(argv[2]));
  const int nb = argc > 1 ? atoi(argv[1]) : 256;
  int* d;
  hipMalloc(&d, 2 * nb * sizeof(int));
  std::vector<int> h(2 * nb);
  hipStream_t s2;
  hipStreamCreate(&s2);
  for (int rep = 0; rep < 6; ++rep) {
    // reps 3-5: another launch of 7 blocks just before, on the same stream
    if (rep >= 3) probe<<<7, 1024, 0, 0>>>(d, 10);
    hipMemset(d, 0xff, 2 * nb * sizeof(int));
    probe<<<nb, 1024, 0, 0>>>(d, 2000);
    hipMemcpy(h.data(), d, 2 * nb * sizeof(int), hipMemcpyDeviceToHost);
    int match = 0, first = h[0];
    for (int b = 0; b < nb; ++b) match += (h[2 * b] == ((b + first) % 8));
    printf("rep %d: block0 xcc %d, blocks on xcc (b + xcc0) %% 8: %d / %d; xcc of blocks 0..15:", rep, first, match, nb);
    for (int b = 0; b < 16 && b < nb; ++b) printf(" %d", h[2 * b]);
    printf("\n  hw_id (cu/sh/se bits) of blocks 0,8,16,24,..:");
    for (int b = 0; b < nb && b < 256; b += 8) printf(" %x", (h[2 * b + 1] >> 8) & 0xfff);
    printf("\n");
  }
  return 0;
}

// ---- flag ping-pong between block 0 and block d (d = 8: same XCD under a
// round-robin dispatch; d = 1: neighbouring XCD).  mode 0: agent-scope
// relaxed atomics (sc1, coherent across XCDs); mode 1: plain stores after
// vmcnt(0) and L1-bypassing (sc0) buffer loads -- coherent within an XCD's L2
// only.  Every poll is bounded, so a stale line ends the run with a count.
__device__ __forceinline__ int ld_sc0(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 1);
}
__global__ void __launch_bounds__(1024) pingpong(int* flags, int n, int mode, int d, long long* res) {
  __shared__ float pad[21 * 1024];
  pad[threadIdx.x] = 0.f;
  const int b = blockIdx.x;
  if ((b != 0 && b != d) || threadIdx.x != 0) return;
  const bool a = b == 0;
  int* mine = flags + (a ? 0 : 32);
  int* other = flags + (a ? 32 : 0);
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(flags, 0, 64 * 4, 0x00020000);
  const int ooff = (a ? 32 : 0) * 4;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  long long fails = 0;
  const long long t0 = wall_clock64();
  for (int i = 1; i <= n; ++i) {
    if (a) {   // A: publish i, wait for B's i
      if (mode == 0) __hip_atomic_store(mine, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else { *(volatile int*)mine = i; asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
    }
    int spins = 0;
    for (;;) {
      const int v = mode == 0 ? __hip_atomic_load(other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : ld_sc0(rs, ooff);
      if (v >= i) break;
      if (++spins > 200000) { ++fails; break; }
    }
    if (!a) {
      if (mode == 0) __hip_atomic_store(mine, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else { *(volatile int*)mine = i; asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
    }
    if (fails > 4) break;
  }
  const long long t1 = wall_clock64();
  res[a ? 0 : 1] = t1 - t0;
  res[a ? 2 : 3] = fails;
  res[a ? 4 : 5] = xcc & 0xf;
}

int pingpong_main(int n) {
  int* flags;
  long long* res;
  hipMalloc(&flags, 64 * 4);
  hipMalloc(&res, 6 * 8);
  int wclk = 0;
  hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);   // kHz
  for (int mode = 0; mode < 2; ++mode)
    for (int d : {8, 1, 16}) {
      hipMemset(flags, 0, 64 * 4);
      hipMemset(res, 0, 6 * 8);
      pingpong<<<d + 1, 1024>>>(flags, n, mode, d, res);
      long long h[6];
      hipMemcpy(h, res, 48, hipMemcpyDeviceToHost);
      printf("pingpong mode %d (%s) d=%2d: xcc %lld / %lld, %.3f us per round trip, failed polls %lld / %lld\n",
             mode, mode ? "plain st + sc0 ld" : "agent atomics", d, h[4], h[5],
             (double)h[0] / n * 1e3 / wclk, h[2], h[3]);
    }
  return 0;
}
