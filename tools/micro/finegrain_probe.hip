// Probe: can the host write device fine-grained memory through a CPU mapping,
// and how long does a kernel's first read of it take vs a host-coherent
// (hipHostMalloc) buffer?  Build: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <csignal>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__global__ void read_sum(const int* p, int n, long long* clk, int* out) {
  const long long t0 = wall_clock64();
  int s = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
  __shared__ int red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int i = 0; i < 256; ++i) t += red[i];
    out[0] = t;
    clk[0] = wall_clock64() - t0;
  }
}

int main() {
  const int n = 256;
  int* dev = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&dev), n * 4, hipDeviceMallocFinegrained));
  int* host = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&host), n * 4, hipHostMallocCoherent | hipHostMallocMapped));
  long long* clk; int* out;
  CK(hipMalloc(&clk, 8)); CK(hipMalloc(&out, 4));
  int khz = 0; CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  hipPointerAttribute_t at;
  CK(hipPointerGetAttributes(&at, dev));
  printf("finegrained device ptr %p hostPointer %p type %d\n", (void*)dev, at.hostPointer, (int)at.type);
  for (int i = 0; i < n; ++i) host[i] = i;
  for (int rep = 0; rep < 3; ++rep) {
    read_sum<<<1, 256>>>(host, n, clk, out);
    CK(hipDeviceSynchronize());
    long long c; int o;
    CK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(&o, out, 4, hipMemcpyDeviceToHost));
    printf("host-coherent ring: sum %d, first read ~%.2f us\n", o, c * 1e3 / khz);
  }
  int* hp = reinterpret_cast<int*>(at.hostPointer);
  if (!hp) { printf("no host mapping of the fine-grained device allocation\n"); return 0; }
  for (int i = 0; i < n; ++i) hp[i] = 2 * i;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  for (int rep = 0; rep < 3; ++rep) {
    read_sum<<<1, 256>>>(dev, n, clk, out);
    CK(hipDeviceSynchronize());
    long long c; int o;
    CK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(&o, out, 4, hipMemcpyDeviceToHost));
    printf("fine-grained device ring (host-written): sum %d (want %d), first read ~%.2f us\n", o, n * (n - 1), c * 1e3 / khz);
  }
  return 0;
}
