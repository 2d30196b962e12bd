// Building blocks of the LDS-DMA pipelined large-batch GEMMs (gemm_fwd.hip,
// gemm_bwdp.hip): 32-deep K stages staged global -> LDS with
// global_load_lds_dwordx4 (no VGPR round trip) in a ring of three, counted
// vmcnt waits and one raw barrier per stage.
#pragma once
#include "oac_common.h"

namespace oac {

#ifdef OAC_PIPE_CLOCK   // micro-benchmark builds (tools/micro): per-stage clocks of wave 0
__device__ long long g_pipe_clock[4096 * 32];
#define PIPE_CLK(slot) do { if (threadIdx.x == 0 && blockIdx.x < 4096 && (slot) < 32) \
    g_pipe_clock[blockIdx.x * 32 + (slot)] = (long long)__builtin_readcyclecounter(); } while (0)
#else
#define PIPE_CLK(slot) do {} while (0)
#endif

constexpr int kFK = 32;     // k per stage: one 128-byte row piece per operand row
constexpr int kFBuf = 3;    // stages in the LDS ring

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Bank swizzle of a k-contiguous operand image (128-byte rows, 16-byte chunk
// c of row r at slot c ^ kc_swz(r)).  ds_read_b128 is serviced in 16-lane
// groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, the same + 32) over 64 banks
// = two 128-byte rows, so a group's 8 even and 8 odd rows each need 8
// distinct slots: r >> 1 gives that for the fragment reads (row = block base
// + lane), r itself repeated every group's slots twice (2-way: SQ
// LDS_BANK_CONFLICT was ~half of the forward's LDS cycles)
__device__ __forceinline__ int kc_swz(int r) { return (r >> 1) & 7; }

// LDS-DMA of 16 bytes per lane into dst + 16 lane (dst wave-uniform).  Inline
// asm, so the compiler neither tracks it nor inserts its conservative
// vmcnt(0) before every later ds_read of the same LDS array (the builtin
// does: it cannot tell the ring's stages apart); the waits are counted here.
__device__ __forceinline__ void glds16(const float* src, float* dst) {
  const unsigned d = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) void*)dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(d) : "memory");
}

// blocks dispatch round-robin over the 8 XCDs; a tile's neighbours along n
// (same X rows) are given consecutive ids on one XCD so its L2 serves the
// second read of the rows (bijective for any grid size)
__device__ __forceinline__ int xcd_tile(int bid, int n) {
  const int q = n >> 3, r = n & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// The same dispatch, chunks of kXcdChunk consecutive tiles (a row block's
// column tiles: the same X rows) dealt round-robin over the XCDs: each XCD
// gets every task's share instead of a contiguous range of tasks, so tasks of
// unequal work (the critic layer 0's rank continuation) do not pile onto two
// XCDs.  Tiles [0, T), T = the largest multiple of 8 chunks, go by chunks; the
// tail keeps its id (bijective for any grid size).
constexpr int kXcdChunk = 4;
template <int C = kXcdChunk>
__device__ __forceinline__ int xcd_tile_rr(int bid, int n) {
  const int T = n / (8 * C) * (8 * C);
  if (bid >= T) return bid;
  const int x = bid & 7, j = bid >> 3;
  return ((j / C) * 8 + x) * C + j % C;
}

}  // namespace oac
