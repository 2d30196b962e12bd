// Register-direct grouped fp32 GEMM for the large-batch stages (B >= 1024:
// BASELINE configs 2-4): gemm_cfg 2 (forward batches, 64x32 wave blocks)
// and 3 (backward batches -- dX = dY W and dW = dY^T [X | 1] -- with 32x32
// wave blocks and 3 k-groups in flight), chosen per launch in plan_common.h
// launch_cfg.
//
// The LDS-staged 64x64 kernel (gemm.hip) reached ~21 % of the fp32 MFMA peak
// at B=4096: one barrier per 32-deep K block, dword staging loads and one
// 32x32 accumulator per wave.  Here every wave owns a (32 WM) x (32 WN) output
// block -- WM x WN accumulators of v_mfma_f32_32x32x2_f32 -- and feeds the
// MFMAs straight from L2 into VGPRs (gemm_operand.h: a k-contiguous operand is
// one 16-byte load per lane per 4 MFMAs; a batch-major operand of a backward
// product one coalesced dword per lane and k), so per 8-deep k-group a lane
// issues WM + WN loads for 4 WM WN MFMAs, with no LDS and no barrier: the
// waves of a workgroup run independently and the next groups' loads are in
// flight while the current group's MFMAs issue (register multi-buffer).  Four
// waves (2 x 2) form a (64 WM) x (64 WN) workgroup tile so neighbouring waves
// share operand lines in L1/L2.  Split-K (the dW tasks, K = batch) writes
// slabs exactly like the other kernels; every epilogue reads the accumulator
// registers directly.
//
// Backward products, B=4096 SAC step (rocprofv3 per launch, LDS kernel ->
// this one, before the split retune): critic layer 1 72.1 -> 59.7 us, critic
// layer 0 49.9 -> 37.9 us; with 32x32 wave blocks, kchunk >= 128 and 3
// groups in flight the step went 2,044 -> 2,214 steps/s (tools/env_sweep.sh).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "oac_common.h"
#include "kernels.h"
#include "gemm_operand.h"
#include "gemm_epilogue.h"
#include "adam_common.h"

namespace oac {

template <int AK, int BK, int WM, int WN>
struct Frag {
  float ax[WM][4], ay[WM][4], bx[WN][4], by[WN][4];
};

template <int AK, int BK, int WM, int WN>
__device__ __forceinline__ void frag_load(const Lane (&la)[WM], const Lane (&lb)[WN], int g, int half,
                                          int kmax, Frag<AK, BK, WM, WN>& f) {
  const int kb = 8 * g + 4 * half;
#pragma unroll
  for (int i = 0; i < WM; ++i) load4<AK>(la[i], kb, kmax, f.ax[i], f.ay[i]);
#pragma unroll
  for (int j = 0; j < WN; ++j) load4<BK>(lb[j], kb, kmax, f.bx[j], f.by[j]);
}

template <int AK, int BK, int WM, int WN>
__device__ __forceinline__ void frag_mma(const Lane (&la)[WM], const Lane (&lb)[WN], int g, int half,
                                         int k_lo, int k_hi, const Frag<AK, BK, WM, WN>& f,
                                         floatx16 (&acc)[WM][WN]) {
  const int kb = 8 * g + 4 * half;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float a[WM], b[WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)   // k < k_lo: a continuation pass's first group (A side only)
      a[i] = kb + c >= k_lo ? fix1<AK>(la[i], kb + c, k_hi, f.ax[i][c], f.ay[i][c]) : 0.f;
#pragma unroll
    for (int j = 0; j < WN; ++j) b[j] = fix1<BK>(lb[j], kb + c, k_hi, f.bx[j][c], f.by[j][c]);
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// acc += A[mw.., k_lo..k_hi) . B[k_lo..k_hi), nw..] over this wave's block
template <int AK, int BK, int WM, int WN, int PF = 2>
__device__ __forceinline__ void rd_loop(const GemmTask& t, const float* A, long lda, const float* Bp,
                                        long ldb, int M, int Nlanes, bool ones, int mw, int nw,
                                        int k_lo, int k_hi, floatx16 (&acc)[WM][WN]) {
  const int lane = threadIdx.x & 63;
  const int l32 = lane & 31, half = lane >> 5;
  const bool ar1 = (AK == OP_KC_R1 || AK == OP_MN_R1);
  Lane la[WM], lb[WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
    la[i] = lane_init<AK>(mw + 32 * i + l32, M, false, ar1 ? t.a_mask : A, ar1 ? t.ld_mask : lda,
                          t.a_s, t.a_v);
#pragma unroll
  for (int j = 0; j < WN; ++j)
    lb[j] = lane_init<BK>(nw + 32 * j + l32, Nlanes, ones, Bp, ldb, nullptr, nullptr);
  const int g_lo = k_lo >> 3, g_hi = (k_hi + 7) >> 3, kmax = k_hi - 1;
  if (g_lo >= g_hi) return;
  // PF k-groups in flight: group g + PF is requested as soon as group g's
  // fragments are consumed
  Frag<AK, BK, WM, WN> f[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (g_lo + q < g_hi) frag_load<AK, BK, WM, WN>(la, lb, g_lo + q, half, kmax, f[q]);
#pragma unroll 1
  for (int g = g_lo; g < g_hi; g += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      if (g + q < g_hi) {
        frag_mma<AK, BK, WM, WN>(la, lb, g + q, half, k_lo, k_hi, f[q], acc);
        if (g + q + PF < g_hi) frag_load<AK, BK, WM, WN>(la, lb, g + q + PF, half, kmax, f[q]);
      }
    }
  }
}

template <int WM, int WN, int PF>
__global__ void __launch_bounds__(256)
gemm_big_kernel(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                const GemmBatch batch) {
  const int bid = blockIdx.x;
  if (batch.publish && bid == 0 && threadIdx.x == 0)
    publish_step_consts(batch.publish, batch.pub_beta1, batch.pub_beta2);
  if (bid >= total_tiles) return;
  int ti = 0;   // task from the preloaded tile starts
  ti = bid >= tb1 ? 1 : ti; ti = bid >= tb2 ? 2 : ti; ti = bid >= tb3 ? 3 : ti;
  ti = bid >= tb4 ? 4 : ti; ti = bid >= tb5 ? 5 : ti; ti = bid >= tb6 ? 6 : ti;
  ti = bid >= tb7 ? 7 : ti;
  ti = __builtin_amdgcn_readfirstlane(ti);
  GemmTask t = batch.t[ti];
  int local = bid - t.tile_begin;
  int k_lo = 0, k_hi = t.K;
  if (t.ksplit > 1) {
    const int split = local % t.ksplit;
    local /= t.ksplit;
    k_lo = split * t.kchunk;
    k_hi = min(t.K, k_lo + t.kchunk);
    t.C += (long)split * t.slab_stride;
    t.bias_grad += (long)split * t.slab_stride;
  }
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m0 = (local / t.tiles_n) * (64 * WM);
  const int n0 = (local % t.tiles_n) * (64 * WN);
  const int mw = m0 + (wave >> 1) * 32 * WM;
  const int nw = n0 + (wave & 1) * 32 * WN;
  if (mw >= t.M || nw >= t.N) return;   // wave-uniform: no barriers in this kernel
  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // operand kinds per task (wave-uniform): forward products (both operands
  // k-contiguous), dX = dY W (dY k-contiguous, possibly a rank-1 seed through
  // a ReLU mask; W n-contiguous) and dW = dY^T [X | 1] (both batch-major, so
  // m/n-contiguous: one coalesced dword per lane and k)
  const int nl = t.b_ones ? t.N - 1 : t.N;
  const bool ones = t.b_ones != 0;
  const bool r1 = t.a_mode != A_PLAIN;
  if (t.a_kc && t.b_kc)
    rd_loop<OP_KC, OP_KC, WM, WN, PF>(t, t.A, t.lda, t.B, t.ldb, t.M, nl, ones, mw, nw, k_lo, k_hi, acc);
  else if (t.a_kc && !r1)
    rd_loop<OP_KC, OP_MN, WM, WN, PF>(t, t.A, t.lda, t.B, t.ldb, t.M, nl, ones, mw, nw, k_lo, k_hi, acc);
  else if (t.a_kc)
    rd_loop<OP_KC_R1, OP_MN, WM, WN, PF>(t, t.A, t.lda, t.B, t.ldb, t.M, nl, ones, mw, nw, k_lo, k_hi, acc);
  else if (!r1)
    rd_loop<OP_MN, OP_MN, WM, WN, PF>(t, t.A, t.lda, t.B, t.ldb, t.M, nl, ones, mw, nw, k_lo, k_hi, acc);
  else
    rd_loop<OP_MN_R1, OP_MN, WM, WN, PF>(t, t.A, t.lda, t.B, t.ldb, t.M, nl, ones, mw, nw, k_lo, k_hi, acc);
  rd_epilogue<WM, WN>(t, mw, nw, acc, false);
  if (t.epi == EPI_BIAS_RANK_RELU) {
    // + U V^T: when U / V continue A / B along k (the batch actions follow the
    // observations in a replay row, the action columns follow the observation
    // columns in W0), the same accumulators run on over k in [K, K + R) --
    // the critic's 393-wide layer 0 with the obs-only projection P
    // snapshotted on the way
    // (a separate rank-R operand -- the policy's action buffer a~ against the
    // action columns of W0 -- runs the same accumulators over k in [0, R) of U / V)
    if (t.U == t.A + t.K && t.ldu == t.lda && t.V == t.B + t.K && t.ldv == t.ldb)
      rd_loop<OP_KC, OP_KC, WM, WN, PF>(t, t.A, t.lda, t.B, t.ldb, t.M, t.N, false, mw, nw, t.K,
                                        t.K + t.R, acc);
    else
      rd_loop<OP_KC, OP_KC, WM, WN, PF>(t, t.U, t.ldu, t.V, t.ldv, t.M, t.N, false, mw, nw, 0, t.R,
                                        acc);
    epi_dispatch<WM, WN, EPI_BIAS_RANK_RELU>(t, mw, nw, acc, true);
  }
}

// wave block (32 WM) x (32 WN), default 64 x 32 (workgroup 128 x 64): at
// B=4096, 1,828 steps/s against 1,827 for 32 x 64, 1,775 for 64 x 64 and 1,741
// for 32 x 32; 3 k-groups in flight instead of 2 changed nothing (+-1 %).
// Backward batches (dX / dW, cfg 3) use 32 x 32 wave blocks (64 x 64
// workgroups): at B=4096 their products are 256 wide, and the 4x larger
// grid hides the per-wave operand latency better than the larger blocks do.
static int big_wm(bool bwd) { return bwd ? 1 : 2; }
static int big_wn(bool bwd) { (void)bwd; return 1; }
int gemm_big_tile_m(bool bwd) { return 64 * big_wm(bwd); }
int gemm_big_tile_n(bool bwd) { return 64 * big_wn(bwd); }

hipError_t gemm_big_launch(const GemmBatch& b, hipStream_t s, bool bwd) {
  if (b.total_tiles <= 0) return hipSuccess;
  for (int i = 0; i < b.ntasks; ++i) {
    const GemmTask& t = b.t[i];
    if (t.K2 > 0 || t.epi == EPI_HEAD_BWD || b.fuse_adam ||
        (t.b_kc && !t.a_kc) || (t.b_kc && t.a_mode != A_PLAIN))
      return hipErrorInvalidValue;   // kinds handled in gemm_big_kernel
    if (t.epi == EPI_BIAS_RANK_RELU && (!t.C2 || t.ksplit > 1)) return hipErrorInvalidValue;
  }
  int tb[8];
  for (int i = 0; i < 8; ++i) tb[i] = i < b.ntasks ? b.t[i].tile_begin : 0x7fffffff;
  const int pf = bwd ? 3 : 2;   // k-groups in flight
#define OAC_BIG(WM_, WN_, PF_) \
  if (big_wm(bwd) == WM_ && big_wn(bwd) == WN_ && pf == PF_) { \
    OAC_LAUNCH((gemm_big_kernel<WM_, WN_, PF_>), dim3(b.total_tiles), dim3(256), 0, s, b.total_tiles, \
               tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b); \
    return hipGetLastError(); }
  OAC_BIG(2, 1, 2) OAC_BIG(1, 1, 3)
#undef OAC_BIG
  return hipErrorInvalidValue;
}

}  // namespace oac
