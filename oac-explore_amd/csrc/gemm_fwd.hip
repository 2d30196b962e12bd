// Large-batch forward products (gemm_cfg 6): Y = X W^T (+ b, ReLU; the
// critic's rank-Da action columns as a continuation of the same
// accumulators; the width-1 head partials) at B >= 1024, both operands
// k-contiguous.
//
// The register-direct forward kernel (gemm_big.hip, cfg 2) spends one 16-byte
// global load per lane for every 4 MFMAs of each 32x32 block it owns; on the
// B=4096 step its launches keep the TA (vector address) unit ~70 % busy at
// 43 % of the MFMA peak (tools/pmc_bwd.sh): the load path, not the MFMA pipe,
// bounds them.  Here a 256-thread workgroup (2 x 2 waves, each a (BM/2) x
// (BN/2) block of v_mfma_f32_32x32x2_f32 accumulators) stages BM x 32 of X
// and BN x 32 of W per K stage into LDS with LDS-DMA loads
// (global_load_lds_dwordx4: no VGPR round trip, one 1-KB wave instruction per
// 8 rows), in a ring of three stages: two stages are in flight while the
// third is read, the waits are counted (vmcnt = one stage's loads), and one
// raw barrier per stage orders both the DMA's landing and the ring's reuse.
// The LDS image is lane-linear, so the bank swizzle (16-byte chunk c of row r
// at slot c ^ kc_swz(r), gemm_pipe.h) is applied to the per-lane SOURCE address and undone
// on the ds_read_b128 fragment reads.
//
// The MFMA sequence per accumulator is the register-direct kernel's (8-deep
// k-groups from k = 8 floor(k_lo / 8), c = 0..3 per group, lanes 32-63 on
// the group's upper half), so both kernels produce bitwise equal outputs.
#include <cstdlib>

#include "oac_common.h"
#include "kernels.h"
#include "gemm_epilogue.h"
#include "gemm_pipe.h"
#include "adam_common.h"

namespace oac {

#ifdef OAC_PIPE_CLOCK
#define gemm_fwd_kernel gemm_fwd_kernel_clk   // distinct from the library's kernels of the same names
#define gemm_fwd_kernel_dev gemm_fwd_kernel_dev_clk
#endif

template <int BM, int BN>
struct FwdG {
  static constexpr int WM = BM / 64, WN = BN / 64;   // 32x32 blocks per wave (2 x 2 waves)
  static constexpr int PA = BM / 32, PB = BN / 32;   // LDS-DMA instructions per wave and stage
  static constexpr int LPW = PA + PB;
  static constexpr int STAGE = (BM + BN) * kFK;      // floats
};

// one stage's fragments and MFMAs; mask (wave-uniform): zero k outside [k_lo, k_hi)
template <int WM, int WN>
__device__ __forceinline__ void fwd_stage(const float* as, const float* bs, const int (&aoff)[WM],
                                          const int (&boff)[WN], int xh, int hl, int kst, int half,
                                          int k_lo, int k_hi, bool mask, floatx16 (&acc)[WM][WN]) {
#pragma unroll
  for (int g = 0; g < kFK / 8; ++g) {
    const int slot = 4 * (((2 * g) ^ xh) + hl);   // chunk 2g + half, swizzled by the row
    float4 af[WM], bf[WN];
#pragma unroll
    for (int i = 0; i < WM; ++i) af[i] = *reinterpret_cast<const float4*>(as + aoff[i] + slot);
#pragma unroll
    for (int j = 0; j < WN; ++j) bf[j] = *reinterpret_cast<const float4*>(bs + boff[j] + slot);
    if (mask) {
      const int k = kst + 8 * g + 4 * half;
      const bool o0 = k >= k_lo && k < k_hi, o1 = k + 1 >= k_lo && k + 1 < k_hi;
      const bool o2 = k + 2 >= k_lo && k + 2 < k_hi, o3 = k + 3 >= k_lo && k + 3 < k_hi;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        af[i].x = o0 ? af[i].x : 0.f; af[i].y = o1 ? af[i].y : 0.f;
        af[i].z = o2 ? af[i].z : 0.f; af[i].w = o3 ? af[i].w : 0.f;
      }
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        bf[j].x = o0 ? bf[j].x : 0.f; bf[j].y = o1 ? bf[j].y : 0.f;
        bf[j].z = o2 ? bf[j].z : 0.f; bf[j].w = o3 ? bf[j].w : 0.f;
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          const float a = c == 0 ? af[i].x : c == 1 ? af[i].y : c == 2 ? af[i].z : af[i].w;
          const float b = c == 0 ? bf[j].x : c == 1 ? bf[j].y : c == 2 ? bf[j].z : bf[j].w;
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i][j], 0, 0, 0);
        }
  }
}

// acc += A[m0 .. m0+BM, k_lo..k_hi) . B[n0 .. n0+BN, k_lo..k_hi)^T over this wave's blocks.
// Rows past M / N are clamped to the last row (their outputs are not stored);
// the k range runs in 32-deep stages from 8 floor(k_lo / 8).  A chunk wholly
// past k_hi is fetched from the stage's first chunk instead (always in the
// row); the chunk that straddles k_hi reads up to 3 floats past it (every
// operand buffer is followed by >= 8 readable floats, gemm_operand.h).
// rows: null, or A row m is buffer row rows[m] (the direct gather: the step's
// index slot)
template <int BM, int BN, int NB>
__device__ __forceinline__ void fwd_pipe(const float* A, long lda, int M, const float* B, long ldb,
                                         int N, int k_lo, int k_hi, int m0, int n0, float* lds,
                                         floatx16 (&acc)[BM / 64][BN / 64],
                                         const int* rows = nullptr) {
  using G = FwdG<BM, BN>;
  constexpr int WM = G::WM, WN = G::WN, PA = G::PA, PB = G::PB;
  const int kb0 = k_lo & ~7;
  const int nst = (k_hi - kb0 + kFK - 1) / kFK;
  if (nst <= 0) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // LDS-DMA sources: piece p (8 rows) of an operand is wave p / P's
  // instruction p % P; lane j fills row 8p + j / 8, slot j % 8 = chunk
  // (j % 8) ^ kc_swz(row)
  const float* sa[PA];
  const float* sb[PB];
  int ca[PA], cb[PB];
#pragma unroll
  for (int q = 0; q < PA; ++q) {
    const int r = 8 * (wave * PA + q) + (lane >> 3);
    ca[q] = 4 * ((lane & 7) ^ kc_swz(r));
    const int m = min(m0 + r, M - 1);
    sa[q] = A + (long)(rows ? rows[m] : m) * lda;
  }
#pragma unroll
  for (int q = 0; q < PB; ++q) {
    const int r = 8 * (wave * PB + q) + (lane >> 3);
    cb[q] = 4 * ((lane & 7) ^ kc_swz(r));
    sb[q] = B + (long)min(n0 + r, N - 1) * ldb;
  }
  auto issue = [&](int st) {
    const int kst = kb0 + st * kFK;
    float* base = lds + (st % NB) * G::STAGE;
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int k = kst + ca[q];
      glds16(sa[q] + (k < k_hi ? k : kst), base + (wave * PA + q) * 256);
    }
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int k = kst + cb[q];
      glds16(sb[q] + (k < k_hi ? k : kst), base + BM * kFK + (wave * PB + q) * 256);
    }
  };
  // fragment reads: row r = (wave block) + 32 i + l32, chunk (2g + half) ^ kc_swz(r)
  // (the block bases are multiples of 32, so kc_swz(r) = kc_swz(l32))
  const int l32 = lane & 31, half = lane >> 5;
  const int xh = kc_swz(l32) & 6, hl = half ^ (kc_swz(l32) & 1);
  int aoff[WM], boff[WN];
#pragma unroll
  for (int i = 0; i < WM; ++i) aoff[i] = ((wave >> 1) * (BM / 2) + 32 * i + l32) * kFK;
#pragma unroll
  for (int j = 0; j < WN; ++j) boff[j] = ((wave & 1) * (BN / 2) + 32 * j + l32) * kFK;

  raw_barrier();   // the ring's previous pass (a continuation) is fully read
  PIPE_CLK(1);
  // NB = 3: two stages in flight while one is read; NB = 2 (a smaller LDS
  // footprint, one more workgroup per CU): one
  issue(0);
  if (NB == 3 && nst > 1) issue(1);
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    if (NB == 3 && st + 1 < nst) wait_vm<G::LPW>();
    else wait_vm<0>();
    raw_barrier();   // stage st landed for every wave; stage st - 1 is read by all
    PIPE_CLK(2 + st);
    if (st + NB - 1 < nst) issue(st + NB - 1);
    const int kst = kb0 + st * kFK;
    const float* as = lds + (st % NB) * G::STAGE;
    const float* bs = as + BM * kFK;
    fwd_stage<WM, WN>(as, bs, aoff, boff, xh, hl, kst, half, k_lo, k_hi,
                      kst < k_lo || kst + kFK > k_hi, acc);
  }
}

// Side workgroup sb of nsb (256 threads) of a direct-gather step's forward
// launches (GemmBatch::rg, blocks > 0): with rg.out, its rows of the step's
// batch (row r = 4 sb + wave + 4 nsb k) copied from the replay through the
// index slot -- the gather launch's copy, for the step's later readers --;
// with rg.eps1, its share of the step's Philox eps.  A wave's row indices are
// loaded together, and a row's float4s all in flight before its stores.
__device__ __forceinline__ void fwd_gather_side(const RowGather& g, int sb, int nsb) {
  const long long bc = g.state->batch_counter;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long n4 = g.row_stride >> 2;   // <= 256 (oac_sac row layouts: checked at launch)
  constexpr int KR = 8;
  const int* rows = g.out ? g.ring + (long)(bc % g.slots) * g.B : nullptr;
  for (int r0 = 4 * sb + wave; rows && r0 < g.B; r0 += 4 * nsb * KR) {
    int src_row[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) src_row[k] = rows[min(r0 + 4 * nsb * k, g.B - 1)];
#pragma unroll 1
    for (int k = 0; k < KR; ++k) {
      const int r = r0 + 4 * nsb * k;
      if (r >= g.B) break;
      const float4* src = reinterpret_cast<const float4*>(g.replay) + (long)src_row[k] * n4;
      float4* dst = reinterpret_cast<float4*>(g.out) + (long)r * n4;
      // four named registers, not an array: the array form went through
      // scratch (80 bytes of private segment, a store and a reload per float4)
      const long c0 = lane, c1 = lane + 64, c2 = lane + 128, c3 = lane + 192;
      const float4 v0 = src[c0 < n4 ? c0 : 0], v1 = src[c1 < n4 ? c1 : 0];
      const float4 v2 = src[c2 < n4 ? c2 : 0], v3 = src[c3 < n4 ? c3 : 0];
      if (c0 < n4) dst[c0] = v0;
      if (c1 < n4) dst[c1] = v1;
      if (c2 < n4) dst[c2] = v2;
      if (c3 < n4) dst[c3] = v3;
    }
  }
  if (!g.eps1) return;
  for (int e = sb * 256 + threadIdx.x; e < g.n_eps; e += nsb * 256) {
    g.eps1[e] = philox_normal(g.seed, (unsigned long long)bc, 1u, (unsigned)e);
    g.eps2[e] = philox_normal(g.seed, (unsigned long long)bc, 2u, (unsigned)e);
  }
}

template <int BM, int BN, int NB>
__device__ __forceinline__ void gemm_fwd_body(int total_tiles, int tb1, int tb2, int tb3, int tb4,
                                              int tb5, int tb6, int tb7, const GemmBatch& batch,
                                              float* lds) {
  using G = FwdG<BM, BN>;
  constexpr int WM = G::WM, WN = G::WN;
  if (batch.publish && blockIdx.x == 0 && threadIdx.x == 0)
    publish_step_consts(batch.publish, batch.pub_beta1, batch.pub_beta2);
  if ((int)blockIdx.x >= total_tiles) {   // side workgroups of a direct gather (GemmBatch::rg)
    fwd_gather_side(batch.rg, blockIdx.x - total_tiles, gridDim.x - total_tiles);
    return;
  }
  const int bid = xcd_tile_rr(blockIdx.x, total_tiles);
  // the direct gather's index slot (the A rows of the a_rows tasks)
  const int* rows = batch.rg.ring && batch.rg.slots > 0
                        ? batch.rg.ring + (long)(batch.rg.state->batch_counter % batch.rg.slots) * batch.rg.B
                        : nullptr;
  int ti = 0;
  ti = bid >= tb1 ? 1 : ti; ti = bid >= tb2 ? 2 : ti; ti = bid >= tb3 ? 3 : ti;
  ti = bid >= tb4 ? 4 : ti; ti = bid >= tb5 ? 5 : ti; ti = bid >= tb6 ? 6 : ti;
  ti = bid >= tb7 ? 7 : ti;
  ti = __builtin_amdgcn_readfirstlane(ti);
  const GemmTask& t = batch.t[ti];
  const int local = bid - t.tile_begin;
  const int m0 = (local / t.tiles_n) * BM;
  const int n0 = (local % t.tiles_n) * BN;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mw = m0 + (wave >> 1) * (BM / 2), nw = n0 + (wave & 1) * (BN / 2);
  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  PIPE_CLK(0);
  const int* arows = t.a_rows ? rows : nullptr;
  fwd_pipe<BM, BN, NB>(t.A, t.lda, t.M, t.B, t.ldb, t.N, 0, t.K, m0, n0, lds, acc, arows);
  PIPE_CLK(29);
  rd_epilogue<WM, WN, kEpiFwd>(t, mw, nw, acc, false);
  PIPE_CLK(30);
  if (t.epi == EPI_BIAS_RANK_RELU) {   // + U V^T on the same accumulators (gemm_big.hip)
    if (t.U == t.A + t.K && t.ldu == t.lda && t.V == t.B + t.K && t.ldv == t.ldb)
      fwd_pipe<BM, BN, NB>(t.A, t.lda, t.M, t.B, t.ldb, t.N, t.K, t.K + t.R, m0, n0, lds, acc, arows);
    else
      fwd_pipe<BM, BN, NB>(t.U, t.ldu, t.M, t.V, t.ldv, t.N, 0, t.R, m0, n0, lds, acc);
    epi_dispatch<WM, WN, EPI_BIAS_RANK_RELU>(t, mw, nw, acc, true);
  }
  PIPE_CLK(31);
}

// waves per SIMD the registers must allow so that the 2-stage ring's LDS, not
// the VGPRs, sets the workgroups per CU (128x64: 48 KB -> three; 128x128:
// 64 KB -> two; 64x64: four)
template <int BM, int BN, int NB>
__global__ void __launch_bounds__(256, NB == 2 ? (BM == 128 && BN == 128 ? 2 : BM == 128 ? 3 : 4) : 1)
gemm_fwd_kernel(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) float lds[NB * FwdG<BM, BN>::STAGE];
  gemm_fwd_body<BM, BN, NB>(total_tiles, tb1, tb2, tb3, tb4, tb5, tb6, tb7, batch, lds);
}
// the batch in device memory (kernels.h BatchCache)
template <int BM, int BN, int NB>
__global__ void __launch_bounds__(256, NB == 2 ? (BM == 128 && BN == 128 ? 2 : BM == 128 ? 3 : 4) : 1)
gemm_fwd_kernel_dev(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                    const GemmBatchG* __restrict__ bp) {
  __shared__ __attribute__((aligned(16))) float lds[NB * FwdG<BM, BN>::STAGE];
  gemm_fwd_body<BM, BN, NB>(total_tiles, tb1, tb2, tb3, tb4, tb5, tb6, tb7, *(const GemmBatch*)bp, lds);
}

// forward batches this kernel takes: both operands k-contiguous, plain A, no
// split, no second product, the forward epilogues of the register-direct
// kernel; a_rows tasks (the direct gather) with the batch's RowGather, whose
// rank-R columns (if any) continue the same rows
bool gemm_fwd_supports(const GemmBatch& b) {
  if (b.fuse_adam || b.ntasks < 1) return false;
  if (b.rg.blocks > 0 && !b.rg.state) return false;
  if ((b.rg.ring || b.rg.out) &&
      (!b.rg.ring || !b.rg.state || b.rg.slots < 1 || b.rg.row_stride % 4 || b.rg.row_stride / 4 > 256))
    return false;
  for (int i = 0; i < b.ntasks; ++i) {
    const GemmTask& t = b.t[i];
    if (!t.a_kc || !t.b_kc || t.a_mode != A_PLAIN || t.ksplit > 1 || t.K2 > 0) return false;
    if (t.a_rows && (!b.rg.ring || (t.epi == EPI_BIAS_RANK_RELU && t.U != t.A + t.K))) return false;
    if (t.epi != EPI_STORE && t.epi != EPI_BIAS && t.epi != EPI_BIAS_RELU &&
        t.epi != EPI_BIAS_RANK_RELU && t.epi != EPI_BIAS_RELU_DOT)
      return false;
    if (t.epi == EPI_BIAS_RANK_RELU && !t.C2) return false;
    if (t.epi == EPI_BIAS_RELU_DOT && (!t.C2 || !t.aux)) return false;
  }
  return true;
}

// Tiles by gemm_cfg: 6 = 128 x 128, 7 = 128 x 64, 8 = 64 x 64 (plan_common.h
// launch_cfg picks one per launch).  OAC_TUNE_FWD_TILE_M / _N force one tile
// for every forward launch (tile sweeps).
int gemm_fwd_tile_m(int cfg) {
  const int v = tuning(OAC_TUNE_FWD_TILE_M);
  return v ? v : cfg == 8 ? 64 : 128;
}
int gemm_fwd_tile_n(int cfg) {
  const int v = tuning(OAC_TUNE_FWD_TILE_N);
  return v ? v : cfg == 6 ? 128 : 64;
}

hipError_t gemm_fwd_launch(const GemmBatch& b, int cfg, hipStream_t s, BatchCache* bc = nullptr, int pos = -1) {
  if (b.total_tiles <= 0) return hipSuccess;
  if (!gemm_fwd_supports(b)) return hipErrorInvalidValue;
  int tb[8];
  for (int i = 0; i < 8; ++i) tb[i] = i < b.ntasks ? b.t[i].tile_begin : 0x7fffffff;
  const int bm = gemm_fwd_tile_m(cfg), bn = gemm_fwd_tile_n(cfg);
  // LDS ring depth: 2 for 128x64 tiles (48 KB: three workgroups per CU;
  // B=4096 SAC layer 0, 768 tiles, 65.6 -> 61.1 us), 3 otherwise (128x128 is
  // register-bound to one workgroup per CU either way); OAC_TUNE_FWD_NB forces one
  const int nb_env = tuning(OAC_TUNE_FWD_NB);
  const int nb = (nb_env == 2 || nb_env == 3) ? nb_env : (bm == 128 && bn == 64) ? 2 : 3;
  const int grid = b.total_tiles + b.rg.blocks;
  const GemmBatch* d = bc ? bc->get(b, pos, s) : nullptr;
#define OAC_FWD(BM_, BN_, NB_) \
  if (bm == BM_ && bn == BN_ && nb == NB_) { \
    if (d) \
      OAC_LAUNCH((gemm_fwd_kernel_dev<BM_, BN_, NB_>), dim3(grid), dim3(256), 0, s, b.total_tiles, \
                 tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], (const GemmBatchG*)d); \
    else \
      OAC_LAUNCH((gemm_fwd_kernel<BM_, BN_, NB_>), dim3(grid), dim3(256), 0, s, b.total_tiles, \
                 tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b); \
    return hipGetLastError(); }
  OAC_FWD(128, 128, 3) OAC_FWD(128, 64, 3) OAC_FWD(64, 128, 3) OAC_FWD(64, 64, 3)
  OAC_FWD(128, 128, 2) OAC_FWD(128, 64, 2) OAC_FWD(64, 64, 2)
#undef OAC_FWD
  return hipErrorInvalidValue;
}

}  // namespace oac
