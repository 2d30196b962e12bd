// Large-batch backward products on the LDS-DMA pipeline (gemm_cfg 9 / 10 /
// 11: 128x64 / 64x64 / 128x128 workgroup tiles): dX = dY W (dY k-contiguous,
// possibly a rank-1 seed s[m] v[k] through a ReLU mask; W n-contiguous) and
// dW = dY^T [X | 1] (both operands batch-major, dY possibly rank-1 masked),
// split-K slabs as the other kernels write them.
//
// Same pipeline as the forward kernel (gemm_pipe.h, gemm_fwd.hip): 2 x 2 waves
// of (BM/2) x (BN/2) v_mfma_f32_32x32x2_f32 blocks, 32-deep K stages in a
// three-stage LDS ring filled by global_load_lds_dwordx4.  A k-contiguous
// operand is staged as in the forward kernel ([row][32 k], 16-byte chunks
// swizzled by the row, one ds_read_b128 per 4 k); a batch-major operand as
// the rows of its k range ([32 k][BM or BN], lane-linear: one 1-KB LDS-DMA
// instruction per 2 or 4 k-rows) and read with one ds_read_b32 per k, the 32
// lanes of a half-wave on 32 consecutive columns.  The rank-1 factors indexed
// by k (v of a dX seed, s of a dW seed) are copied into LDS once per
// workgroup; those indexed by the output row sit in registers.
//
// dW's ones column (the bias gradient) is not a 32-wide MFMA block: the waves
// at the first column block sum their A fragments on the VALU (4 adds per 4
// MFMAs) and store the row sums, so the column tiles cover the N - 1 real
// columns only (a 257-wide dW is 4 tiles of 64, not 5).
#include <cstdlib>

#include "oac_common.h"
#include "kernels.h"
#include "gemm_epilogue.h"
#include "gemm_pipe.h"
#include "adam_common.h"

namespace oac {

#ifdef OAC_PIPE_CLOCK
#define gemm_bwdp_kernel gemm_bwdp_kernel_clk   // distinct from the library's kernels of the same names
#define gemm_bwdp_kernel_dev gemm_bwdp_kernel_dev_clk
#endif

enum PKind { PK_KC = 0, PK_KC_R1 = 1, PK_MN = 2, PK_MN_R1 = 3 };

constexpr int kVec = 1024;   // LDS floats for a rank-1 factor indexed by k
// consecutive tile ids per XCD: a dW's 16 (m, n) tiles of one K chunk (256 x
// 256 at 64 x 64), a dX's 4 row blocks of 4 column tiles
constexpr int kBwdXcdChunk = 16;

template <int BM, int BN, int NB = kFBuf>
struct BwdG {
  static constexpr int WM = BM / 64, WN = BN / 64;
  static constexpr int PA = BM / 32, PB = BN / 32;   // LDS-DMA instructions per wave and stage
  static constexpr int LPW = PA + PB;
  static constexpr int STAGE = (BM + BN) * kFK;
  static constexpr int LDS = NB * STAGE + kVec;      // ring of NB stages + the rank-1 vector
};

// one operand's LDS-DMA sources.  KC: ROWS x 32 k, 8 rows per instruction,
// lane j -> row 8p + j / 8, chunk (j % 8) ^ kc_swz(row).  MN: 32 k x ROWS,
// 256 / ROWS k-rows per instruction, lane j -> k-row p RP + j / (ROWS / 4),
// columns 4 (j % (ROWS / 4)) .. + 3.
template <bool KC, int ROWS>
struct PSrc {
  static constexpr int P = ROWS / 32;
  const float* row[P];   // KC: the operand row; MN: the column base (row 0)
  int off[P];            // KC: chunk offset in floats; MN: k-row within the stage
  long ld;

  __device__ __forceinline__ void init(const float* base, long ld_, int r0, int rmax, int wave,
                                       int lane) {
    ld = ld_;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int p = wave * P + q;
      if (KC) {
        const int r = 8 * p + (lane >> 3);
        off[q] = 4 * ((lane & 7) ^ kc_swz(r));
        row[q] = base + (long)min(r0 + r, rmax - 1) * ld_;
      } else {
        constexpr int LPR = ROWS / 4;             // lanes per k-row
        off[q] = p * (256 / ROWS) + lane / LPR;
        const int col = r0 + 4 * (lane % LPR);
        row[q] = base + (col < rmax ? col : 0);   // a chunk wholly past the columns reads column 0
      }
    }
  }
  // stage kst .. kst + 31 into dst (an operand image of the stage); rows
  // k >= k_hi read row kst as a stand-in (the fix-ups zero them).  (A source
  // kept per lane and advanced by one stage per issue, instead of the multiply
  // by ld, measured 0.3-1 % slower in the step on two boxes, round 6.)
  __device__ __forceinline__ void issue(int kst, int k_hi, float* dst, int wave) const {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int k = kst + off[q];
      const float* src = KC ? row[q] + (k < k_hi ? k : kst) : row[q] + (long)(k < k_hi ? k : kst) * ld;
      glds16(src, dst + (wave * P + q) * 256);
    }
  }
};

// fragment values of k = kst + 8g + 4 half + c (c = 0..3) at operand row rr
// (stage-relative: 0 .. ROWS-1) of an LDS image
template <bool KC, int ROWS>
__device__ __forceinline__ float4 pfrag(const float* img, int rr, int g, int half) {
  if (KC) {
    const int slot = 4 * ((2 * g + half) ^ kc_swz(rr));
    return *reinterpret_cast<const float4*>(img + rr * kFK + slot);
  } else {
    const float* p = img + (8 * g + 4 * half) * ROWS + rr;
    return make_float4(p[0], p[ROWS], p[2 * ROWS], p[3 * ROWS]);
  }
}

__device__ __forceinline__ float f4c(const float4& v, int c) {
  return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}

// acc += A . B over k in [k_lo, k_hi) for one workgroup tile; bsum: row sums
// of A (the dW ones column) when ones
template <int BM, int BN, int AK, int NB>
__device__ __forceinline__ void bwdp_pipe(const GemmTask& t, int m0, int n0, int nx, int k_lo,
                                          int k_hi, bool ones, float* lds, float* vec,
                                          floatx16 (&acc)[BM / 64][BN / 64], float (&bsum)[BM / 64]) {
  using G = BwdG<BM, BN, NB>;
  constexpr int WM = G::WM, WN = G::WN;
  constexpr bool AKC = AK == PK_KC || AK == PK_KC_R1;
  constexpr bool AR1 = AK == PK_KC_R1 || AK == PK_MN_R1;
  const int lane = threadIdx.x & 63, l32 = lane & 31, half = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kb0 = k_lo & ~7;
  const int nst = (k_hi - kb0 + kFK - 1) / kFK;
  PSrc<AKC, BM> sa;
  PSrc<false, BN> sb;
  sa.init(AR1 ? t.a_mask : t.A, AR1 ? t.ld_mask : t.lda, m0, t.M, wave, lane);
  sb.init(t.B, t.ldb, n0, nx, wave, lane);
  const int ar = (wave >> 1) * (BM / 2) + l32, br = (wave & 1) * (BN / 2) + l32;
  // the ring's first two stages are in flight before the rank-1 factors are
  // requested, so their round trips overlap (the factors' waits also cover
  // the two stages: both were issued before them)
  sa.issue(kb0, k_hi, lds, wave);
  sb.issue(kb0, k_hi, lds + BM * kFK, wave);
  if (NB == 3 && nst > 1) {
    sa.issue(kb0 + kFK, k_hi, lds + G::STAGE, wave);
    sb.issue(kb0 + kFK, k_hi, lds + G::STAGE + BM * kFK, wave);
  }
  // rank-1 factors: the one indexed by k into LDS (kb0-relative), the one
  // indexed by the output row into registers
  float fm[WM];
#pragma unroll
  for (int i = 0; i < WM; ++i) fm[i] = 0.f;
  if (AR1) {
    const float* fk = AK == PK_KC_R1 ? t.a_v : t.a_s;   // KC_R1: v[k]; MN_R1: s[k]
    const float* fr = AK == PK_KC_R1 ? t.a_s : t.a_v;   // KC_R1: s[m]; MN_R1: v[m]
    const int n = nst * kFK;
    for (int i = threadIdx.x; i < n; i += 256) {
      const int k = kb0 + i;
      vec[i] = (k >= k_lo && k < k_hi) ? fk[k] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      fm[i] = fr[min(m0 + (wave >> 1) * (BM / 2) + 32 * i + l32, t.M - 1)];
      asm volatile("" ::"v"(fm[i]));   // consumed here: the wait stays out of the loop
    }
    // every wave's DMA and factor loads done (the compiler does not count
    // the DMA) and its vec stores in LDS, then vec is complete for all
    wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
  }
  PIPE_CLK(1);
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    if (NB == 3 && st + 1 < nst) wait_vm<G::LPW>();
    else wait_vm<0>();
    raw_barrier();   // stage st landed for every wave; stage st - 1 is read by all
    PIPE_CLK(2 + st);
    if (st + NB - 1 < nst) {
      float* nb = lds + ((st + NB - 1) % NB) * G::STAGE;
      sa.issue(kb0 + (st + NB - 1) * kFK, k_hi, nb, wave);
      sb.issue(kb0 + (st + NB - 1) * kFK, k_hi, nb + BM * kFK, wave);
    }
    const int kst = kb0 + st * kFK;
    const float* as = lds + (st % NB) * G::STAGE;
    const float* bs = as + BM * kFK;
    const bool mask = kst < k_lo || kst + kFK > k_hi;
    // the whole stage's fragments first (one LDS round trip per stage, not
    // one per 8-deep group), then the VALU fix-ups, then the MFMA run
    constexpr int NG = kFK / 8;
    float4 af[NG][WM], bf[NG][WN], kv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
      for (int i = 0; i < WM; ++i) af[g][i] = pfrag<AKC, BM>(as, ar + 32 * i, g, half);
#pragma unroll
      for (int j = 0; j < WN; ++j) bf[g][j] = pfrag<false, BN>(bs, br + 32 * j, g, half);
      if (AR1) kv[g] = *reinterpret_cast<const float4*>(vec + st * kFK + 8 * g + 4 * half);
    }
    // per 8-deep group: the VALU fix-ups of group g + 1 can issue while the
    // MFMAs of group g run (the fragments of every group are already in flight)
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (mask) {   // k outside [k_lo, k_hi): zero both operands (the staged rows there are stand-ins)
        const int k = kst + 8 * g + 4 * half;
        const bool o0 = k >= k_lo && k < k_hi, o1 = k + 1 >= k_lo && k + 1 < k_hi;
        const bool o2 = k + 2 >= k_lo && k + 2 < k_hi, o3 = k + 3 >= k_lo && k + 3 < k_hi;
#pragma unroll
        for (int i = 0; i < WM; ++i) {
          af[g][i].x = o0 ? af[g][i].x : 0.f; af[g][i].y = o1 ? af[g][i].y : 0.f;
          af[g][i].z = o2 ? af[g][i].z : 0.f; af[g][i].w = o3 ? af[g][i].w : 0.f;
        }
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          bf[g][j].x = o0 ? bf[g][j].x : 0.f; bf[g][j].y = o1 ? bf[g][j].y : 0.f;
          bf[g][j].z = o2 ? bf[g][j].z : 0.f; bf[g][j].w = o3 ? bf[g][j].w : 0.f;
        }
      }
      if (AR1) {   // the rank-1 seed through its ReLU mask: fm (row factor) x kv (k factor)
#pragma unroll
        for (int i = 0; i < WM; ++i) {
          af[g][i].x = af[g][i].x > 0.f ? fm[i] * kv[g].x : 0.f;
          af[g][i].y = af[g][i].y > 0.f ? fm[i] * kv[g].y : 0.f;
          af[g][i].z = af[g][i].z > 0.f ? fm[i] * kv[g].z : 0.f;
          af[g][i].w = af[g][i].w > 0.f ? fm[i] * kv[g].w : 0.f;
        }
      }
      if (ones) {
#pragma unroll
        for (int i = 0; i < WM; ++i)
          bsum[i] += (af[g][i].x + af[g][i].y) + (af[g][i].z + af[g][i].w);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(af[g][i], c), f4c(bf[g][j], c),
                                                             acc[i][j], 0, 0, 0);
    }
  }
}

constexpr unsigned kEpiBwd = (1u << EPI_STORE) | (1u << EPI_MASK) | (1u << EPI_GRAD);

template <int BM, int BN, int AK, int NB>
__device__ __forceinline__ void bwdp_tile(const GemmBatch& batch, int ti, int local, float* lds) {
  using G = BwdG<BM, BN, NB>;
  constexpr int WM = G::WM, WN = G::WN;
  GemmTask t = batch.t[ti];
  int k_lo = 0, k_hi = t.K;
  if (t.ksplit > 1) {
    // split-major: the (m, n) tiles of one K chunk have consecutive ids, so
    // the XCD mapping (xcd_tile_rr) puts tiles that share that chunk's rows
    // of both operands on one XCD, where its L2 serves the re-reads
    const int per = ((t.M + BM - 1) / BM) * t.tiles_n;
    const int split = local / per;
    local -= split * per;
    k_lo = split * t.kchunk;
    k_hi = min(t.K, k_lo + t.kchunk);
    t.C += (long)split * t.slab_stride;
    t.bias_grad += (long)split * t.slab_stride;
  }
  // dW with the ones column: tiles over the N - 1 real columns, bias by row sums
  const bool grad_ones = t.epi == EPI_GRAD && t.b_ones;
  const int nx = grad_ones ? t.N - 1 : t.N;
  const int m0 = (local / t.tiles_n) * BM;
  const int n0 = (local % t.tiles_n) * BN;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mw = m0 + (wave >> 1) * (BM / 2), nw = n0 + (wave & 1) * (BN / 2);
  const bool ones = grad_ones && nw == 0;   // wave-uniform
  floatx16 acc[WM][WN];
  float bsum[WM];
#pragma unroll
  for (int i = 0; i < WM; ++i) {
    bsum[i] = 0.f;
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  }
  PIPE_CLK(0);
  bwdp_pipe<BM, BN, AK, NB>(t, m0, n0, nx, k_lo, k_hi, ones, lds, lds + NB * G::STAGE, acc, bsum);
  PIPE_CLK(29);
  if (grad_ones) {
    t.N = nx;
    t.b_ones = 0;
    if (ones) {   // both half-waves summed their k's of the same rows
      const int lane = threadIdx.x & 63;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const float s = bsum[i] + __shfl_xor(bsum[i], 32);
        const int m = mw + 32 * i + lane;
        if (lane < 32 && m < t.M) t.bias_grad[m] = s;
      }
    }
  }
  rd_epilogue<WM, WN, kEpiBwd>(t, mw, nw, acc, false);
  PIPE_CLK(30);
  PIPE_CLK(31);
}

template <int BM, int BN, int NB>
__device__ __forceinline__ void gemm_bwdp_body(int total_tiles, int tb1, int tb2, int tb3, int tb4,
                                               int tb5, int tb6, int tb7, const GemmBatch& batch,
                                               float* lds) {
  if (batch.publish && blockIdx.x == 0 && threadIdx.x == 0)
    publish_step_consts(batch.publish, batch.pub_beta1, batch.pub_beta2);
  const int side0 = batch.side_first ? 0 : total_tiles;   // side workgroups: the flat Adam
  const int tile0 = batch.side_first ? batch.side_adam : 0;  // (GemmBatch::side_adam)
  if ((int)blockIdx.x >= side0 && (int)blockIdx.x < side0 + batch.side_adam) {
    adam_side_block(batch, blockIdx.x - side0, batch.side_adam);
    return;
  }
  const int bid = xcd_tile_rr<kBwdXcdChunk>(blockIdx.x - tile0, total_tiles);
  int ti = 0;
  ti = bid >= tb1 ? 1 : ti; ti = bid >= tb2 ? 2 : ti; ti = bid >= tb3 ? 3 : ti;
  ti = bid >= tb4 ? 4 : ti; ti = bid >= tb5 ? 5 : ti; ti = bid >= tb6 ? 6 : ti;
  ti = bid >= tb7 ? 7 : ti;
  ti = __builtin_amdgcn_readfirstlane(ti);
  const GemmTask& t = batch.t[ti];
  const int local = bid - t.tile_begin;
  const int ak = (t.a_kc ? PK_KC : PK_MN) + (t.a_mode == A_RANK1_MASK ? 1 : 0);
  switch (ak) {
    case PK_KC: bwdp_tile<BM, BN, PK_KC, NB>(batch, ti, local, lds); break;
    case PK_KC_R1: bwdp_tile<BM, BN, PK_KC_R1, NB>(batch, ti, local, lds); break;
    case PK_MN: bwdp_tile<BM, BN, PK_MN, NB>(batch, ti, local, lds); break;
    default: bwdp_tile<BM, BN, PK_MN_R1, NB>(batch, ti, local, lds); break;
  }
}

// waves per SIMD the registers must allow so that the 2-stage ring's LDS sets
// the workgroups per CU: 64x64 tiles (36 KB) four, 128x64 (52 KB) three,
// 128x128 (68 KB) two
template <int BM, int BN, int NB>
__global__ void __launch_bounds__(256, NB == 2 ? (BM == 128 && BN == 128 ? 2 : BM == 128 ? 3 : 4) : 1)
gemm_bwdp_kernel(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                 const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) float lds[BwdG<BM, BN, NB>::LDS];
  gemm_bwdp_body<BM, BN, NB>(total_tiles, tb1, tb2, tb3, tb4, tb5, tb6, tb7, batch, lds);
}
// the batch in device memory (kernels.h BatchCache)
template <int BM, int BN, int NB>
__global__ void __launch_bounds__(256, NB == 2 ? (BM == 128 && BN == 128 ? 2 : BM == 128 ? 3 : 4) : 1)
gemm_bwdp_kernel_dev(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                     const GemmBatchG* __restrict__ bp) {
  __shared__ __attribute__((aligned(16))) float lds[BwdG<BM, BN, NB>::LDS];
  gemm_bwdp_body<BM, BN, NB>(total_tiles, tb1, tb2, tb3, tb4, tb5, tb6, tb7, *(const GemmBatch*)bp, lds);
}

// a backward batch this kernel takes: dX (A k-contiguous, B n-contiguous) or dW
// (both batch-major) products, plain or rank-1-mask A, STORE / MASK / GRAD
// epilogues, no second product; a rank-1 factor indexed by k fits the LDS
// vector (dX: K <= 1024; dW: the split chunk)
bool gemm_bwdp_supports(const GemmBatch& b) {
  if (b.fuse_adam || b.ntasks < 1) return false;
  for (int i = 0; i < b.ntasks; ++i) {
    const GemmTask& t = b.t[i];
    if (t.b_kc || t.K2 > 0 || t.a_rows) return false;
    if (t.epi != EPI_STORE && t.epi != EPI_MASK && t.epi != EPI_GRAD) return false;
    if (t.epi == EPI_GRAD && t.a_kc) return false;
    if (t.epi != EPI_GRAD && t.ksplit > 1) return false;
    if (t.b_ones && (t.epi != EPI_GRAD || t.N < 2)) return false;
    const int span = (t.ksplit > 1 ? t.kchunk : t.K) + 8 + kFK;
    if (t.a_mode == A_RANK1_MASK && span > kVec) return false;
  }
  return true;
}

int gemm_bwdp_tile_m(int cfg) { return cfg == 10 || cfg == 12 ? 64 : 128; }
int gemm_bwdp_tile_n(int cfg) { return cfg == 11 || cfg == 13 ? 128 : 64; }

hipError_t gemm_bwdp_launch(const GemmBatch& b, int cfg, hipStream_t s, BatchCache* bc = nullptr, int pos = -1) {
  if (b.total_tiles <= 0) return hipSuccess;
  if (!gemm_bwdp_supports(b)) return hipErrorInvalidValue;
  int tb[8];
  for (int i = 0; i < 8; ++i) tb[i] = i < b.ntasks ? b.t[i].tile_begin : 0x7fffffff;
  const GemmBatch* d = bc ? bc->get(b, pos, s) : nullptr;
#define OAC_BWDP(C_, BM_, BN_, NB_) \
  if (cfg == C_) { \
    if (d) \
      OAC_LAUNCH((gemm_bwdp_kernel_dev<BM_, BN_, NB_>), dim3(b.total_tiles + b.side_adam), dim3(256), 0, s, \
                 b.total_tiles, tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], (const GemmBatchG*)d); \
    else \
      OAC_LAUNCH((gemm_bwdp_kernel<BM_, BN_, NB_>), dim3(b.total_tiles + b.side_adam), dim3(256), 0, s, \
                 b.total_tiles, tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b); \
    return hipGetLastError(); }
  // cfg 12: 64x64 tiles on a 2-stage ring (36 KB of LDS: four workgroups per CU)
  OAC_BWDP(9, 128, 64, 3) OAC_BWDP(10, 64, 64, 3) OAC_BWDP(11, 128, 128, 3) OAC_BWDP(12, 64, 64, 2)
  OAC_BWDP(13, 128, 128, 2) OAC_BWDP(14, 128, 64, 2)
#undef OAC_BWDP
  return hipErrorInvalidValue;
}

}  // namespace oac
