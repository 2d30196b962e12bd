// Large-batch backward products on the LDS-DMA pipeline: dX = dY W (dY
// k-contiguous, possibly a rank-1 seed s[m] v[k] through a ReLU mask; W
// n-contiguous) and dW = dY^T [X | 1] (both operands batch-major, dY possibly
// rank-1 masked), split-K slabs as the other kernels write them.  Tile
// configurations (gemm_cfg): 12 = 64x64 tiles on a 2-stage ring (the
// default), 9 / 10 / 11 = 128x64 / 64x64 / 128x128 on 3-stage rings, 13 / 14 =
// 128x128 / 128x64 on 2-stage rings, 15 = 64x64 with 16-deep stages on a
// 4-stage ring, 17 = cfg 12 software-pipelined; cfg 12 with the last-arrival
// Adam (GemmBatch::la_adam) is an instance of its own.
//
// Same pipeline as the forward kernel (gemm_pipe.h, gemm_fwd.hip): 2 x 2 waves
// of (BM/2) x (BN/2) v_mfma_f32_32x32x2_f32 blocks, FK-deep K stages (32, or
// 16) in an NB-stage LDS ring filled by global_load_lds_dwordx4.  A k-contiguous
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

// FK: k per stage (32: 128-byte row pieces; 16: 64-byte ones on a deeper ring
// in the same LDS -- NB - 1 stages in flight ahead of the one computed, so a
// stage's DMA has (NB - 1) x FK/2 MFMAs of one wave to land in, not FK/2)
template <int BM, int BN, int NB = kFBuf, int FK = kFK>
struct BwdG {
  static constexpr int WM = BM / 64, WN = BN / 64;
  // LDS-DMA instructions per wave and stage (1 KB each, 4 waves)
  static constexpr int PA = BM * FK / 1024, PB = BN * FK / 1024;
  static constexpr int LPW = PA + PB;
  static constexpr int STAGE = (BM + BN) * FK;
  static constexpr int LDS = NB * STAGE + kVec;      // ring of NB stages + the rank-1 vector
  // workgroups per CU the LDS allows; the registers are bounded to match
  // (the 3-stage 32-deep rings keep their unbounded register allocation)
  static constexpr int OCC = (NB == 3 && FK == 32) ? 1 : 163840 / (LDS * 4);
  static_assert(PA >= 1 && PB >= 1 && PA * 1024 == BM * FK && PB * 1024 == BN * FK, "stage split");
};

// chunk swizzle of a k-contiguous image with FK-float rows (gemm_pipe.h
// kc_swz for FK = 32): a 16-lane ds_read_b128 group's rows (FK = 32: 2 rows
// per 64 banks, FK = 16: 4) take distinct (row mod, slot) pairs
template <int FK>
__device__ __forceinline__ int kc_swz_k(int r) {
  return FK == 32 ? kc_swz(r) : (r >> 2) & 3;
}

// one operand's LDS-DMA sources.  KC: ROWS x FK k, 1024 / (4 FK) rows per
// instruction, lane j -> row (64 / LR) p + j / LR (LR = FK / 4 lanes per row),
// chunk (j % LR) ^ kc_swz_k(row).  MN: FK k x ROWS, 256 / ROWS k-rows per
// instruction, lane j -> k-row p RP + j / (ROWS / 4), columns 4 (j % (ROWS / 4)) .. + 3.
template <bool KC, int ROWS, int FK = kFK>
struct PSrc {
  static constexpr int P = ROWS * FK / 1024;
  static constexpr int LR = FK / 4;
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
        const int r = (64 / LR) * p + lane / LR;
        off[q] = 4 * ((lane % LR) ^ kc_swz_k<FK>(r));
        row[q] = base + (long)min(r0 + r, rmax - 1) * ld_;
      } else {
        constexpr int LPR = ROWS / 4;             // lanes per k-row
        off[q] = p * (256 / ROWS) + lane / LPR;
        const int col = r0 + 4 * (lane % LPR);
        row[q] = base + (col < rmax ? col : 0);   // a chunk wholly past the columns reads column 0
      }
    }
  }
  // stage kst .. kst + FK - 1 into dst (an operand image of the stage); rows
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
template <bool KC, int ROWS, int FK>
__device__ __forceinline__ float4 pfrag(const float* img, int rr, int g, int half) {
  if (KC) {
    const int slot = 4 * ((2 * g + half) ^ kc_swz_k<FK>(rr));
    return *reinterpret_cast<const float4*>(img + rr * FK + slot);
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
// stage st landed for this wave: `ahead` later stages (at most NB - 2) may
// still be in flight
template <int LPW, int NB>
__device__ __forceinline__ void wait_stage(int ahead) {
  if (NB >= 4 && ahead >= 2) wait_vm<2 * LPW>();
  else if (NB >= 3 && ahead >= 1) wait_vm<LPW>();
  else wait_vm<0>();
}

// one stage's operand fragments in registers: groups of 8 k (4 per half-wave)
template <int BM, int BN, int FK>
struct BwdFrag {
  static constexpr int NG = FK / 8, WM = BM / 64, WN = BN / 64;
  float4 af[NG][WM], bf[NG][WN], kv[NG];
};

// fragments of groups [G0, G1) of the stage image at `as` (A) / as + BM FK (B)
template <int BM, int BN, int AK, int FK, int G0, int G1, bool KVU = false>
__device__ __forceinline__ void bwdp_load(BwdFrag<BM, BN, FK>& f, const float* as, const float* vst,
                                          int ar, int br, int half) {
  constexpr bool AKC = AK == PK_KC || AK == PK_KC_R1;
  constexpr bool AR1 = AK == PK_KC_R1 || AK == PK_MN_R1;
  const float* bs = as + BM * FK;
#pragma unroll
  for (int g = G0; g < G1; ++g) {
#pragma unroll
    for (int i = 0; i < BM / 64; ++i) f.af[g][i] = pfrag<AKC, BM, FK>(as, ar + 32 * i, g, half);
#pragma unroll
    for (int j = 0; j < BN / 64; ++j) f.bf[g][j] = pfrag<false, BN, FK>(bs, br + 32 * j, g, half);
    if (AR1 && !KVU) f.kv[g] = *reinterpret_cast<const float4*>(vst + 8 * g + 4 * half);
  }
}

// the VALU fix-ups and the MFMA run of groups [G0, G1) of the stage at k = kst
// (KVU: the rank-1 k factor read from LDS here, at its use, instead of with
// the fragments -- fewer registers for the software-pipelined loop)
template <int BM, int BN, int AK, int FK, int G0, int G1, bool KVU = false>
__device__ __forceinline__ void bwdp_mma(BwdFrag<BM, BN, FK>& f, int kst, int k_lo, int k_hi,
                                         bool mask, bool ones, int half, const float (&fm)[BM / 64],
                                         floatx16 (&acc)[BM / 64][BN / 64], float (&bsum)[BM / 64],
                                         const float* vst = nullptr) {
  constexpr int WM = BM / 64, WN = BN / 64;
  constexpr bool AR1 = AK == PK_KC_R1 || AK == PK_MN_R1;
#pragma unroll
  for (int g = G0; g < G1; ++g) {
    if (AR1 && KVU) f.kv[g] = *reinterpret_cast<const float4*>(vst + 8 * g + 4 * half);
    if (mask) {   // k outside [k_lo, k_hi): zero both operands (the staged rows there are stand-ins)
      const int k = kst + 8 * g + 4 * half;
      const bool o0 = k >= k_lo && k < k_hi, o1 = k + 1 >= k_lo && k + 1 < k_hi;
      const bool o2 = k + 2 >= k_lo && k + 2 < k_hi, o3 = k + 3 >= k_lo && k + 3 < k_hi;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        f.af[g][i].x = o0 ? f.af[g][i].x : 0.f; f.af[g][i].y = o1 ? f.af[g][i].y : 0.f;
        f.af[g][i].z = o2 ? f.af[g][i].z : 0.f; f.af[g][i].w = o3 ? f.af[g][i].w : 0.f;
      }
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        f.bf[g][j].x = o0 ? f.bf[g][j].x : 0.f; f.bf[g][j].y = o1 ? f.bf[g][j].y : 0.f;
        f.bf[g][j].z = o2 ? f.bf[g][j].z : 0.f; f.bf[g][j].w = o3 ? f.bf[g][j].w : 0.f;
      }
    }
    if (AR1) {   // the rank-1 seed through its ReLU mask: fm (row factor) x kv (k factor)
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        f.af[g][i].x = f.af[g][i].x > 0.f ? fm[i] * f.kv[g].x : 0.f;
        f.af[g][i].y = f.af[g][i].y > 0.f ? fm[i] * f.kv[g].y : 0.f;
        f.af[g][i].z = f.af[g][i].z > 0.f ? fm[i] * f.kv[g].z : 0.f;
        f.af[g][i].w = f.af[g][i].w > 0.f ? fm[i] * f.kv[g].w : 0.f;
      }
    }
    if (ones) {
#pragma unroll
      for (int i = 0; i < WM; ++i)
        bsum[i] += (f.af[g][i].x + f.af[g][i].y) + (f.af[g][i].z + f.af[g][i].w);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(f.af[g][i], c), f4c(f.bf[g][j], c),
                                                           acc[i][j], 0, 0, 0);
  }
}

template <int BM, int BN, int AK, int FK>
__device__ __forceinline__ void bwdp_load1(BwdFrag<BM, BN, FK>& f, int g, const float* as, const float* vst,
                                           int ar, int br, int half) {
  if (g == 1) bwdp_load<BM, BN, AK, FK, 1, 2, true>(f, as, vst, ar, br, half);
  if (FK >= 24 && g == 2) bwdp_load<BM, BN, AK, FK, 2, 3, true>(f, as, vst, ar, br, half);
  if (FK >= 32 && g == 3) bwdp_load<BM, BN, AK, FK, 3, 4, true>(f, as, vst, ar, br, half);
}
template <int BM, int BN, int AK, int FK>
__device__ __forceinline__ void bwdp_mma1(BwdFrag<BM, BN, FK>& f, int g, int kst, int k_lo, int k_hi,
                                          bool mask, bool ones, int half, const float (&fm)[BM / 64],
                                          floatx16 (&acc)[BM / 64][BN / 64], float (&bsum)[BM / 64],
                                          const float* vst) {
  if (g == 1) bwdp_mma<BM, BN, AK, FK, 1, 2, true>(f, kst, k_lo, k_hi, mask, ones, half, fm, acc, bsum, vst);
  if (FK >= 24 && g == 2)
    bwdp_mma<BM, BN, AK, FK, 2, 3, true>(f, kst, k_lo, k_hi, mask, ones, half, fm, acc, bsum, vst);
  if (FK >= 32 && g == 3)
    bwdp_mma<BM, BN, AK, FK, 3, 4, true>(f, kst, k_lo, k_hi, mask, ones, half, fm, acc, bsum, vst);
}

template <int BM, int BN, int AK, int NB, int FK, bool SWP>
__device__ __forceinline__ void bwdp_pipe(const GemmTask& t, int m0, int n0, int nx, int k_lo,
                                          int k_hi, bool ones, float* lds, float* vec,
                                          floatx16 (&acc)[BM / 64][BN / 64], float (&bsum)[BM / 64]) {
  using G = BwdG<BM, BN, NB, FK>;
  constexpr int WM = G::WM;
  constexpr bool AKC = AK == PK_KC || AK == PK_KC_R1;
  constexpr bool AR1 = AK == PK_KC_R1 || AK == PK_MN_R1;
  const int lane = threadIdx.x & 63, l32 = lane & 31, half = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kb0 = k_lo & ~7;
  const int nst = (k_hi - kb0 + FK - 1) / FK;
  PSrc<AKC, BM, FK> sa;
  PSrc<false, BN, FK> sb;
  sa.init(AR1 ? t.a_mask : t.A, AR1 ? t.ld_mask : t.lda, m0, t.M, wave, lane);
  sb.init(t.B, t.ldb, n0, nx, wave, lane);
  const int ar = (wave >> 1) * (BM / 2) + l32, br = (wave & 1) * (BN / 2) + l32;
  // the ring's first NB - 1 stages are in flight before the rank-1 factors
  // are requested, so their round trips overlap (the factors' waits also
  // cover those stages: all were issued before them)
#pragma unroll
  for (int q = 0; q < NB - 1; ++q) {
    if (q == 0 || q < nst) {
      sa.issue(kb0 + q * FK, k_hi, lds + q * G::STAGE, wave);
      sb.issue(kb0 + q * FK, k_hi, lds + q * G::STAGE + BM * FK, wave);
    }
  }
  // rank-1 factors: the one indexed by k into LDS (kb0-relative), the one
  // indexed by the output row into registers
  float fm[WM];
#pragma unroll
  for (int i = 0; i < WM; ++i) fm[i] = 0.f;
  if (AR1) {
    const float* fk = AK == PK_KC_R1 ? t.a_v : t.a_s;   // KC_R1: v[k]; MN_R1: s[k]
    const float* fr = AK == PK_KC_R1 ? t.a_s : t.a_v;   // KC_R1: s[m]; MN_R1: v[m]
    const int n = nst * FK;
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
  constexpr int NG = FK / 8;
  if (SWP) {
    // software-pipelined: stage st + 1's fragments are read from LDS during
    // stage st's MFMA run (its barrier after the first group), so the LDS
    // round trip and the barrier overlap the MFMAs instead of preceding them;
    // the MFMA order per accumulator is the plain loop's (bitwise equal)
    using F = BwdFrag<BM, BN, FK>;
    F f0, f1;
    wait_stage<G::LPW, NB>(min(NB - 2, nst - 1));
    raw_barrier();
    PIPE_CLK(2);
    if (NB - 1 < nst) {
      float* nb = lds + (NB - 1) * G::STAGE;
      sa.issue(kb0 + (NB - 1) * FK, k_hi, nb, wave);
      sb.issue(kb0 + (NB - 1) * FK, k_hi, nb + BM * FK, wave);
    }
    bwdp_load<BM, BN, AK, FK, 0, NG, true>(f0, lds, vec, ar, br, half);
    auto step = [&](int st, F& cur, F& nxt) {
      const int kst = kb0 + st * FK;
      const bool mask = kst < k_lo || kst + FK > k_hi;
      const bool more = st + 1 < nst;
      const float* as = lds + ((st + 1) % NB) * G::STAGE;
      const float* vs = vec + (st + 1) * FK;
      const float* vc = vec + st * FK;
      bwdp_mma<BM, BN, AK, FK, 0, 1, true>(cur, kst, k_lo, k_hi, mask, ones, half, fm, acc, bsum, vc);
      __builtin_amdgcn_sched_barrier(0);
      if (more) {
        // this stage's LDS reads all returned (its buffer is refilled below)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        wait_stage<G::LPW, NB>(min(NB - 2, nst - 2 - st));
        raw_barrier();   // stage st + 1 landed for every wave; stage st is read by all
        PIPE_CLK(3 + st);
        if (st + NB < nst) {
          float* nb = lds + (st % NB) * G::STAGE;
          sa.issue(kb0 + (st + NB) * FK, k_hi, nb, wave);
          sb.issue(kb0 + (st + NB) * FK, k_hi, nb + BM * FK, wave);
        }
        bwdp_load<BM, BN, AK, FK, 0, 1, true>(nxt, as, vs, ar, br, half);
      }
      // group g's MFMAs, then the next stage's group g into the registers
      // they free (one group of registers beyond one stage's)
#pragma unroll
      for (int g = 1; g < NG; ++g) {
        // (scheduling fences: the compiler would otherwise hoist the next
        // stage's reads above the MFMAs and spill)
        __builtin_amdgcn_sched_barrier(0);
        bwdp_mma1<BM, BN, AK, FK>(cur, g, kst, k_lo, k_hi, mask, ones, half, fm, acc, bsum, vc);
        __builtin_amdgcn_sched_barrier(0);
        if (more) bwdp_load1<BM, BN, AK, FK>(nxt, g, as, vs, ar, br, half);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
#pragma unroll 1
    for (int st = 0; st < nst; st += 2) {
      step(st, f0, f1);
      if (st + 1 < nst) step(st + 1, f1, f0);
    }
    return;
  }
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    wait_stage<G::LPW, NB>(min(NB - 2, nst - 1 - st));
    raw_barrier();   // stage st landed for every wave; stage st - 1 is read by all
    PIPE_CLK(2 + st);
    if (st + NB - 1 < nst) {
      float* nb = lds + ((st + NB - 1) % NB) * G::STAGE;
      sa.issue(kb0 + (st + NB - 1) * FK, k_hi, nb, wave);
      sb.issue(kb0 + (st + NB - 1) * FK, k_hi, nb + BM * FK, wave);
    }
    const int kst = kb0 + st * FK;
    const float* as = lds + (st % NB) * G::STAGE;
    const bool mask = kst < k_lo || kst + FK > k_hi;
    // the whole stage's fragments first (one LDS round trip per stage, not
    // one per 8-deep group), then per 8-deep group the VALU fix-ups (those of
    // group g + 1 can issue while the MFMAs of group g run) and the MFMA run
    BwdFrag<BM, BN, FK> f;
    bwdp_load<BM, BN, AK, FK, 0, NG>(f, as, vec + st * FK, ar, br, half);
    bwdp_mma<BM, BN, AK, FK, 0, NG>(f, kst, k_lo, k_hi, mask, ones, half, fm, acc, bsum);
  }
}

constexpr unsigned kEpiBwd = (1u << EPI_STORE) | (1u << EPI_MASK) | (1u << EPI_GRAD);

// Last-arrival Adam (GemmBatch::la_adam).  Element i of the group (index from
// adam.gslab): its S split-K slabs summed as adam_flat_kernel sums them
// (slab_chunk: chunks of kSlabChunk in slab order, the chunk sums in order),
// read write-through (agent scope: the other splits' workgroups stored them
// write-through and arrived after their stores drained), then
// adam_flat_finish's update -- the same bits as the Adam launch.
__device__ __forceinline__ void la_elem(const AdamConsts& c, const AdamArgs& a, long i, int S) {
  const float* gs = a.gslab + i;
  const long ss = a.slab_stride;
  float g = 0.f;
#pragma unroll 1
  for (int k0 = 0; k0 < S; k0 += kSlabChunk) {
    float x[kSlabChunk];
#pragma unroll
    for (int j = 0; j < kSlabChunk; ++j)   // the chunk's loads in flight together
      x[j] = k0 + j < S ? __hip_atomic_load(const_cast<float*>(gs + (long)(k0 + j) * ss), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)
                        : 0.f;
    float cs = x[0];
#pragma unroll
    for (int j = 1; j < kSlabChunk; ++j)
      if (k0 + j < S) cs += x[j];
    g = k0 == 0 ? cs : g + cs;
  }
  a.g[i] = g;
  if (a.gscale != 1.f) g *= a.gscale;
  float p = a.p[i], m = a.m[i], v = a.v[i];
  adam1(c, p, g, m, v);
  a.p[i] = p; a.m[i] = m; a.v[i] = v;
  if (c.polyak) a.target[i] = polyak1(c, a.target[i], p);
}

// The arrival of a dW tile's split (every wave's write-through stores
// drained first); the last of the t.ksplit arrivals updates the tile's
// elements: rows [m0, m0 + BM) x columns [n0, n0 + BN) of the weight (ldc),
// and the bias rows when the tile owns the ones column (n0 == 0)
template <int BM, int BN>
__device__ __forceinline__ void la_tail(const GemmBatch& batch, const GemmTask& t, int tile, int m0,
                                        int n0, int nx, bool grad_ones, const float* c0,
                                        const float* bg0) {
  __shared__ unsigned la_prev;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* ticket = batch.la_ticket + t.tile_begin + tile;
  if (threadIdx.x == 0)
    la_prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (la_prev != (unsigned)(t.ksplit - 1)) return;
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const AdamArgs& a = batch.adam;
  const AdamConsts c = adam_consts(a.state, a.advance, a.lr, a.beta1, a.beta2, a.eps, a.target,
                                   a.tau, a.period);
  const int S = t.ksplit;
  const long wb = c0 - a.gslab;
  const int n = n0 + (threadIdx.x & 63);
  if (n < nx) {
#pragma unroll 1
    for (int r = threadIdx.x >> 6; r < BM; r += 4) {
      const int m = m0 + r;
      if (m < t.M) la_elem(c, a, wb + (long)m * t.ldc + n, S);
    }
  }
  if (grad_ones && n0 == 0 && (int)threadIdx.x < BM && m0 + (int)threadIdx.x < t.M)
    la_elem(c, a, (bg0 - a.gslab) + m0 + threadIdx.x, S);
  if (batch.la_book && tile == 0 && threadIdx.x == 0) step_bookkeeping_lead(a.state, a.alpha, a.advance);
}

template <int BM, int BN, int AK, int NB, int FK, bool SWP, bool LA>
__device__ __forceinline__ void bwdp_tile(const GemmBatch& batch, int ti, int local, float* lds) {
  using G = BwdG<BM, BN, NB, FK>;
  constexpr int WM = G::WM, WN = G::WN;
  GemmTask t = batch.t[ti];
  const float* c0 = t.C;
  const float* bg0 = t.bias_grad;
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
  bwdp_pipe<BM, BN, AK, NB, FK, SWP>(t, m0, n0, nx, k_lo, k_hi, ones, lds, lds + NB * G::STAGE, acc, bsum);
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
        if (lane < 32 && m < t.M) {
          if (LA) __hip_atomic_store(t.bias_grad + m, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else t.bias_grad[m] = s;
        }
      }
    }
  }
  rd_epilogue<WM, WN, kEpiBwd, LA>(t, mw, nw, acc, false);
  if (LA && t.epi == EPI_GRAD) la_tail<BM, BN>(batch, t, local, m0, n0, nx, grad_ones, c0, bg0);
  PIPE_CLK(30);
  PIPE_CLK(31);
}

template <int BM, int BN, int NB, int FK, bool SWP, bool LA = false>
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
    case PK_KC: bwdp_tile<BM, BN, PK_KC, NB, FK, SWP, LA>(batch, ti, local, lds); break;
    case PK_KC_R1: bwdp_tile<BM, BN, PK_KC_R1, NB, FK, SWP, LA>(batch, ti, local, lds); break;
    case PK_MN: bwdp_tile<BM, BN, PK_MN, NB, FK, SWP, LA>(batch, ti, local, lds); break;
    default: bwdp_tile<BM, BN, PK_MN_R1, NB, FK, SWP, LA>(batch, ti, local, lds); break;
  }
}

// waves per SIMD the registers must allow so that the ring's LDS sets the
// workgroups per CU (BwdG::OCC; the software-pipelined loop: 64x64 only): 64x64 tiles on a 2-stage 32-deep ring or a
// 4-stage 16-deep one (36 KB) four, 128x64 (52 KB) three, 128x128 (68 KB) two
template <int BM, int BN, int NB, int FK, bool SWP, bool LA = false>
__global__ void __launch_bounds__(256, (SWP ? 4 : BwdG<BM, BN, NB, FK>::OCC))
gemm_bwdp_kernel(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                 const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) float lds[BwdG<BM, BN, NB, FK>::LDS];
  gemm_bwdp_body<BM, BN, NB, FK, SWP, LA>(total_tiles, tb1, tb2, tb3, tb4, tb5, tb6, tb7, batch, lds);
}
// the batch in device memory (kernels.h BatchCache)
template <int BM, int BN, int NB, int FK, bool SWP, bool LA = false>
__global__ void __launch_bounds__(256, (SWP ? 4 : BwdG<BM, BN, NB, FK>::OCC))
gemm_bwdp_kernel_dev(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                     const GemmBatchG* __restrict__ bp) {
  __shared__ __attribute__((aligned(16))) float lds[BwdG<BM, BN, NB, FK>::LDS];
  gemm_bwdp_body<BM, BN, NB, FK, SWP, LA>(total_tiles, tb1, tb2, tb3, tb4, tb5, tb6, tb7, *(const GemmBatch*)bp,
                                          lds);
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

int gemm_bwdp_tile_m(int cfg) { return cfg == 10 || cfg == 12 || cfg == 15 || cfg == 17 ? 64 : 128; }
int gemm_bwdp_tile_n(int cfg) { return cfg == 11 || cfg == 13 ? 128 : 64; }

hipError_t gemm_bwdp_launch(const GemmBatch& b, int cfg, hipStream_t s, BatchCache* bc = nullptr, int pos = -1) {
  if (b.total_tiles <= 0) return hipSuccess;
  if (!gemm_bwdp_supports(b)) return hipErrorInvalidValue;
  int tb[8];
  for (int i = 0; i < 8; ++i) tb[i] = i < b.ntasks ? b.t[i].tile_begin : 0x7fffffff;
  const GemmBatch* d = bc ? bc->get(b, pos, s) : nullptr;
#define OAC_BWDP_LA(C_, BM_, BN_, NB_, FK_, SWP_, LA_) \
  if (cfg == C_) { \
    if (d) \
      OAC_LAUNCH((gemm_bwdp_kernel_dev<BM_, BN_, NB_, FK_, SWP_, LA_>), dim3(b.total_tiles + b.side_adam), \
                 dim3(256), 0, s, b.total_tiles, tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], \
                 (const GemmBatchG*)d); \
    else \
      OAC_LAUNCH((gemm_bwdp_kernel<BM_, BN_, NB_, FK_, SWP_, LA_>), dim3(b.total_tiles + b.side_adam), \
                 dim3(256), 0, s, b.total_tiles, tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b); \
    return hipGetLastError(); }
#define OAC_BWDP(C_, BM_, BN_, NB_, FK_, SWP_) OAC_BWDP_LA(C_, BM_, BN_, NB_, FK_, SWP_, false)
  // the last-arrival Adam: its own instance of the default tiles (the
  // write-through stores and the tail stay out of every other kernel)
  if (b.la_adam) {
    OAC_BWDP_LA(12, 64, 64, 2, 32, false, true)
    return hipErrorInvalidValue;
  }
  // cfg 12: 64x64 tiles on a 2-stage ring (36 KB of LDS: four workgroups per CU)
  // cfg 15: 64x64 tiles on a 4-stage 16-deep ring (the LDS of cfg 12, three
  // stages in flight instead of one); cfg 17: cfg 12 software-pipelined
  // (bwdp_pipe SWP).  Neither beat cfg 12 in the step.
  OAC_BWDP(9, 128, 64, 3, 32, false) OAC_BWDP(10, 64, 64, 3, 32, false)
  OAC_BWDP(11, 128, 128, 3, 32, false) OAC_BWDP(12, 64, 64, 2, 32, false)
  OAC_BWDP(13, 128, 128, 2, 32, false) OAC_BWDP(14, 128, 64, 2, 32, false)
  OAC_BWDP(15, 64, 64, 4, 16, false) OAC_BWDP(17, 64, 64, 2, 32, true)
#undef OAC_BWDP
#undef OAC_BWDP_LA
  return hipErrorInvalidValue;
}

}  // namespace oac
