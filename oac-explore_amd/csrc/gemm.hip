// Grouped fp32 GEMM on CDNA4 fp32-input MFMA (v_mfma_f32_32x32x2_f32).
//
// One launch runs every independent product of an MLP stage (the six
// layer-0 projections, the four layer-1 products, the dW/dX pairs of a
// backward layer, ...) as a list of tasks; the block index selects the task
// and the output tile.  fp32 in / fp32 accumulate: the MFMA result is
// bit-for-bit a k-ordered fmaf chain, so parity with the fp32 CPU reference
// is at the 1e-7 level (no TF32/xf32 exists on gfx950, and bf16 would break
// the 1e-5 gate).
//
// Tile engine: 256 threads = 4 waves.  A and B tiles are staged global ->
// registers -> LDS in k-major layout [k][m] / [k][n] (padded), so every MFMA
// operand fetch is one conflict-free ds_read_b32 per lane (lane l reads
// A[k=l>>5][m=l&31], B[k=l>>5][n=l&31]).  The next K block is prefetched into
// registers while the current one is multiplied (one barrier per K block,
// double-buffered LDS).  Waves tile the output as WM x WN, and WK > 1 splits
// the K loop across waves (for the small-M/N stages of a batch-256 step),
// reduced through LDS in fixed order (deterministic).
#include <cstring>

#include "oac_common.h"
#include "adam_common.h"
#include "kernels.h"

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int BM, int BN, int BK, int WM, int WN, int WK>
struct GemmCfg {
  static constexpr int kBM = BM, kBN = BN, kBK = BK, kWM = WM, kWN = WN, kWK = WK;
  static constexpr int TI = BM / WM / 32;  // 32x32 accumulators per wave (m)
  static constexpr int TJ = BN / WN / 32;  // (n)
  static constexpr int PAD = 1;
  static constexpr int LDA_S = BM + PAD;
  static constexpr int LDB_S = BN + PAD;
  static constexpr int NA = BM * BK / 256;  // staged A floats per thread
  static constexpr int NB = BN * BK / 256;
  static constexpr int STAGE_FLOATS = BK * LDA_S + BK * LDB_S;
  static constexpr int RED_FLOATS = (WK - 1) * WM * WN * TI * TJ * 16 * 64;
  static constexpr int LDS_FLOATS =
      (2 * STAGE_FLOATS > RED_FLOATS) ? 2 * STAGE_FLOATS : RED_FLOATS;
  static_assert(WM * WN * WK == 4, "4 waves");
  static_assert((BM * BK) % 256 == 0 && (BN * BK) % 256 == 0, "staging");
  static_assert(BK % (2 * WK) == 0, "k split");
};

// Staging loads.  Every load of the unrolled loop is issued unconditionally
// (out-of-range elements read a clamped in-bounds address and are zeroed by a
// select), and the per-task layout branches are hoisted around the whole loop,
// so hipcc issues all NA+NB loads back to back and waits once -- a per-element
// branch would make it wait vmcnt(0) per element (one dependent L2 round trip
// per float).
template <class C, bool KC>
__device__ __forceinline__ void idx_mk(int e, int& mn, int& k) {
  if (KC) { k = e % C::kBK; mn = e / C::kBK; }   // walk the contiguous k
  else    { mn = e % C::kBM; k = e / C::kBM; }   // walk the contiguous m / n
}

template <class C, int TILE, bool KC>
__device__ __forceinline__ void idx_tile(int e, int& mn, int& k) {
  if (KC) { k = e % C::kBK; mn = e / C::kBK; }
  else    { mn = e % TILE; k = e / TILE; }
}

template <class C, bool KC, bool RANK1>
__device__ __forceinline__ void load_a_all(const GemmTask& t, int m0, int k0, float (&ra)[C::NA]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < C::NA; ++i) {
    int m, k;
    idx_tile<C, C::kBM, KC>(tid + 256 * i, m, k);
    m += m0; k += k0;
    const bool ok = (m < t.M) & (k < t.K);
    const int row = ok ? (KC ? m : k) : 0;
    const int col = ok ? (KC ? k : m) : 0;
    float v;
    if (!RANK1) {
      v = t.A[(long)row * t.lda + col];
    } else {
      const float mk = t.a_mask[(long)row * t.ld_mask + col];
      const float sv = t.a_s[row] * t.a_v[col];
      v = mk > 0.f ? sv : 0.f;
    }
    ra[i] = ok ? v : 0.f;
  }
}

template <class C, bool KC>
__device__ __forceinline__ void load_b_all(const GemmTask& t, int n0, int k0, float (&rb)[C::NB]) {
  const int tid = threadIdx.x;
  const int nreal = t.b_ones ? t.N - 1 : t.N;
#pragma unroll
  for (int i = 0; i < C::NB; ++i) {
    int n, k;
    idx_tile<C, C::kBN, KC>(tid + 256 * i, n, k);
    n += n0; k += k0;
    const bool ok = (n < nreal) & (k < t.K);
    const int row = ok ? (KC ? n : k) : 0;
    const int col = ok ? (KC ? k : n) : 0;
    const float v = t.B[(long)row * t.ldb + col];
    const bool one = (n == nreal) & (t.b_ones != 0) & (k < t.K);
    rb[i] = ok ? v : (one ? 1.f : 0.f);
  }
}

template <class C>
__device__ __forceinline__ void stage_load(const GemmTask& t, int m0, int n0, int k0,
                                           float (&ra)[C::NA], float (&rb)[C::NB]) {
  if (t.a_mode == A_PLAIN) {
    if (t.a_kc) load_a_all<C, true, false>(t, m0, k0, ra);
    else load_a_all<C, false, false>(t, m0, k0, ra);
  } else {
    if (t.a_kc) load_a_all<C, true, true>(t, m0, k0, ra);
    else load_a_all<C, false, true>(t, m0, k0, ra);
  }
  if (t.b_kc) load_b_all<C, true>(t, n0, k0, rb);
  else load_b_all<C, false>(t, n0, k0, rb);
}

template <class C, bool AKC, bool BKC>
__device__ __forceinline__ void stage_store_t(float* As, float* Bs, const float (&ra)[C::NA],
                                              const float (&rb)[C::NB]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < C::NA; ++i) {
    int m, k;
    idx_tile<C, C::kBM, AKC>(tid + 256 * i, m, k);
    As[k * C::LDA_S + m] = ra[i];
  }
#pragma unroll
  for (int i = 0; i < C::NB; ++i) {
    int n, k;
    idx_tile<C, C::kBN, BKC>(tid + 256 * i, n, k);
    Bs[k * C::LDB_S + n] = rb[i];
  }
}

template <class C>
__device__ __forceinline__ void stage_store(const GemmTask& t, float* As, float* Bs,
                                            const float (&ra)[C::NA], const float (&rb)[C::NB]) {
  if (t.a_kc) {
    if (t.b_kc) stage_store_t<C, true, true>(As, Bs, ra, rb);
    else stage_store_t<C, true, false>(As, Bs, ra, rb);
  } else {
    if (t.b_kc) stage_store_t<C, false, true>(As, Bs, ra, rb);
    else stage_store_t<C, false, false>(As, Bs, ra, rb);
  }
}

template <int EPI>
__device__ __forceinline__ void epi_store(const GemmTask& t, int m, int n, float acc,
                                          const float* lds_u, const float* lds_v, int mt, int nt) {
  if (m >= t.M || n >= t.N) return;
  const long o = (long)m * t.ldc + n;
  if (EPI == EPI_STORE) {
    t.C[o] = acc;
  } else if (EPI == EPI_GRAD) {
    if (t.b_ones && n == t.N - 1) t.bias_grad[m] = acc;
    else t.C[o] = acc;
  } else if (EPI == EPI_BIAS) {
    t.C[o] = acc + t.bias[n];
  } else if (EPI == EPI_BIAS_RELU) {
    t.C[o] = fmaxf(acc + t.bias[n], 0.f);
  } else if (EPI == EPI_BIAS_RANK_RELU) {
    const float p = acc + t.bias[n];
    t.C[o] = p;
    // U / V tile rows staged in LDS by the caller ([row][R], R odd-padded)
    const float* u = lds_u + mt * (t.R | 1);
    const float* v = lds_v + nt * (t.R | 1);
    float s = 0.f;
    for (int j = 0; j < t.R; ++j) s = fmaf(u[j], v[j], s);
    t.C2[(long)m * t.ldc2 + n] = fmaxf(p + s, 0.f);
  } else if (EPI == EPI_ADD_RELU) {
    t.C[o] = fmaxf(acc + t.aux[(long)m * t.ld_aux + n], 0.f);
  } else if (EPI == EPI_MASK) {
    t.C[o] = t.aux[(long)m * t.ld_aux + n] > 0.f ? acc : 0.f;
  }
}

template <class C, int EPI>
__device__ __forceinline__ void epilogue_tile(const GemmTask& t, int m0, int n0, int wm, int wn,
                                              int lane, const floatx16 (&accf)[C::TI][C::TJ],
                                              const float* lds_u, const float* lds_v) {
#pragma unroll
  for (int i = 0; i < C::TI; ++i)
#pragma unroll
    for (int j = 0; j < C::TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int mt = (wm * C::TI + i) * 32 + row;
        const int nt = (wn * C::TJ + j) * 32 + (lane & 31);
        epi_store<EPI>(t, m0 + mt, n0 + nt, accf[i][j][r], lds_u, lds_v, mt, nt);
      }
}

template <class C>
__global__ void __launch_bounds__(256) gemm_grouped_kernel(const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) float lds[C::LDS_FLOATS];

  // task lookup (uniform)
  int ti = 0;
  const int bid = blockIdx.x;
  if (batch.publish && bid == 0 && threadIdx.x == 0)
    publish_step_consts(batch.publish, batch.pub_beta1, batch.pub_beta2);
#pragma unroll 1
  for (int i = 1; i < batch.ntasks; ++i)
    if (bid >= batch.t[i].tile_begin) ti = i;
  GemmTask t = batch.t[ti];
  int local = bid - t.tile_begin;
  if (t.ksplit > 1) {
    // split-K: this block owns K range [split*kchunk, (split+1)*kchunk)
    const int split = local % t.ksplit;
    local /= t.ksplit;
    const int k_lo = split * t.kchunk;
    const int k_hi = min(t.K, k_lo + t.kchunk);
    // shift the k origin of both operands
    if (t.a_mode == A_PLAIN) t.A += t.a_kc ? (long)k_lo : (long)k_lo * t.lda;
    else {
      if (t.a_kc) { t.a_v += k_lo; t.a_mask += k_lo; }
      else { t.a_s += k_lo; t.a_mask += (long)k_lo * t.ld_mask; }
    }
    t.B += t.b_kc ? (long)k_lo : (long)k_lo * t.ldb;
    t.K = k_hi - k_lo;
    t.C += (long)split * t.slab_stride;
    t.bias_grad += (long)split * t.slab_stride;
  }
  const int m0 = (local / t.tiles_n) * C::kBM;
  const int n0 = (local % t.tiles_n) * C::kBN;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wk = wave / (C::kWM * C::kWN);
  const int wmn = wave % (C::kWM * C::kWN);
  const int wm = wmn / C::kWN;
  const int wn = wmn % C::kWN;

  floatx16 acc[C::TI][C::TJ];
#pragma unroll
  for (int i = 0; i < C::TI; ++i)
#pragma unroll
    for (int j = 0; j < C::TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float ra[C::NA], rb[C::NB];
  const int nkb = (t.K + C::kBK - 1) / C::kBK;
  stage_load<C>(t, m0, n0, 0, ra, rb);
  float* buf0 = lds;
  float* buf1 = lds + C::STAGE_FLOATS;
  stage_store<C>(t, buf0, buf0 + C::kBK * C::LDA_S, ra, rb);
  __syncthreads();

  const int lrow = lane >> 5;   // k within the MFMA pair
  const int lcol = lane & 31;
#pragma unroll 1
  for (int kb = 0; kb < nkb; ++kb) {
    float* cur = (kb & 1) ? buf1 : buf0;
    float* nxt = (kb & 1) ? buf0 : buf1;
    if (kb + 1 < nkb) stage_load<C>(t, m0, n0, (kb + 1) * C::kBK, ra, rb);
    const float* As = cur;
    const float* Bs = cur + C::kBK * C::LDA_S;
#pragma unroll
    for (int kk = wk; kk < C::kBK / 2; kk += C::kWK) {
      const int k = 2 * kk + lrow;
      float a[C::TI], b[C::TJ];
#pragma unroll
      for (int i = 0; i < C::TI; ++i)
        a[i] = As[k * C::LDA_S + (wm * C::TI + i) * 32 + lcol];
#pragma unroll
      for (int j = 0; j < C::TJ; ++j)
        b[j] = Bs[k * C::LDB_S + (wn * C::TJ + j) * 32 + lcol];
#pragma unroll
      for (int i = 0; i < C::TI; ++i)
#pragma unroll
        for (int j = 0; j < C::TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kb + 1 < nkb) stage_store<C>(t, nxt, nxt + C::kBK * C::LDA_S, ra, rb);
    __syncthreads();
  }

  if constexpr (C::kWK > 1) {
    // split-K partials -> LDS (lane-contiguous), reduced by the wk==0 waves in
    // fixed order.
    constexpr int per_wave = C::TI * C::TJ * 16 * 64;
    if (wk > 0) {
      float* dst = lds + ((wk - 1) * C::kWM * C::kWN + wmn) * per_wave;
#pragma unroll
      for (int i = 0; i < C::TI; ++i)
#pragma unroll
        for (int j = 0; j < C::TJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) dst[((i * C::TJ + j) * 16 + r) * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (wk == 0) {
#pragma unroll 1
      for (int w = 1; w < C::kWK; ++w) {
        const float* src = lds + ((w - 1) * C::kWM * C::kWN + wmn) * per_wave;
#pragma unroll
        for (int i = 0; i < C::TI; ++i)
#pragma unroll
          for (int j = 0; j < C::TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] += src[((i * C::TJ + j) * 16 + r) * 64 + lane];
      }
    }
  }
  // rank-R epilogue operands (U rows of this M tile, V rows of this N tile)
  // staged through LDS once per tile instead of strided per-element loads
  float* lds_u = lds;
  float* lds_v = lds + C::kBM * (t.R | 1);
  if (t.epi == EPI_BIAS_RANK_RELU) {
    __syncthreads();
    const int Rp = t.R | 1;
    for (int e = threadIdx.x; e < C::kBM * t.R; e += 256) {
      const int r = e / t.R, j = e % t.R;
      const int m = min(m0 + r, t.M - 1);
      lds_u[r * Rp + j] = t.U[(long)m * t.ldu + j];
    }
    for (int e = threadIdx.x; e < C::kBN * t.R; e += 256) {
      const int r = e / t.R, j = e % t.R;
      const int n = min(n0 + r, t.N - 1);
      lds_v[r * Rp + j] = t.V[(long)n * t.ldv + j];
    }
    __syncthreads();
  }
  if (wk != 0) return;
  const floatx16 (&accf)[C::TI][C::TJ] = acc;
  switch (t.epi) {
    case EPI_STORE: epilogue_tile<C, EPI_STORE>(t, m0, n0, wm, wn, lane, accf, lds_u, lds_v); break;
    case EPI_BIAS: epilogue_tile<C, EPI_BIAS>(t, m0, n0, wm, wn, lane, accf, lds_u, lds_v); break;
    case EPI_BIAS_RELU: epilogue_tile<C, EPI_BIAS_RELU>(t, m0, n0, wm, wn, lane, accf, lds_u, lds_v); break;
    case EPI_BIAS_RANK_RELU: epilogue_tile<C, EPI_BIAS_RANK_RELU>(t, m0, n0, wm, wn, lane, accf, lds_u, lds_v); break;
    case EPI_ADD_RELU: epilogue_tile<C, EPI_ADD_RELU>(t, m0, n0, wm, wn, lane, accf, lds_u, lds_v); break;
    case EPI_MASK: epilogue_tile<C, EPI_MASK>(t, m0, n0, wm, wn, lane, accf, lds_u, lds_v); break;
    case EPI_GRAD: epilogue_tile<C, EPI_GRAD>(t, m0, n0, wm, wn, lane, accf, lds_u, lds_v); break;
    default: break;
  }
}

// LDS-tiled kernel (cfg 1, 64x64x32 tiles, 32x32 per wave): the fallback for
// large-batch products the pipelined kernels do not take; cfg 0 is the
// latency-optimised kernel of gemm_small.hip.  (128x128 / 128x64 / 64x128 /
// 64x64x16 variants measured 0.6-1.02x and were retired.)
using CfgLarge = GemmCfg<64, 64, 32, 2, 2, 1>;

hipError_t gemm_fwd_launch(const GemmBatch& b, int cfg, hipStream_t s, BatchCache* bc = nullptr,
                           int pos = -1);
int gemm_fwd_tile_m(int cfg);
int gemm_fwd_tile_n(int cfg);

hipError_t gemm_bwdp_launch(const GemmBatch& b, int cfg, hipStream_t s, BatchCache* bc = nullptr,
                            int pos = -1);
int gemm_bwdp_tile_m(int cfg);
int gemm_bwdp_tile_n(int cfg);

int gemm_tile_m(int cfg) {
  if (cfg >= 9) return gemm_bwdp_tile_m(cfg);
  if (cfg >= 6) return gemm_fwd_tile_m(cfg);
  return cfg == 0 ? 32 : 64;
}
int gemm_tile_n(int cfg) {
  if (cfg >= 9) return gemm_bwdp_tile_n(cfg);
  if (cfg >= 6) return gemm_fwd_tile_n(cfg);
  return cfg == 0 ? 32 : 64;
}

void gemm_small_finalize(GemmBatch& b);
hipError_t gemm_small_launch(const GemmBatch& b, hipStream_t s, BatchCache* bc, int pos);


// Fills tile_begin / tiles_n / total_tiles for a tile configuration.
void gemm_batch_finalize(GemmBatch& b, int cfg) {
  if (cfg == 0) { gemm_small_finalize(b); return; }
  const int bm = gemm_tile_m(cfg), bn = gemm_tile_n(cfg);
  int tiles = 0;
  for (int i = 0; i < b.ntasks; ++i) {
    GemmTask& t = b.t[i];
    const int tm = (t.M + bm - 1) / bm;
    // gemm_bwdp.hip (cfg 9-11): a dW's ones column is not a column tile
    const int nx = (cfg >= 9 && t.epi == EPI_GRAD && t.b_ones) ? t.N - 1 : t.N;
    const int tn = (nx + bn - 1) / bn;
    t.tile_begin = tiles;
    t.tiles_n = tn;
    if (t.ksplit < 1) t.ksplit = 1;
    tiles += tm * tn * t.ksplit;
  }
  b.total_tiles = tiles;
}

hipError_t gemm_batch_launch(const GemmBatch& b, int cfg, hipStream_t s, BatchCache* bc, int pos) {
  if (b.total_tiles <= 0) return hipSuccess;
  if (b.side_adam > 0 && (cfg < 9 || cfg > 17)) return hipErrorInvalidValue;   // side Adam: gemm_bwdp only
  if (b.la_adam && (cfg != 12 || b.total_tiles > kLaTickets))   // last-arrival Adam: gemm_bwdp cfg 12
    return hipErrorInvalidValue;
  // rows read through the direct gather's index slot (a_rows) and the side
  // workgroups that copy the batch / draw eps (rg): only the small kernel and
  // gemm_fwd implement them -- any other kernel would read replay rows 0..M-1
  // and leave the batch copy and eps unwritten
  bool gathers = b.rg.ring != nullptr;
  for (int i = 0; i < b.ntasks; ++i) gathers = gathers || b.t[i].a_rows;
  if (gathers && cfg != 0 && (cfg < 6 || cfg > 8)) return hipErrorInvalidValue;
  for (int i = 0; i < b.ntasks; ++i)   // folded reductions (GemmTask::fold): the small kernel only,
    if (b.t[i].fold && (cfg != 0 || b.t[i].ksplit > 1 || b.t[i].b_ones || b.t[i].a_kc ||
                        b.t[i].a_mode != A_RANK1_MASK || b.t[i].epi != EPI_GRAD))   // unsplit
      return hipErrorInvalidValue;
  if (cfg == 0) return gemm_small_launch(b, s, bc, pos);
  if (b.fuse_adam) return hipErrorInvalidValue;   // fused optimizer: small-batch kernel only
  for (int i = 0; i < b.ntasks; ++i) {             // dual products / head backward: small kernel
    if (b.t[i].K2 > 0 || b.t[i].epi == EPI_HEAD_BWD) return hipErrorInvalidValue;
    // the width-1 head dot: small kernel or gemm_fwd (6-8)
    if (b.t[i].epi == EPI_BIAS_RELU_DOT && (cfg < 6 || cfg > 8)) return hipErrorInvalidValue;
  }
  if (cfg >= 9) return gemm_bwdp_launch(b, cfg, s, bc, pos);
  if (cfg >= 6) return gemm_fwd_launch(b, cfg, s, bc, pos);
  if (cfg != 1) return hipErrorInvalidValue;
  OAC_LAUNCH(gemm_grouped_kernel<CfgLarge>, dim3(b.total_tiles), dim3(256), 0, s, b);
  return hipGetLastError();
}

}  // namespace oac
