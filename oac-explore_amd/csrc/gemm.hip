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
#include "oac_common.h"

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

__device__ __forceinline__ float load_a(const GemmTask& t, int m, int k) {
  if (m >= t.M || k >= t.K) return 0.f;
  const int row = t.a_kc ? m : k;
  const int col = t.a_kc ? k : m;
  if (t.a_mode == A_PLAIN) return t.A[(long)row * t.lda + col];
  const float mk = t.a_mask[(long)row * t.ld_mask + col];
  return mk > 0.f ? t.a_s[row] * t.a_v[col] : 0.f;
}

__device__ __forceinline__ float load_b(const GemmTask& t, int k, int n) {
  if (n >= t.N || k >= t.K) return 0.f;
  if (t.b_ones && n == t.N - 1) return 1.f;
  return t.b_kc ? t.B[(long)n * t.ldb + k] : t.B[(long)k * t.ldb + n];
}

template <class C>
__device__ __forceinline__ void stage_load(const GemmTask& t, int m0, int n0, int k0,
                                           float (&ra)[C::NA], float (&rb)[C::NB]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < C::NA; ++i) {
    const int e = tid + 256 * i;
    int m, k;
    if (t.a_kc) { k = e % C::kBK; m = e / C::kBK; }   // walk the contiguous k
    else        { m = e % C::kBM; k = e / C::kBM; }   // walk the contiguous m
    ra[i] = load_a(t, m0 + m, k0 + k);
  }
#pragma unroll
  for (int i = 0; i < C::NB; ++i) {
    const int e = tid + 256 * i;
    int n, k;
    if (t.b_kc) { k = e % C::kBK; n = e / C::kBK; }
    else        { n = e % C::kBN; k = e / C::kBN; }
    rb[i] = load_b(t, k0 + k, n0 + n);
  }
}

template <class C>
__device__ __forceinline__ void stage_store(const GemmTask& t, float* As, float* Bs,
                                            const float (&ra)[C::NA], const float (&rb)[C::NB]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < C::NA; ++i) {
    const int e = tid + 256 * i;
    int m, k;
    if (t.a_kc) { k = e % C::kBK; m = e / C::kBK; }
    else        { m = e % C::kBM; k = e / C::kBM; }
    As[k * C::LDA_S + m] = ra[i];
  }
#pragma unroll
  for (int i = 0; i < C::NB; ++i) {
    const int e = tid + 256 * i;
    int n, k;
    if (t.b_kc) { k = e % C::kBK; n = e / C::kBK; }
    else        { n = e % C::kBN; k = e / C::kBN; }
    Bs[k * C::LDB_S + n] = rb[i];
  }
}

__device__ __forceinline__ void epilogue_elem(const GemmTask& t, int m, int n, float acc) {
  if (m >= t.M || n >= t.N) return;
  switch (t.epi) {
    case EPI_STORE:
      t.C[(long)m * t.ldc + n] = acc;
      break;
    case EPI_BIAS:
      t.C[(long)m * t.ldc + n] = acc + t.bias[n];
      break;
    case EPI_BIAS_RELU:
      t.C[(long)m * t.ldc + n] = fmaxf(acc + t.bias[n], 0.f);
      break;
    case EPI_BIAS_RANK_RELU: {
      const float p = acc + t.bias[n];
      t.C[(long)m * t.ldc + n] = p;
      const float* u = t.U + (long)m * t.ldu;
      const float* v = t.V + (long)n * t.ldv;
      float s = 0.f;
      for (int j = 0; j < t.R; ++j) s = fmaf(u[j], v[j], s);
      t.C2[(long)m * t.ldc2 + n] = fmaxf(p + s, 0.f);
      break;
    }
    case EPI_ADD_RELU:
      t.C[(long)m * t.ldc + n] = fmaxf(acc + t.aux[(long)m * t.ld_aux + n], 0.f);
      break;
    case EPI_MASK:
      t.C[(long)m * t.ldc + n] = t.aux[(long)m * t.ld_aux + n] > 0.f ? acc : 0.f;
      break;
    case EPI_SLAB:
      t.C[(long)m * t.ldc + n] = acc;   // C already offset to this split's slab
      break;
    default:
      break;
  }
}

template <class C>
__global__ void __launch_bounds__(256) gemm_grouped_kernel(const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) float lds[C::LDS_FLOATS];

  // task lookup (uniform)
  int ti = 0;
  const int bid = blockIdx.x;
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
  if (wk != 0) return;

#pragma unroll
  for (int i = 0; i < C::TI; ++i)
#pragma unroll
    for (int j = 0; j < C::TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int m = m0 + (wm * C::TI + i) * 32 + row;
        const int n = n0 + (wn * C::TJ + j) * 32 + lcol;
        epilogue_elem(t, m, n, acc[i][j][r]);
      }
}

// Small tiles + split-K over the 4 waves: batch-256 stages (few output tiles,
// long K).  Large tiles: batch-4096 stages.
using CfgSmall = GemmCfg<32, 32, 64, 1, 1, 4>;
using CfgLarge = GemmCfg<64, 64, 32, 2, 2, 1>;

int gemm_tile_m(int cfg) { return cfg == 0 ? CfgSmall::kBM : CfgLarge::kBM; }
int gemm_tile_n(int cfg) { return cfg == 0 ? CfgSmall::kBN : CfgLarge::kBN; }

// Fills tile_begin / tiles_n / total_tiles for a tile configuration.
void gemm_batch_finalize(GemmBatch& b, int cfg) {
  const int bm = gemm_tile_m(cfg), bn = gemm_tile_n(cfg);
  int tiles = 0;
  for (int i = 0; i < b.ntasks; ++i) {
    GemmTask& t = b.t[i];
    const int tm = (t.M + bm - 1) / bm;
    const int tn = (t.N + bn - 1) / bn;
    t.tile_begin = tiles;
    t.tiles_n = tn;
    if (t.ksplit < 1) t.ksplit = 1;
    tiles += tm * tn * t.ksplit;
  }
  b.total_tiles = tiles;
}

hipError_t gemm_batch_launch(const GemmBatch& b, int cfg, hipStream_t s) {
  if (b.total_tiles <= 0) return hipSuccess;
  if (cfg == 0)
    hipLaunchKernelGGL(gemm_grouped_kernel<CfgSmall>, dim3(b.total_tiles), dim3(256), 0, s, b);
  else
    hipLaunchKernelGGL(gemm_grouped_kernel<CfgLarge>, dim3(b.total_tiles), dim3(256), 0, s, b);
  return hipGetLastError();
}

}  // namespace oac
