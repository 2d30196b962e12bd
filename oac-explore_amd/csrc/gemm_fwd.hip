// Large-batch forward products (gemm_cfg 6): Y = X W^T (+ b, ReLU; the
// critic's rank-Da action columns as a continuation of the same accumulators)
// at B >= 1024, both operands k-contiguous.
//
// The register-direct forward kernel (gemm_big.hip, cfg 2) spends one 16-byte
// global load per lane for every 4 MFMAs of each 32x32 block it owns; on the
// B=4096 step its launches keep the TA (vector address) unit ~70 % busy at
// 43 % of the MFMA peak (tools/pmc_bwd.sh), so the load path, not the MFMA
// pipe, bounds them.  Here a 256-thread workgroup stages TM x 32 of X and
// TN x 32 of W per K stage into LDS with 16-byte loads (once per workgroup,
// not once per wave), keeping the k-contiguous layout ([row][k], rows padded to
// 36 floats: ds_write_b128 / ds_read_b128 without bank conflicts), and each
// wave reads its fragments with one ds_read_b128 per 32x32 block and 4 k, the
// same lane layout the register-direct kernels use (k = 8g + 4 half + c).
// Double-buffered: the next stage's global loads are in flight while the
// current stage's 64 MFMAs per wave issue; one barrier per stage.
#include <cstdlib>

#include "oac_common.h"
#include "kernels.h"
#include "adam_common.h"

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

constexpr int kFwdKD = 32;          // k per stage
constexpr int kFwdRow = kFwdKD + 4; // LDS row stride (floats)

template <int TM, int TN>
struct FwdGeom {
  static constexpr int WM = TM / 64, WN = TN / 64;         // 32x32 blocks per wave (2 x 2 waves)
  static constexpr int PA = TM * kFwdKD / (4 * 256);       // float4 per thread per stage, A
  static constexpr int PB = TN * kFwdKD / (4 * 256);
  static constexpr int floats = 2 * (TM + TN) * kFwdRow;
};

__device__ __forceinline__ int fwd_acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// acc += A[m0 + .., k_lo..k_hi) . B[n0 + .., k_lo..k_hi)^T over this wave's blocks
template <int TM, int TN>
__device__ __forceinline__ void fwd_loop(const float* A, long lda, int M, const float* B, long ldb,
                                         int N, int k_lo, int k_hi, int m0, int n0, float* lds,
                                         floatx16 (&acc)[TM / 64][TN / 64]) {
  using G = FwdGeom<TM, TN>;
  constexpr int WM = G::WM, WN = G::WN, PA = G::PA, PB = G::PB;
  const int nst = (k_hi - k_lo + kFwdKD - 1) / kFwdKD;
  if (nst <= 0) return;
  float* As[2] = {lds, lds + TM * kFwdRow};
  float* Bs[2] = {lds + 2 * TM * kFwdRow, lds + 2 * TM * kFwdRow + TN * kFwdRow};
  const int t = threadIdx.x, lane = t & 63, l32 = lane & 31, half = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // staging map: float4 e = t + 256 q -> row e / 8, k 4 (e % 8)
  const float* arow[PA];
  const float* brow[PB];
  bool aok[PA], bok[PB];
#pragma unroll
  for (int q = 0; q < PA; ++q) {
    const int r = (t + 256 * q) >> 3;
    aok[q] = m0 + r < M;
    arow[q] = A + (long)(aok[q] ? m0 + r : 0) * lda;
  }
#pragma unroll
  for (int q = 0; q < PB; ++q) {
    const int r = (t + 256 * q) >> 3;
    bok[q] = n0 + r < N;
    brow[q] = B + (long)(bok[q] ? n0 + r : 0) * ldb;
  }
  const int kq = 4 * (t & 7);
  f4u ra[PA], rb[PB];
  auto gload = [&](int k0) {
    const int k = k0 + kq;
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      f4u v = *reinterpret_cast<const f4u*>(arow[q] + k);
      if (!aok[q] || k + 4 > k_hi) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = (aok[q] && k + c < k_hi) ? v[c] : 0.f;
      }
      ra[q] = v;
    }
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      f4u v = *reinterpret_cast<const f4u*>(brow[q] + k);
      if (!bok[q] || k + 4 > k_hi) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = (bok[q] && k + c < k_hi) ? v[c] : 0.f;
      }
      rb[q] = v;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int r = (t + 256 * q) >> 3;
      *reinterpret_cast<float4*>(As[buf] + r * kFwdRow + kq) = make_float4(ra[q][0], ra[q][1], ra[q][2], ra[q][3]);
    }
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int r = (t + 256 * q) >> 3;
      *reinterpret_cast<float4*>(Bs[buf] + r * kFwdRow + kq) = make_float4(rb[q][0], rb[q][1], rb[q][2], rb[q][3]);
    }
  };
  // The loads read up to 3 floats past k_hi inside a row (masked): every
  // operand buffer is followed by >= 8 readable floats (gemm_operand.h).
  gload(k_lo);
  sstore(0);
  __syncthreads();
  const int ar0 = (TM / 2) * wm + l32, br0 = (TN / 2) * wn + l32;
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    const bool more = st + 1 < nst;
    if (more) gload(k_lo + (st + 1) * kFwdKD);
    const float* ab = As[cur];
    const float* bb = Bs[cur];
#pragma unroll
    for (int g = 0; g < kFwdKD / 8; ++g) {
      const int kk = 8 * g + 4 * half;
      float4 af[WM], bf[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i) af[i] = *reinterpret_cast<const float4*>(ab + (ar0 + 32 * i) * kFwdRow + kk);
#pragma unroll
      for (int j = 0; j < WN; ++j) bf[j] = *reinterpret_cast<const float4*>(bb + (br0 + 32 * j) * kFwdRow + kk);
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
    if (more) sstore(cur ^ 1);
    __syncthreads();
  }
}

template <int TM, int TN>
__device__ __forceinline__ void fwd_epilogue(const GemmTask& t, int m0, int n0,
                                             const floatx16 (&acc)[TM / 64][TN / 64], bool second) {
  constexpr int WM = TM / 64, WN = TN / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int mw = m0 + (TM / 2) * (wave >> 1), nw = n0 + (TN / 2) * (wave & 1);
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int n = nw + 32 * j + (lane & 31);
    if (n >= t.N) continue;
    const float bias = t.bias ? t.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mw + 32 * i + fwd_acc_row(r, lane);
        if (m >= t.M) continue;
        const float v = acc[i][j][r] + bias;
        switch (t.epi) {
          case EPI_STORE: t.C[(long)m * t.ldc + n] = acc[i][j][r]; break;
          case EPI_BIAS: t.C[(long)m * t.ldc + n] = v; break;
          case EPI_BIAS_RELU: t.C[(long)m * t.ldc + n] = fmaxf(v, 0.f); break;
          case EPI_BIAS_RANK_RELU:
            if (!second) t.C[(long)m * t.ldc + n] = v;
            else t.C2[(long)m * t.ldc2 + n] = fmaxf(v, 0.f);
            break;
          default: break;
        }
      }
  }
}

template <int TM, int TN>
__global__ void __launch_bounds__(256)
gemm_fwd_kernel(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                const GemmBatch batch) {
  constexpr int WM = TM / 64, WN = TN / 64;
  __shared__ __attribute__((aligned(16))) float lds[FwdGeom<TM, TN>::floats];
  const int bid = blockIdx.x;
  if (batch.publish && bid == 0 && threadIdx.x == 0)
    publish_step_consts(batch.publish, batch.pub_beta1, batch.pub_beta2);
  if (bid >= total_tiles) return;
  int ti = 0;
  ti = bid >= tb1 ? 1 : ti; ti = bid >= tb2 ? 2 : ti; ti = bid >= tb3 ? 3 : ti;
  ti = bid >= tb4 ? 4 : ti; ti = bid >= tb5 ? 5 : ti; ti = bid >= tb6 ? 6 : ti;
  ti = bid >= tb7 ? 7 : ti;
  ti = __builtin_amdgcn_readfirstlane(ti);
  const GemmTask& t = batch.t[ti];
  const int local = bid - t.tile_begin;
  const int m0 = (local / t.tiles_n) * TM;
  const int n0 = (local % t.tiles_n) * TN;
  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  fwd_loop<TM, TN>(t.A, t.lda, t.M, t.B, t.ldb, t.N, 0, t.K, m0, n0, lds, acc);
  fwd_epilogue<TM, TN>(t, m0, n0, acc, false);
  if (t.epi == EPI_BIAS_RANK_RELU) {   // + U V^T on the same accumulators
    if (t.U == t.A + t.K && t.ldu == t.lda && t.V == t.B + t.K && t.ldv == t.ldb)
      fwd_loop<TM, TN>(t.A, t.lda, t.M, t.B, t.ldb, t.N, t.K, t.K + t.R, m0, n0, lds, acc);
    else
      fwd_loop<TM, TN>(t.U, t.ldu, t.M, t.V, t.ldv, t.N, 0, t.R, m0, n0, lds, acc);
    fwd_epilogue<TM, TN>(t, m0, n0, acc, true);
  }
}

// forward batches this kernel takes: both operands k-contiguous, plain A, no
// split, no second product, bias / ReLU / rank epilogues
bool gemm_fwd_supports(const GemmBatch& b) {
  if (b.fuse_adam || b.ntasks < 1) return false;
  for (int i = 0; i < b.ntasks; ++i) {
    const GemmTask& t = b.t[i];
    if (!t.a_kc || !t.b_kc || t.a_mode != A_PLAIN || t.ksplit > 1 || t.K2 > 0) return false;
    if (t.epi != EPI_STORE && t.epi != EPI_BIAS && t.epi != EPI_BIAS_RELU &&
        t.epi != EPI_BIAS_RANK_RELU)
      return false;
    if (t.epi == EPI_BIAS_RANK_RELU && !t.C2) return false;
  }
  return true;
}

// OAC_FWD2_TILE: 128 (128 x 128 tiles, default) or 64 (128 x 64)
int gemm_fwd_tile_n() {
  static const int v = [] { const char* e = getenv("OAC_FWD2_TILE"); return (e && atoi(e) == 64) ? 64 : 128; }();
  return v;
}

hipError_t gemm_fwd_launch(const GemmBatch& b, hipStream_t s) {
  if (b.total_tiles <= 0) return hipSuccess;
  if (!gemm_fwd_supports(b)) return hipErrorInvalidValue;
  int tb[8];
  for (int i = 0; i < 8; ++i) tb[i] = i < b.ntasks ? b.t[i].tile_begin : 0x7fffffff;
  if (gemm_fwd_tile_n() == 64)
    OAC_LAUNCH((gemm_fwd_kernel<128, 64>), dim3(b.total_tiles), dim3(256), 0, s, b.total_tiles,
               tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b);
  else
    OAC_LAUNCH((gemm_fwd_kernel<128, 128>), dim3(b.total_tiles), dim3(256), 0, s, b.total_tiles,
               tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b);
  return hipGetLastError();
}

}  // namespace oac
