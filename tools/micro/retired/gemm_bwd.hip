// Large-batch backward products (gemm_cfg 5): dX = dY W and dW = dY^T [X | 1]
// at B >= 1024, with the batch-major operands fetched two columns per lane
// and the K range of a workgroup split over its four waves.
//
// gemm_big.hip feeds a batch-major (m- or n-contiguous) operand one dword per
// lane and k: 2-3 KB of loads per 4 MFMAs of a 32x32 wave block, and a rank-1
// seed s.v.1[h>0] costs a third stream for v.  Here
//   * every wave computes the workgroup's whole 64 x 64 tile as 2 x 2 blocks of
//     v_mfma_f32_32x32x2_f32; a batch-major operand is read as float2 per lane
//     -- lane l holds columns 2(l&31) and 2(l&31)+1, block i takes the i-th of
//     them -- so one 8-byte load per lane feeds both blocks of that side;
//     a k-contiguous operand (dY of dX) stays one 16-byte load per block and
//     4 k;
//   * the rank-1 factor indexed by k is lane-uniform per half-wave and comes
//     through scalar loads; the factor indexed by m is held per lane;
//   * the four waves take four quarters of the workgroup's K range (so a
//     split-K dW needs 4x fewer slabs for the same number of waves in flight)
//     and are summed in LDS in a fixed tree ((w0 + w1) + (w2 + w3)):
//     deterministic, independent of timing.
// Per 8-deep k-group a wave issues 4 (+4) loads for 16 MFMAs instead of 8-12
// loads for 4.
#include <cstdlib>

#include "oac_common.h"
#include "kernels.h"
#include "adam_common.h"

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));

enum BwdA { BA_KC = 0, BA_KC_R1 = 1, BA_MN = 2, BA_MN_R1 = 3 };


// raw operand fragments of one 8-deep k-group (lane: k = 8g + 4*half + c)
struct BwdFrag {
  float a[2][4];   // [block][c]  (KC: the 16-byte row segment; MN: float2 per c)
  float b[2][4];   // [block][c]
};

__device__ __forceinline__ int acc_row_b(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

template <int AK, int kBwdPF>   // kBwdPF: k-groups in flight per wave
__device__ __forceinline__ void bwd_tile(GemmTask t, int local, float* red) {
  // XCD-aware order: a task's block range is padded to a multiple of 8 and
  // starts on a multiple of 8, so blocks local, local + 8, ... share an XCD
  // (round-robin placement; speed only, never correctness).  Each XCD takes a
  // contiguous run of the (split-major) work list: the K chunks of a split-K
  // dW land on one XCD with all their tiles, and its L2 serves the chunk's
  // operand rows to every tile instead of each XCD fetching them.
  const int T = ((t.M + 63) >> 6) * t.tiles_n;
  const int S = t.ksplit > 1 ? t.ksplit : 1;
  const int per = (T * S + 7) >> 3;
  const int lin = (local & 7) * per + (local >> 3);
  if (lin >= T * S) return;
  local = lin % T;
  int k_lo = 0, k_hi = t.K;
  if (t.ksplit > 1) {
    const int split = lin / T;
    k_lo = split * t.kchunk;
    k_hi = min(t.K, k_lo + t.kchunk);
    t.C += (long)split * t.slab_stride;
    t.bias_grad += (long)split * t.slab_stride;
  }
  const int lane = threadIdx.x & 63, l32 = lane & 31, half = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mt = (local / t.tiles_n) * 64;
  const int nt = (local % t.tiles_n) * 64;
  // this wave's quarter of [k_lo, k_hi), in whole k-groups
  const int q = (((k_hi - k_lo + 3) / 4) + 7) & ~7;
  const int wk_lo = min(k_hi, k_lo + wave * q), wk_hi = min(k_hi, wk_lo + q);
  const bool a_mn = AK == BA_MN || AK == BA_MN_R1;
  const bool r1 = AK == BA_KC_R1 || AK == BA_MN_R1;

  // ---- per-lane operand setup
  // A rows: KC m_i = mt + 32 i + l32 ; MN m_i = mt + 2 l32 + i
  const int M = t.M;
  int am[2];
  bool av[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    am[i] = a_mn ? mt + 2 * l32 + i : mt + 32 * i + l32;
    av[i] = am[i] < M;
  }
  const float* abase = r1 ? t.a_mask : t.A;
  const long lda = r1 ? t.ld_mask : t.lda;
  const float* arow[2];   // KC: row pointers
  const float* acol = abase + (av[0] ? (a_mn ? mt + 2 * l32 : 0) : 0);   // MN: column pair base
#pragma unroll
  for (int i = 0; i < 2; ++i) arow[i] = abase + (long)(av[i] ? am[i] : 0) * lda;
  float af[2] = {1.f, 1.f};   // rank-1 factor indexed by m (KC: s[m]; MN: v[m])
  if (r1)
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = av[i] ? (a_mn ? t.a_v[am[i]] : t.a_s[am[i]]) : 0.f;
  const float* kfac = a_mn ? t.a_s : t.a_v;   // rank-1 factor indexed by k (lane-uniform per half)
  // B columns n_j = nt + 2 l32 + j ; ones column at n == N - 1 when b_ones
  const int nl = t.b_ones ? t.N - 1 : t.N;
  const int bn0 = nt + 2 * l32;
  bool bv[2], bo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    bv[j] = bn0 + j < nl;
    bo[j] = t.b_ones && bn0 + j == nl;
  }
  const float* bcol = t.B + (bn0 < nl ? bn0 : 0);
  const long ldb = t.ldb;

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int kmax = t.K - 1;
  auto load = [&](int g, BwdFrag& f) {
    const int kb = 8 * g + 4 * half;
    if (!a_mn) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f4u x = *reinterpret_cast<const f4u*>(arow[i] + kb);
        f.a[i][0] = x.x; f.a[i][1] = x.y; f.a[i][2] = x.z; f.a[i][3] = x.w;
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const f2u x = *reinterpret_cast<const f2u*>(acol + (long)min(kb + c, kmax) * lda);
        f.a[0][c] = x.x; f.a[1][c] = x.y;
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f2u y = *reinterpret_cast<const f2u*>(bcol + (long)min(kb + c, kmax) * ldb);
      f.b[0][c] = y.x; f.b[1][c] = y.y;
    }
  };
  auto mma = [&](int g, const BwdFrag& f) {
    const int k0 = 8 * g;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = k0 + 4 * half + c;
      const bool kin = k >= wk_lo && k < wk_hi;
      float kf = 1.f;
      if (r1) {   // scalar loads: the two halves' k values
        const float lo = kfac[min(k0 + c, kmax)], hi = kfac[min(k0 + 4 + c, kmax)];
        kf = half ? hi : lo;
      }
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float x = f.a[i][c];
        if (r1) x = x > 0.f ? af[i] * kf : 0.f;
        a[i] = (kin && av[i]) ? x : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = bv[j] ? f.b[j][c] : (bo[j] ? 1.f : 0.f);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
  const int g_lo = wk_lo >> 3, g_hi = (wk_hi + 7) >> 3;
  if (g_lo < g_hi) {
    BwdFrag f[kBwdPF];
#pragma unroll
    for (int p = 0; p < kBwdPF; ++p)
      if (g_lo + p < g_hi) load(g_lo + p, f[p]);
#pragma unroll 1
    for (int g = g_lo; g < g_hi; g += kBwdPF) {
#pragma unroll
      for (int p = 0; p < kBwdPF; ++p) {
        if (g + p < g_hi) {
          mma(g + p, f[p]);
          if (g + p + kBwdPF < g_hi) load(g + p + kBwdPF, f[p]);
        }
      }
    }
  }

  // ---- fixed-order sum of the four waves: (w0 + w1) + (w2 + w3)
  float* slot = red + (wave >> 1) * (4 * 16 * 64);   // waves 1 / 3 -> slot 0 / 1
  if (wave & 1) {
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) slot[(b * 16 + r) * 64 + lane] = acc[b >> 1][b & 1][r];
  }
  __syncthreads();
  if (!(wave & 1)) {
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[b >> 1][b & 1][r] += slot[(b * 16 + r) * 64 + lane];
  }
  __syncthreads();
  // wave 0 hands (w0 + w1) of blocks i = 1 to wave 2, wave 2 (w2 + w3) of i = 0 to wave 0
  if (wave == 0 || wave == 2) {
    const int give = wave == 0 ? 1 : 0;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(give * 32 + j * 16 + r) * 64 + lane] = acc[give][j][r];
  }
  __syncthreads();
  if (wave & 1) return;
  const int bi = wave == 0 ? 0 : 1;   // the block row this wave finishes
  floatx16 fin[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) fin[j][r] = acc[bi][j][r] + red[(bi * 32 + j * 16 + r) * 64 + lane];

  // ---- epilogue: rows m of block bi, the lane's column pair.  The ReLU
  // masks of a dX are all loaded before the first store (C and aux may alias
  // as far as the compiler knows, so interleaved they would cost one
  // dependent memory round trip per register)
  float mk0[16], mk1[16];
  if (t.epi == EPI_MASK) {
    const int N = t.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rho = acc_row_b(r, lane);
      const int m = a_mn ? mt + 2 * rho + bi : mt + 32 * bi + rho;
      const float* mk = t.aux + (long)min(m, M - 1) * t.ld_aux + bn0;
      mk0[r] = bn0 < N ? mk[0] : 0.f;
      mk1[r] = bn0 + 1 < N ? mk[1] : 0.f;
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rho = acc_row_b(r, lane);
    const int m = a_mn ? mt + 2 * rho + bi : mt + 32 * bi + rho;
    if (m >= M) continue;
    const float v0 = fin[0][r], v1 = fin[1][r];
    const long o = (long)m * t.ldc + bn0;
    if (t.epi == EPI_GRAD) {
      if (bv[0] && bv[1]) {
        *reinterpret_cast<f2u*>(t.C + o) = f2u{v0, v1};
      } else {
        if (bv[0]) t.C[o] = v0;
        if (bo[0]) t.bias_grad[m] = v0;
        if (bo[1]) t.bias_grad[m] = v1;
      }
    } else {
      const int N = t.N;
      float w0 = v0, w1 = v1;
      if (t.epi == EPI_MASK) {
        w0 = mk0[r] > 0.f ? v0 : 0.f;
        w1 = mk1[r] > 0.f ? v1 : 0.f;
      }
      if (bn0 + 1 < N) *reinterpret_cast<f2u*>(t.C + o) = f2u{w0, w1};
      else if (bn0 < N) t.C[o] = w0;
    }
  }
}

template <int PF>
__global__ void __launch_bounds__(256)
gemm_bwd_kernel(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                const GemmBatch batch) {
  __shared__ __attribute__((aligned(16))) float red[2 * 4 * 16 * 64];   // 32 KB
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
  // operand kind of the task's A (workgroup-uniform)
  const int ak = (t.a_kc ? BA_KC : BA_MN) + (t.a_mode == A_RANK1_MASK ? 1 : 0);
  switch (ak) {
    case BA_KC: bwd_tile<BA_KC, PF>(t, local, red); break;
    case BA_KC_R1: bwd_tile<BA_KC_R1, PF>(t, local, red); break;
    case BA_MN: bwd_tile<BA_MN, PF>(t, local, red); break;
    default: bwd_tile<BA_MN_R1, PF>(t, local, red); break;
  }
}

// a backward batch this kernel takes: every task a dX (A k-contiguous, B
// n-contiguous) or dW (both batch-major) product with a plain or rank-1-mask A
// (the kind picked per task), a STORE / MASK / GRAD epilogue, no second product
bool gemm_bwd_supports(const GemmBatch& b) {
  if (b.fuse_adam || b.ntasks < 1) return false;
  for (int i = 0; i < b.ntasks; ++i) {
    const GemmTask& t = b.t[i];
    if (t.b_kc || t.K2 > 0) return false;
    if (t.epi != EPI_STORE && t.epi != EPI_MASK && t.epi != EPI_GRAD) return false;
    if (t.epi == EPI_GRAD && t.a_kc) return false;
    if (t.epi != EPI_GRAD && t.ksplit > 1) return false;
  }
  return true;
}

hipError_t gemm_bwd_launch(const GemmBatch& b, hipStream_t s) {
  if (b.total_tiles <= 0) return hipSuccess;
  if (!gemm_bwd_supports(b)) return hipErrorInvalidValue;
  int tb[8];
  for (int i = 0; i < 8; ++i) tb[i] = i < b.ntasks ? b.t[i].tile_begin : 0x7fffffff;
  // OAC_BWD2_PF: k-groups in flight per wave (2 / 3 / 4)
  static const int pf = [] { const char* e = getenv("OAC_BWD2_PF"); return e ? atoi(e) : 3; }();
  if (pf == 2)
    OAC_LAUNCH(gemm_bwd_kernel<2>, dim3(b.total_tiles), dim3(256), 0, s, b.total_tiles, tb[1],
               tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b);
  else if (pf == 4)
    OAC_LAUNCH(gemm_bwd_kernel<4>, dim3(b.total_tiles), dim3(256), 0, s, b.total_tiles, tb[1],
               tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b);
  else
    OAC_LAUNCH(gemm_bwd_kernel<3>, dim3(b.total_tiles), dim3(256), 0, s, b.total_tiles, tb[1],
               tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b);
  return hipGetLastError();
}

}  // namespace oac
