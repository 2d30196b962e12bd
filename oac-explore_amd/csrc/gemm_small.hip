// Latency-optimised grouped fp32 GEMM for the batch-256 step (the regime the
// BASELINE metric is quoted in): every stage is a handful of 256x256-ish
// products with K = 17..393, i.e. ~1 us of MFMA work per launch, so the
// kernel is built around the load latency, not around operand reuse.
//
// * One 32x32 output tile per workgroup, K split across NW waves (up to 16);
//   each wave multiplies its k-groups with v_mfma_f32_32x32x2_f32 and the
//   partial tiles are reduced through LDS in fixed wave order
//   (deterministic), then ONE coalesced epilogue pass (thread = element).
// * No LDS staging: operands go global(L2) -> VGPR -> MFMA.  A k-group is 8
//   consecutive k; MFMA c (c=0..3) of a group pairs k = 8g+c (lanes 0..31)
//   with k = 8g+4+c (lanes 32..63), so a k-contiguous operand is ONE 16-byte
//   load per lane per 4 MFMAs; other layouts load one dword per lane per MFMA
//   (coalesced across the 32 lanes of a half-wave).  The next group's loads
//   are issued before the current group's MFMAs (register double buffer).
#include "oac_common.h"
#include "kernels.h"

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// Operand fetch for one k-group: out[c] = X(mn, k = kbase + c), c = 0..3,
// where kbase = 8g + 4*(lane>>5).  `kc`: k contiguous in memory.
struct OpDesc {
  const float* p;     // base
  long ld;            // row stride
  int kc;             // 1: element (mn,k) at p[mn*ld + k]; 0: p[k*ld + mn]
  int vec;            // kc && ld%4==0 && aligned: one float4 load
  int rank1;          // value = s[row]*v[col]*(mask[row*ldm+col] > 0)
  const float* s; const float* v; long ldm;
  int n_mn;           // rows (M or N) in range
  int ones;           // virtual ones column at mn == n_mn (dW bias column)
  int K;
};

__device__ __forceinline__ void fetch4(const OpDesc& d, int mn, int kbase, float (&out)[4]) {
  const bool mn_ok = mn < d.n_mn;
  const int mnc = mn_ok ? mn : 0;
  if (d.vec) {
    const bool ok = mn_ok && (kbase < d.K);          // K % 4 == 0 on the vec path
    const float4 x = *reinterpret_cast<const float4*>(d.p + (long)mnc * d.ld + (ok ? kbase : 0));
    out[0] = ok ? x.x : 0.f; out[1] = ok ? x.y : 0.f;
    out[2] = ok ? x.z : 0.f; out[3] = ok ? x.w : 0.f;
    if (d.ones && mn == d.n_mn) {
#pragma unroll
      for (int c = 0; c < 4; ++c) out[c] = (kbase + c < d.K) ? 1.f : 0.f;
    }
    return;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int k = kbase + c;
    const bool ok = mn_ok && (k < d.K);
    const int kk = ok ? k : 0;
    const int row = d.kc ? mnc : kk;
    const int col = d.kc ? kk : mnc;
    float x;
    if (!d.rank1) {
      x = d.p[(long)row * d.ld + col];
    } else {
      const float mk = d.p[(long)row * d.ldm + col];
      x = mk > 0.f ? d.s[row] * d.v[col] : 0.f;
    }
    out[c] = ok ? x : ((d.ones && mn == d.n_mn && k < d.K) ? 1.f : 0.f);
  }
}

__device__ __forceinline__ void epi_one(const GemmTask& t, int m, int n, float acc,
                                        const float* lds_u, const float* lds_v, int mt, int nt) {
  if (m >= t.M || n >= t.N) return;
  const long o = (long)m * t.ldc + n;
  switch (t.epi) {
    case EPI_STORE: t.C[o] = acc; break;
    case EPI_GRAD:
      if (t.b_ones && n == t.N - 1) t.bias_grad[m] = acc;
      else t.C[o] = acc;
      break;
    case EPI_BIAS: t.C[o] = acc + t.bias[n]; break;
    case EPI_BIAS_RELU: t.C[o] = fmaxf(acc + t.bias[n], 0.f); break;
    case EPI_BIAS_RANK_RELU: {
      const float p = acc + t.bias[n];
      t.C[o] = p;
      const int Rp = t.R | 1;
      const float* u = lds_u + mt * Rp;
      const float* v = lds_v + nt * Rp;
      float s = 0.f;
      for (int j = 0; j < t.R; ++j) s = fmaf(u[j], v[j], s);
      t.C2[(long)m * t.ldc2 + n] = fmaxf(p + s, 0.f);
      break;
    }
    case EPI_ADD_RELU: t.C[o] = fmaxf(acc + t.aux[(long)m * t.ld_aux + n], 0.f); break;
    case EPI_MASK: t.C[o] = t.aux[(long)m * t.ld_aux + n] > 0.f ? acc : 0.f; break;
    default: break;
  }
}

template <int NW>
__global__ void __launch_bounds__(64 * NW) gemm_small_kernel(const GemmBatch batch) {
  // partial tiles: NW x 16 regs x 64 lanes ; reused for the epilogue operands
  constexpr int RED = NW * 16 * 64;
  constexpr int LDS = RED > 2 * 32 * 65 ? RED : 2 * 32 * 65;
  constexpr int PER = 1024 / (64 * NW);   // epilogue elements per thread
  __shared__ __attribute__((aligned(16))) float red[LDS];
  int ti = 0;
  const int bid = blockIdx.x;
#pragma unroll 1
  for (int i = 1; i < batch.ntasks; ++i)
    if (bid >= batch.t[i].tile_begin) ti = i;
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
  const int m0 = (local / t.tiles_n) * 32;
  const int n0 = (local % t.tiles_n) * 32;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int l32 = lane & 31;
  const int half = lane >> 5;

  // operand descriptors (the k origin is folded into K: k indices are absolute)
  OpDesc da, db;
  da.p = t.a_mode == A_PLAIN ? t.A : t.a_mask;
  da.ld = t.a_mode == A_PLAIN ? t.lda : t.ld_mask;
  da.ldm = t.ld_mask;
  da.kc = t.a_kc;
  da.rank1 = t.a_mode == A_RANK1_MASK;
  da.s = t.a_s; da.v = t.a_v;
  da.n_mn = t.M; da.ones = 0; da.K = k_hi;
  da.vec = (!da.rank1) && t.a_kc && ((t.lda & 3) == 0) &&
           ((reinterpret_cast<unsigned long>(t.A) & 15) == 0) && ((t.K & 3) == 0);
  db.p = t.B; db.ld = t.ldb; db.ldm = 0; db.kc = t.b_kc; db.rank1 = 0; db.s = nullptr;
  db.v = nullptr; db.K = k_hi;
  db.n_mn = t.b_ones ? t.N - 1 : t.N; db.ones = t.b_ones;
  db.vec = t.b_kc && ((t.ldb & 3) == 0) && ((reinterpret_cast<unsigned long>(t.B) & 15) == 0) &&
           ((t.K & 3) == 0);
  if (da.rank1 && t.a_kc) {  // K-contiguous rank-1 view: row = m (s), col = k (v)
    da.vec = 0;
  }

  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  // k-groups of 8 owned by this wave: g = g_lo + wave, wave + NW, ...
  const int g_lo = k_lo >> 3;                 // k_lo is a multiple of 8 (kchunk % 8 == 0)
  const int g_hi = (k_hi + 7) >> 3;
  const int mrow = m0 + l32;                  // A row of this lane
  const int ncol = n0 + l32;                  // B column of this lane
  float a_cur[4], b_cur[4], a_nxt[4], b_nxt[4];
  int g = g_lo + wave;
  if (g < g_hi) {
    fetch4(da, mrow, 8 * g + 4 * half, a_cur);
    fetch4(db, ncol, 8 * g + 4 * half, b_cur);
  }
#pragma unroll 1
  for (; g < g_hi; g += NW) {
    const int gn = g + NW;
    if (gn < g_hi) {
      fetch4(da, mrow, 8 * gn + 4 * half, a_nxt);
      fetch4(db, ncol, 8 * gn + 4 * half, b_nxt);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur[c], b_cur[c], acc, 0, 0, 0);
#pragma unroll
    for (int c = 0; c < 4; ++c) { a_cur[c] = a_nxt[c]; b_cur[c] = b_nxt[c]; }
  }

  // fixed-order split-K reduction through LDS
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(wave * 16 + r) * 64 + lane] = acc[r];
  __syncthreads();
  float vals[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * 64 * NW;
    const int r = e >> 6, l = e & 63;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[(w * 16 + r) * 64 + l];
    vals[i] = s;
  }
  float* lds_u = red;
  float* lds_v = red + 32 * 65;
  if (t.epi == EPI_BIAS_RANK_RELU) {   // stage the rank-R operands (reusing the LDS)
    __syncthreads();
    const int Rp = t.R | 1;
    for (int e = threadIdx.x; e < 32 * t.R; e += 64 * NW) {
      const int r = e / t.R, j = e % t.R;
      lds_u[r * Rp + j] = t.U[(long)min(m0 + r, t.M - 1) * t.ldu + j];
      lds_v[r * Rp + j] = t.V[(long)min(n0 + r, t.N - 1) * t.ldv + j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * 64 * NW;
    const int r = e >> 6, l = e & 63;
    const int mt = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    const int nt = l & 31;
    epi_one(t, m0 + mt, n0 + nt, vals[i], lds_u, lds_v, mt, nt);
  }
}

// tile geometry shared with the plan builder
int gemm_small_waves(const GemmBatch& b) {
  int kmax = 1;
  for (int i = 0; i < b.ntasks; ++i) {
    const int k = b.t[i].ksplit > 1 ? b.t[i].kchunk : b.t[i].K;
    kmax = k > kmax ? k : kmax;
  }
  const int groups = (kmax + 7) / 8;
  int nw = 1;
  while (nw < 16 && nw * 2 <= groups) nw *= 2;   // >= 1 group per wave... up to 16 waves
  return nw;
}

void gemm_small_finalize(GemmBatch& b) {
  int tiles = 0;
  for (int i = 0; i < b.ntasks; ++i) {
    GemmTask& t = b.t[i];
    if (t.ksplit < 1) t.ksplit = 1;
    t.tile_begin = tiles;
    t.tiles_n = (t.N + 31) / 32;
    tiles += ((t.M + 31) / 32) * t.tiles_n * t.ksplit;
  }
  b.total_tiles = tiles;
}

hipError_t gemm_small_launch(const GemmBatch& b, hipStream_t s) {
  if (b.total_tiles <= 0) return hipSuccess;
  const int nw = gemm_small_waves(b);
  switch (nw) {
    case 1: hipLaunchKernelGGL(gemm_small_kernel<1>, dim3(b.total_tiles), dim3(64), 0, s, b); break;
    case 2: hipLaunchKernelGGL(gemm_small_kernel<2>, dim3(b.total_tiles), dim3(128), 0, s, b); break;
    case 4: hipLaunchKernelGGL(gemm_small_kernel<4>, dim3(b.total_tiles), dim3(256), 0, s, b); break;
    case 8: hipLaunchKernelGGL(gemm_small_kernel<8>, dim3(b.total_tiles), dim3(512), 0, s, b); break;
    default: hipLaunchKernelGGL(gemm_small_kernel<16>, dim3(b.total_tiles), dim3(1024), 0, s, b); break;
  }
  return hipGetLastError();
}

}  // namespace oac
