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
#include "adam_common.h"
#include "policy_math.h"
#include "gemm_operand.h"
#include "gemm_pipe.h"

#include <algorithm>
#include <cstdlib>

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));

#ifdef OAC_STAGE_CLOCK   // per-stage wall clock of thread 0 of each block (tools/micro only)
__device__ long long g_gs_clock[4096 * 8];
#define GS_STAGE(i) do { __builtin_amdgcn_s_waitcnt(0); \
  if (threadIdx.x == 0 && blockIdx.x < 4096) g_gs_clock[blockIdx.x * 8 + (i)] = wall_clock64(); } while (0)
#else
#define GS_STAGE(i)
#endif

// Staged k-contiguous operands (STG kernels): the workgroup's 32 operand rows
// over [kst, k_hi) are copied into LDS by LDS-DMA (global_load_lds_dwordx4,
// gemm_pipe.h glds16) before the k loop -- 8 lanes per 128-byte line, where a
// fragment-shaped 16-byte load per lane touches one line per lane (64 per
// wave instruction) -- and the k loop reads its fragments from the image.
// Row stride S floats, S = 4 (mod 64): the 32 rows' 16-byte fragment reads
// at one k start on 32 distinct 4-bank groups, half-waves 4 floats apart.
__host__ __device__ inline int stage_stride(int span) {
  const int s = (span + 7) & ~7;   // fragment reads reach the next multiple of 8
  return s + ((4 - s) & 63);
}

// rows r = 0..31 of operand X(m0 + r, k) = base[row(r) * ld + k], k in
// [kst, k_hi), into img[r * S + (k - kst)]; row(r) = rows[r] (the direct
// gather's tile rows) or min(m0 + r, M - 1).  Issued by every wave; the
// caller waits (vmcnt(0)) and meets at a barrier before reading the image.
template <int NW>
__device__ __forceinline__ void stage_kc(const float* base, long ld, const int* rows, int m0, int M,
                                         int kst, int k_hi, float* img, int S) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = (k_hi - kst + 3) >> 2;   // 16-byte chunks per row
  const int nq = (nch + 63) >> 6;          // wave instructions per row
#pragma unroll 1
  for (int it = wave; it < 32 * nq; it += NW) {
    const int r = it / nq, q = it - r * nq;
    const long row = rows ? (long)rows[r] : (long)min(m0 + r, M - 1);
    const int c = 64 * q + lane;
    if (c < nch) glds16(base + row * ld + kst + 4 * c, img + r * S + 256 * q);
  }
}

struct Stage { const float* img; int S; int kst; };

constexpr int kHeadParts = 16;   // A_HEAD_BWD: parts of dL/da summed per row (<= 16)

// acc += A[m0.., k_lo..k_hi) . B[k_lo..k_hi), n0..]  for this wave's k-groups
// arow >= 0: this lane's A row is buffer row arow (the direct gather's index,
// loaded by the caller ahead of everything else)
// SA / SB: the operand's fragments come from its LDS image (KC kinds only)
template <int NW, int AK, int BK, int GPW = (NW >= 16 ? 4 : 5), bool SA = false, bool SB = false>
__device__ __forceinline__ void k_loop(const GemmTask& t, int m0, int n0, int k_lo, int k_hi,
                                       floatx16& acc, int arow = -1, Stage sa = Stage{},
                                       Stage sb = Stage{}) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
  const int l32 = lane & 31;
  const int half = lane >> 5;
  const bool ar1 = (AK == OP_KC_R1 || AK == OP_MN_R1);
  Lane la = lane_init<AK>(m0 + l32, t.M, false, ar1 ? t.a_mask : t.A,
                          ar1 ? t.ld_mask : t.lda, t.a_s, t.a_v);
  if (arow >= 0 && (AK == OP_KC || AK == OP_KC_R1))
    la.p = (ar1 ? t.a_mask : t.A) + (long)arow * (ar1 ? t.ld_mask : t.lda);
  const Lane lb = lane_init<BK>(n0 + l32, t.b_ones ? t.N - 1 : t.N, t.b_ones != 0, t.B, t.ldb,
                                nullptr, nullptr);
  constexpr int kGPW = GPW;                   // k-groups in flight per wave (<= 128 VGPRs at 8 waves)
  const int g_lo = k_lo >> 3;                 // k_lo is a multiple of 8 (kchunk % 8 == 0)
  const int g_hi = (k_hi + 7) >> 3;
  const int kmax = k_hi - 1;
  const float* fa = sa.img + l32 * sa.S - sa.kst;   // SA: this lane's image row (k-indexed)
  const float* fb = sb.img + l32 * sb.S - sb.kst;
#pragma unroll 1
  for (int g0 = g_lo + wave; g0 < g_hi; g0 += kGPW * NW) {
    float ax[kGPW][4], ay[kGPW][4], bx[kGPW][4], by[kGPW][4];
#pragma unroll
    for (int j = 0; j < kGPW; ++j)
      if (g0 + j * NW < g_hi) {
        const int kb = 8 * (g0 + j * NW) + 4 * half;
        if (SB) {
          const f4u v = *reinterpret_cast<const f4u*>(fb + kb);
          bx[j][0] = v.x; bx[j][1] = v.y; bx[j][2] = v.z; bx[j][3] = v.w;
        } else {
          load4<BK>(lb, kb, kmax, bx[j], by[j]);   // B first: it never waits on a row index
        }
        if (SA) {
          const f4u v = *reinterpret_cast<const f4u*>(fa + kb);
          ax[j][0] = v.x; ax[j][1] = v.y; ax[j][2] = v.z; ax[j][3] = v.w;
          if (AK == OP_KC_R1) {   // the rank-1 factor v[k]: one (broadcast) 16-byte load
            const f4u w = *reinterpret_cast<const f4u*>(la.s + kb);
            ay[j][0] = w.x; ay[j][1] = w.y; ay[j][2] = w.z; ay[j][3] = w.w;
          }
        } else {
          load4<AK>(la, kb, kmax, ax[j], ay[j]);
        }
      }
#pragma unroll
    for (int j = 0; j < kGPW; ++j)
      if (g0 + j * NW < g_hi) {
        const int kb = 8 * (g0 + j * NW) + 4 * half;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float a = fix1<AK>(la, kb + c, k_hi, ax[j][c], ay[j][c]);
          const float b = fix1<BK>(lb, kb + c, k_hi, bx[j][c], by[j][c]);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
      }
  }
}

template <int NW, int GPW, bool STG>
__device__ __forceinline__ void k_dispatch(const GemmTask& t, int m0, int n0, int k_lo, int k_hi,
                                           floatx16& acc, int arow, Stage sa, Stage sb) {
  const bool r1 = t.a_mode == A_RANK1_MASK;
  if (t.a_kc && t.b_kc)        k_loop<NW, OP_KC, OP_KC, GPW, STG, STG>(t, m0, n0, k_lo, k_hi, acc, arow, sa, sb);   // forward
  else if (t.a_kc && !r1)      k_loop<NW, OP_KC, OP_MN, GPW, STG>(t, m0, n0, k_lo, k_hi, acc, -1, sa);      // dX
  else if (t.a_kc)             k_loop<NW, OP_KC_R1, OP_MN, GPW, STG>(t, m0, n0, k_lo, k_hi, acc, -1, sa);   // dX, rank-1 seed
  else if (!r1)                k_loop<NW, OP_MN, OP_MN, GPW>(t, m0, n0, k_lo, k_hi, acc);      // dW
  else                         k_loop<NW, OP_MN_R1, OP_MN, GPW>(t, m0, n0, k_lo, k_hi, acc);   // dW, rank-1 seed
}

// ---------------------------------------------------------------------------
// A_HEAD_FWD: the fresh-action critic layer 1's A operand computed per 32-row
// block inside the tile (what policy_head_kernel, head.hip, did as a launch of
// its own): (1) the stacked heads [mean | ls_raw] = h2 . W_head^T for the 32
// rows on v_mfma_f32_16x16x4_f32 (2 row x NTc column tiles of 16, K halved
// over two waves, halves added in order), (2) the tanh-Gaussian sample and
// log-prob (policy_math.h, one half-wave per row), (3) the critic's layer 0 on
// the actions, h1 = relu(P + sum_j a_j W0[:, Do + j]) for all H columns, into
// the LDS image the k loop reads.  Every tile of a row block computes the same
// values in the same order; the writing task's n0 == 0 tiles store them.
// LDS (floats): image [32][S] | head partials [2][8][256] | Y [32][65] |
// act [32][33] | lp [32] | W0[:, Do:]^T [32][H]
constexpr int kHfPart = 2 * 8 * 256, kHfY = 32 * 65, kHfAct = 32 * 33;
__host__ __device__ inline int head_fwd_floats(int H) {
  return 32 * stage_stride(H) + kHfPart + kHfY + kHfAct + 32 + 32 * H;
}

template <int NW>
__device__ __forceinline__ void head_fwd_image(const GemmBatch& batch, const GemmTask& t, int m0,
                                               int n0, float* lds) {
  const HeadFwd& hf = batch.hf[t.a_aux & 1];
  const bool wr = (t.a_aux & 2) && n0 == 0;
  const int H = t.K, Da = hf.Da, D2 = 2 * Da, M = t.M;
  const int S = stage_stride(H);
  float* img = lds;
  float* part = img + 32 * S;
  float* Y = part + kHfPart;
  float* act = Y + kHfY;
  float* lp = act + kHfAct;
  float* waT = lp + 32;                      // [Da][H]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g4 = lane >> 4;
  const int ntc = (D2 + 15) >> 4;            // head column tiles of 16 (<= 4)
  const int items = 2 * 2 * ntc;             // (row tile, column tile, k half)
  // (1) heads: wave w < items takes one (row tile, column tile, k half)
  typedef float floatx4 __attribute__((ext_vector_type(4)));
  if (wave < items) {
    const int kh = wave / (2 * ntc), tile = wave - kh * 2 * ntc;
    const int rt = tile / ntc, ct = tile - rt * ntc;
    const float* arow = hf.h2 + (long)min(m0 + 16 * rt + l16, M - 1) * H;
    const int bc = 16 * ct + l16;
    const float* brow = hf.wh + (long)min(bc, D2 - 1) * H;
    const int k0 = kh * (H >> 1), nch = (H >> 1) >> 4;   // 16-k chunks of the half
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
    constexpr int U = 8;   // chunks in flight
#pragma unroll 1
    for (int c0 = 0; c0 < nch; c0 += U) {
      f4u xa[U], xb[U];
#pragma unroll
      for (int c = 0; c < U; ++c) {
        const int kb = k0 + 16 * min(c0 + c, nch - 1) + 4 * g4;
        xa[c] = *reinterpret_cast<const f4u*>(arow + kb);
        xb[c] = *reinterpret_cast<const f4u*>(brow + kb);
      }
#pragma unroll
      for (int c = 0; c < U; ++c)
        if (c0 + c < nch) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[c][j], bc < D2 ? xb[c][j] : 0.f, acc, 0, 0, 0);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) part[(kh * 8 + tile) * 256 + r * 64 + lane] = acc[r];
  }
  // (3)'s W0[:, Do:] transposed into LDS (row n of W0 at a_v + n ld_mask)
  constexpr int kNT = 64 * NW;
  for (int e = threadIdx.x; e < H * Da; e += kNT) {
    const int nn = e / Da, j = e - nn * Da;
    waT[j * H + nn] = t.a_v[(long)nn * t.ld_mask + j];
  }
  const int n = threadIdx.x % H, r0 = threadIdx.x / H, rstep = kNT / H;   // (kNT % H == 0: launcher)
  __syncthreads();
  // Y = the two k halves in order + bias (D reg r: row 4 (l >> 4) + r, col l & 15)
  for (int e = threadIdx.x; e < 2 * ntc * 256; e += kNT) {
    const int tile = e >> 8, r = (e >> 6) & 3, l = e & 63;
    const int rt = tile / ntc, ct = tile - rt * ntc;
    const int row = 16 * rt + 4 * (l >> 4) + r, col = 16 * ct + (l & 15);
    if (col < D2)
      Y[row * 65 + col] = (part[tile * 256 + r * 64 + l] + part[(8 + tile) * 256 + r * 64 + l]) + hf.bh[col];
  }
  __syncthreads();
  // (2) sample + log-prob: one half-wave per row, lane j = action dim
  for (int e = threadIdx.x; e < 32 * 32; e += kNT) {
    const int row = e >> 5, j = e & 31, m = m0 + row;
    float l = 0.f, a = 0.f;
    if (m < M && j < Da) {
      float sd, u;
      l = tanh_gauss_sample(Y[row * 65 + j], Y[row * 65 + Da + j], hf.eps[(long)m * Da + j], a, sd, u);
      if (wr) {
        const long o = (long)m * Da + j;
        hf.act[o] = a; hf.stdv[o] = sd; hf.u[o] = u;
        hf.head[(long)m * D2 + j] = Y[row * 65 + j];
        hf.head[(long)m * D2 + Da + j] = Y[row * 65 + Da + j];
      }
    }
    act[row * 33 + j] = a;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) l += __shfl_xor(l, o, 32);
    if (j == 0) {
      lp[row] = m < M ? l + hf.te : 0.f;
      if (wr && m < M) hf.logp[m] = l;
    }
  }
  __syncthreads();
  if (wr && hf.logp_part && threadIdx.x < 2 && m0 + 16 * threadIdx.x < M) {   // data-parallel alpha
    float sum = 0.f;
    for (int r = 0; r < 16; ++r) sum += lp[16 * threadIdx.x + r];
    hf.logp_part[(m0 >> 4) + threadIdx.x] = sum;
  }
  // (3) h1 = relu(P + sum_j a_j W0[n, Do + j]) for the 32 rows, column n
  float* U = const_cast<float*>(t.U);
  for (int r = r0; r < 32; r += rstep) {
    const int m = min(m0 + r, M - 1);
    float sacc = t.A[(long)m * t.lda + n];
    for (int j = 0; j < Da; ++j) sacc = fmaf(act[r * 33 + j], waT[j * H + n], sacc);
    const float h = fmaxf(sacc, 0.f);
    img[r * S + n] = h;
    if (U && n0 == 0 && m0 + r < M) U[(long)(m0 + r) * t.ldu + n] = h;
  }
  __syncthreads();
}

// Epilogue operands of one output element, loaded before the k loop so their
// latency hides behind it: xb = bias[n] (or the fused-Adam p), xa = aux[m,n]
// (EPI_ADD_RELU / EPI_MASK), aux[n] (EPI_BIAS_RELU_DOT).
// EPI_GRAD with the fused optimizer: p, m, v (and the Polyak target) of the element.
struct EpiIn { float xb, xa, am, av, at, s; };

__device__ __forceinline__ EpiIn epi_prefetch(const GemmBatch& batch, const GemmTask& t, int m,
                                              int n) {
  EpiIn x{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool in = m < t.M && n < t.N;
  const int mc = in ? m : 0, nc = in ? n : 0;
  switch (t.epi) {
    case EPI_HEAD_BWD: {   // act, std, u, eps [B, Da]; ls_raw from the head; alpha
      const long e = (long)mc * t.N + nc;
      x.xb = t.ex[0][e]; x.xa = t.ex[1][e]; x.am = t.ex[2][e]; x.av = t.ex[3][e];
      x.at = t.ex[4][(long)mc * 2 * t.N + t.N + nc];
      x.s = t.ex[5] ? t.ex[5][0] : 0.f;
      break;
    }
    case EPI_GRAD:
      if (batch.fuse_adam) {
        const float* g = (t.b_ones && nc == t.N - 1) ? t.bias_grad + mc : t.C + (long)mc * t.ldc + nc;
        const long i = g - batch.adam.g;
        x.xb = batch.adam.p[i]; x.am = batch.adam.m[i]; x.av = batch.adam.v[i];
        if (batch.adam.target) x.at = batch.adam.target[i];
      }
      break;
    case EPI_BIAS: case EPI_BIAS_RELU: case EPI_BIAS_RANK_RELU:
      x.xb = t.bias[nc]; break;
    case EPI_BIAS_RELU_DOT:
      x.xb = t.bias[nc]; x.xa = t.aux[nc]; break;
    case EPI_ADD_RELU: case EPI_MASK: case EPI_MASK_DA:
      x.xa = t.aux[(long)mc * t.ld_aux + nc]; break;
    default: break;
  }
  return x;
}

__device__ __forceinline__ void epi_one(const GemmBatch& batch, const AdamConsts& ac,
                                        const GemmTask& t, int m, int n, float acc, EpiIn x,
                                        const float* lds_u, const float* lds_v, int mt, int nt) {
  if (m >= t.M || n >= t.N) return;
  const long o = (long)m * t.ldc + n;
  switch (t.epi) {
    case EPI_STORE: t.C[o] = acc; break;
    case EPI_GRAD: {
      float* g = (t.b_ones && n == t.N - 1) ? t.bias_grad + m : t.C + o;
      *g = acc;
      if (batch.fuse_adam) {   // adam_elem on the prefetched p, m, v, target
        const long i = g - batch.adam.g;
        float p = x.xb, m = x.am, v = x.av;
        adam1(ac, p, acc, m, v);
        batch.adam.p[i] = p; batch.adam.m[i] = m; batch.adam.v[i] = v;
        if (ac.polyak) batch.adam.target[i] = polyak1(ac, x.at, p);
      }
      break;
    }
    case EPI_BIAS: t.C[o] = acc + x.xb; break;
    case EPI_BIAS_RELU:
    case EPI_BIAS_RELU_DOT: t.C[o] = fmaxf(acc + x.xb, 0.f); break;
    case EPI_BIAS_RANK_RELU: {
      const float p = acc + x.xb;
      t.C[o] = p;
      const int Rp = t.R | 1;
      const float* u = lds_u + mt * Rp;
      const float* v = lds_v + nt * Rp;
      float s = 0.f;
      for (int j = 0; j < t.R; ++j) s = fmaf(u[j], v[j], s);
      t.C2[(long)m * t.ldc2 + n] = fmaxf(p + s, 0.f);
      break;
    }
    case EPI_ADD_RELU: t.C[o] = fmaxf(acc + x.xa, 0.f); break;
    case EPI_MASK: case EPI_MASK_DA: t.C[o] = x.xa > 0.f ? acc : 0.f; break;
    case EPI_HEAD_BWD: {
      float dmean, dls;
      tanh_gauss_backward(acc, x.xb, x.xa, x.am, x.av, x.at, x.s * (1.f / (float)t.M), dmean, dls);
      t.C[o] = dmean;
      t.C[o + t.N] = dls;
      break;
    }
    default: break;
  }
}

// Launch header as leading scalar kernel arguments: with
// -mllvm -amdgpu-kernarg-preload-count they arrive in SGPRs, so a block finds
// its task without a dependent kernarg round trip; only the task record itself
// is then loaded (one scalar round trip).
struct GemmHead { int total_tiles, publish, tb1, tb2, tb3, tb4, tb5, tb6, tb7; };

static GemmHead gemm_head(const GemmBatch& b) {
  GemmHead h;
  int tb[8];
  for (int i = 0; i < 8; ++i) tb[i] = i < b.ntasks ? b.t[i].tile_begin : 0x7fffffff;
  h.total_tiles = b.total_tiles; h.publish = b.publish != nullptr;
  h.tb1 = tb[1]; h.tb2 = tb[2]; h.tb3 = tb[3]; h.tb4 = tb[4]; h.tb5 = tb[5]; h.tb6 = tb[6]; h.tb7 = tb[7];
  return h;
}

// one workgroup's share of a launch: block `bid` of the batch (the kernel
// below passes blockIdx.x; tools/micro/persist_micro.hip runs several batches
// in one persistent launch with a grid barrier between them)
template <int NW>
struct SmallLds {
  static constexpr int RED = NW * 16 * 64;   // partial tiles: NW x 16 regs x 64 lanes
  static constexpr int N = RED > 2 * 32 * 65 ? RED : 2 * 32 * 65;   // reused for the epilogue operands
};

constexpr int kGatherU = 4;   // float4s per lane of a side block's row copy (rows <= 1 KB)

// the direct gather's 32 tile rows (their own LDS object: the launch's
// dynamic LDS holds the staged images and the reduction)
__device__ __forceinline__ int* tile_rows_of(float*) {
  __shared__ int tile_rows[32];
  return tile_rows;
}

// LDS floats the STG kernel's images take for one task (0: nothing staged)
__host__ __device__ inline int head_fwd_floats(int H);
__host__ __device__ inline int stage_floats(const GemmTask& t) {
  if (t.a_mode == A_HEAD_FWD) return head_fwd_floats(t.K) + 32 * stage_stride(t.K);   // image + B
  if (!t.a_kc || t.ksplit > 1 || t.a_mode == A_HEAD_BWD) return 0;
  int n = 32 * stage_stride(t.K);                       // A (or A's ReLU mask)
  if (t.b_kc) n += 32 * stage_stride(t.K);              // B of a forward product
  if (t.K2 > 0) n += 32 * stage_stride(t.K2);           // the second product's A
  return n;
}

template <int NW, int GPW, bool STG = false>
__device__ __forceinline__ void gemm_small_block(int bid, int total_tiles, int publish, int tb1,
                                                 int tb2, int tb3, int tb4, int tb5, int tb6,
                                                 int tb7, const GemmBatch& batch, float* red) {
  constexpr int PER = 1024 / (64 * NW);   // epilogue elements per thread
  GS_STAGE(0);
  if (publish && bid == 0 && threadIdx.x == 0)
    publish_step_consts(batch.publish, batch.pub_beta1, batch.pub_beta2);
  const int* rows = nullptr;   // direct drop-in gather: this step's index slot (host memory)
  long long bc = 0;
  if (batch.rg.ring) {
    bc = batch.rg.state->batch_counter;
    rows = batch.rg.ring + (long)(bc % batch.rg.slots) * batch.rg.B;
  }
  if (bid >= total_tiles + batch.adam_blocks) {   // side blocks: the batch copy and the eps draws
    // one wave per row: the row's index is one read of the host slot per
    // wave (every lane the same word), the row's float4s all in flight before
    // their stores; then the eps
    const RowGather& g = batch.rg;
    const int sb = bid - total_tiles - batch.adam_blocks;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long n4 = g.row_stride >> 2;
    const int nwv = g.blocks * NW;
    const float4* src = reinterpret_cast<const float4*>(g.replay);
    float4* dst = reinterpret_cast<float4*>(g.out);
    static_assert(kGatherU == 4, "the row copy below holds four float4s per lane");
    for (int r = sb * NW + wave; r < g.B; r += nwv) {
      // four named registers, not an array: the array form went through
      // scratch (a store and a dependent reload per float4)
      const float4* s0 = src + rows[r] * n4;
      float4* d0 = dst + (long)r * n4;
      const long c0 = lane, c1 = lane + 64, c2 = lane + 128, c3 = lane + 192;
      const float4 v0 = s0[c0 < n4 ? c0 : 0], v1 = s0[c1 < n4 ? c1 : 0];
      const float4 v2 = s0[c2 < n4 ? c2 : 0], v3 = s0[c3 < n4 ? c3 : 0];
      if (c0 < n4) d0[c0] = v0;
      if (c1 < n4) d0[c1] = v1;
      if (c2 < n4) d0[c2] = v2;
      if (c3 < n4) d0[c3] = v3;
    }
    for (int e = sb * 64 * NW + threadIdx.x; g.eps1 && e < g.n_eps; e += g.blocks * 64 * NW) {
      g.eps1[e] = philox_normal(g.seed, (unsigned long long)bc, 1u, (unsigned)e);
      g.eps2[e] = philox_normal(g.seed, (unsigned long long)bc, 2u, (unsigned)e);
    }
    return;
  }
  if (bid >= total_tiles) {   // fused optimizer: flat Adam over the other ranges
    const AdamArgs& a = batch.adam;
    const AdamConsts c = adam_consts(a.state, a.advance, a.lr, a.beta1, a.beta2, a.eps,
                                     a.target, a.tau, a.period);
    const long stride = (long)batch.adam_blocks * 64 * NW;
    for (int sgi = 0; sgi < batch.nseg; ++sgi) {
      AdamArgs r = a;
      r.p += batch.seg_off[sgi]; r.m += batch.seg_off[sgi]; r.v += batch.seg_off[sgi];
      if (r.target) r.target += batch.seg_off[sgi];
      const float* g = a.g + batch.seg_off[sgi];
      const long n4 = batch.seg_n[sgi] >> 2;
      for (long i = (long)(bid - total_tiles) * 64 * NW + threadIdx.x; i < n4; i += stride)
        adam_float4(c, r, i, reinterpret_cast<const float4*>(g)[i]);
    }
    return;
  }
  int ti = 0;   // task of this block from the preloaded tile starts (no memory access)
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
  const int m0 = (local / t.tiles_n) * 32;
  const int n0 = (local % t.tiles_n) * 32;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
  GS_STAGE(1);
  // the direct gather's row indices (host memory, the longest wait of the
  // launch): one read of the tile's 32 by wave 0, handed to the other waves
  // through LDS -- one host request per workgroup, not one per wave
  int arow = -1;
  if (t.a_rows && rows) {
    int* tile_rows = tile_rows_of(red);
    if (wave == 0 && lane < 32) tile_rows[lane] = rows[min(m0 + lane, t.M - 1)];
    __syncthreads();
    arow = tile_rows[lane & 31];
  }

  // STG: the k-contiguous operands' 32 rows into LDS images first (their
  // DMA overlaps the epilogue prefetch below)
  const bool hbw = t.a_mode == A_HEAD_BWD;   // A computed below, not loaded
  const bool hfw = t.a_mode == A_HEAD_FWD;   // A computed below, B staged by LDS-DMA
  const bool stg = STG && t.a_kc && t.ksplit <= 1 && !hbw && !hfw;
  Stage sa{}, sb{}, sa2{};
  if (stg) {
    const bool ar1 = t.a_mode == A_RANK1_MASK;
    const int S = stage_stride(t.K);
    sa = Stage{red, S, k_lo};
    stage_kc<NW>(ar1 ? t.a_mask : t.A, ar1 ? t.ld_mask : t.lda, arow >= 0 ? tile_rows_of(red) : nullptr,
                 m0, t.M, k_lo, k_hi, red, S);
    float* nxt = red + 32 * S;
    if (t.b_kc) {
      sb = Stage{nxt, S, k_lo};
      stage_kc<NW>(t.B, t.ldb, nullptr, n0, t.N, k_lo, k_hi, nxt, S);
      nxt += 32 * S;
    }
    if (t.K2 > 0) {
      const int S2 = stage_stride(t.K2);
      sa2 = Stage{nxt, S2, 0};
      stage_kc<NW>(t.A2, t.lda, nullptr, m0, t.M, 0, t.K2, nxt, S2);
    }
  }
  EpiIn xin[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * 64 * NW;
    const int r = e >> 6, l = e & 63;
    xin[i] = epi_prefetch(batch, t, m0 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), n0 + (l & 31));
  }
  // EPI_MASK_DA: the tile's rows of V (the next product's weights) requested
  // now, used after the epilogue
  constexpr int VPF = (1024 + 64 * NW - 1) / (64 * NW);   // 32 rows x R <= 32 per thread
  float vpf[VPF];
  if (t.epi == EPI_MASK_DA) {
#pragma unroll
    for (int q = 0; q < VPF; ++q) {
      const int e = threadIdx.x + q * 64 * NW;
      const int n = e / t.R, j = e - n * t.R;
      vpf[q] = (e < 32 * t.R && n0 + n < t.N) ? t.V[(long)(n0 + n) * t.ldv + j] : 0.f;
    }
  }
  if (stg) {   // every wave's DMA landed, then the images are complete for all
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  if (hfw) {
    // B (the critic's layer-1 rows) into LDS behind the image, its DMA in
    // flight while the heads, the sample and h1 are computed
    const int S = stage_stride(t.K);
    float* bimg = red + head_fwd_floats(t.K);
    stage_kc<NW>(t.B, t.ldb, nullptr, n0, t.N, 0, t.K, bimg, S);
    head_fwd_image<NW>(batch, t, m0, n0, red);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    k_loop<NW, OP_KC, OP_KC, GPW, true, true>(t, m0, n0, 0, t.K, acc, -1, Stage{red, S, 0},
                                             Stage{bimg, S, 0});
  } else if (hbw) {
    // A = [dmean | dls_raw] of the tile's 32 rows from the parts of dL/da
    // (an EPI_MASK_DA launch wrote them), the head backward of EPI_HEAD_BWD:
    // into an LDS image read by the k loop like a staged operand
    const int Da = t.K >> 1, S = stage_stride(t.K);
    const float G = (t.ex[5] ? t.ex[5][0] : 0.f) * (1.f / (float)t.M);
    for (int e = threadIdx.x; e < 32 * Da; e += 64 * NW) {
      const int r = e / Da, j = e - r * Da;
      const int m = min(m0 + r, t.M - 1);
      const long o = (long)m * Da + j;
      // every part's load issued unconditionally (clamped part index): a
      // load behind a runtime condition is waited for one at a time
      float pv[kHeadParts];
#pragma unroll
      for (int q = 0; q < kHeadParts; ++q) pv[q] = t.A[min(q, t.R - 1) * t.lda + o];
      float da = pv[0];
#pragma unroll
      for (int q = 1; q < kHeadParts; ++q)
        if (q < t.R) da += pv[q];
      float dmean, dls;
      tanh_gauss_backward(da, t.ex[0][o], t.ex[1][o], t.ex[2][o], t.ex[3][o],
                          t.ex[4][(long)m * 2 * Da + Da + j], G, dmean, dls);
      red[r * S + j] = dmean;
      red[r * S + Da + j] = dls;
      if (n0 == 0 && t.U && m0 + r < t.M) {   // dhead for the head's weight gradient (next launch)
        float* u = const_cast<float*>(t.U) + (long)m * t.ldu;
        u[j] = dmean;
        u[Da + j] = dls;
      }
    }
    __syncthreads();
    k_loop<NW, OP_KC, OP_MN, GPW, true>(t, m0, n0, 0, t.K, acc, -1, Stage{red, S, 0});
  } else if (stg) {
    k_dispatch<NW, GPW, true>(t, m0, n0, k_lo, k_hi, acc, arow, sa, sb);
  } else {
    k_dispatch<NW, GPW, false>(t, m0, n0, k_lo, k_hi, acc, arow, sa, sb);
  }
  if (t.K2 > 0) {   // second product into the same accumulator (unsplit dX tasks only)
    GemmTask t2 = t;
    t2.A = t.A2; t2.B = t.B2; t2.K = t.K2;
    if (stg) k_loop<NW, OP_KC, OP_MN, GPW, true>(t2, m0, n0, 0, t.K2, acc, -1, sa2);
    else k_loop<NW, OP_KC, OP_MN, GPW>(t2, m0, n0, 0, t.K2, acc);
  }
  if (stg || hbw || hfw) __syncthreads();   // the images are read by all waves before the reduction reuses the LDS

  GS_STAGE(2);
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
  GS_STAGE(3);
  float* lds_u = red;
  float* lds_v = red + 32 * 65;
  if (t.epi == EPI_BIAS_RANK_RELU) {   // stage the rank-R operands (reusing the LDS)
    __syncthreads();
    const int Rp = t.R | 1;
    for (int e = threadIdx.x; e < 32 * t.R; e += 64 * NW) {
      const int r = e / t.R, j = e % t.R;
      const int mr = min(m0 + r, t.M - 1);
      lds_u[r * Rp + j] = t.U[(long)(t.a_rows ? rows[mr] : mr) * t.ldu + j];
      lds_v[r * Rp + j] = t.V[(long)min(n0 + r, t.N - 1) * t.ldv + j];
    }
    __syncthreads();
  }
  AdamConsts ac{};
  if (batch.fuse_adam)
    ac = adam_consts(batch.adam.state, batch.adam.advance, batch.adam.lr, batch.adam.beta1,
                     batch.adam.beta2, batch.adam.eps, batch.adam.target, batch.adam.tau,
                     batch.adam.period);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * 64 * NW;
    const int r = e >> 6, l = e & 63;
    const int mt = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    const int nt = l & 31;
    epi_one(batch, ac, t, m0 + mt, n0 + nt, vals[i], xin[i], lds_u, lds_v, mt, nt);
    if (t.epi == EPI_BIAS_RELU_DOT) {
      // the 32 lanes of a half-wave hold one row's 32 columns: fixed butterfly
      const int m = m0 + mt, n = n0 + nt;
      float x = (m < t.M && n < t.N) ? fmaxf(vals[i] + xin[i].xb, 0.f) * xin[i].xa : 0.f;
#pragma unroll
      for (int off = 16; off > 0; off >>= 1) x += __shfl_xor(x, off, 32);
      if (nt == 0 && m < t.M) t.C2[(long)(n0 >> 5) * t.ldc2 + m] = x;   // tile-major
    }
  }
  if (t.epi == EPI_MASK_DA) {
    // the tile's part of C . V[:, :R]: the masked tile and V's 32 rows in LDS,
    // one thread per (row, j), the 32 columns in order
    __syncthreads();   // (the LDS held the reduction)
    float* ct = red;             // [32][33]
    float* vb = red + 32 * 33;   // [32][R]
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + i * 64 * NW;
      const int r = e >> 6, l = e & 63;
      const int mt = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), nt = l & 31;
      const bool in = m0 + mt < t.M && n0 + nt < t.N;
      ct[mt * 33 + nt] = (in && xin[i].xa > 0.f) ? vals[i] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < VPF; ++q) {
      const int e = threadIdx.x + q * 64 * NW;
      if (e < 32 * t.R) vb[e] = vpf[q];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 32 * t.R; e += 64 * NW) {
      const int r = e / t.R, j = e - r * t.R;
      float sacc = 0.f;
#pragma unroll 8
      for (int n = 0; n < 32; ++n) sacc = fmaf(ct[r * 33 + n], vb[n * t.R + j], sacc);
      if (m0 + r < t.M) t.C2[(long)(n0 >> 5) * t.ldc2 + (long)(m0 + r) * t.R + j] = sacc;
    }
  }
  if (batch.fuse_adam && bid == 0 && threadIdx.x == 0)
    step_bookkeeping(batch.adam.state, batch.adam.alpha, batch.adam.advance);
  GS_STAGE(4);
}

// 8- and 16-wave workgroups: 4 waves per SIMD (<= 128 VGPRs), so two 8-wave
// workgroups share a CU past 256 tiles (fewer waves: no bound, their many
// epilogue elements per thread would spill)
template <int NW, int GPW, bool STG>
__global__ void __launch_bounds__(64 * NW, NW >= 8 ? 4 : 1)
gemm_small_kernel(int total_tiles, int publish, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6,
                  int tb7, const GemmBatch batch) {
  extern __shared__ __attribute__((aligned(16))) float red[];   // SmallLds<NW>::N or the images
  gemm_small_block<NW, GPW, STG>(blockIdx.x, total_tiles, publish, tb1, tb2, tb3, tb4, tb5, tb6,
                                 tb7, batch, red);
}

// tile geometry shared with the plan builder
int gemm_small_waves(const GemmBatch& b) {
  int kmax = 1;
  for (int i = 0; i < b.ntasks; ++i) {
    const int k = b.t[i].ksplit > 1 ? b.t[i].kchunk : std::max(b.t[i].K, b.t[i].K2);
    kmax = k > kmax ? k : kmax;
  }
  const int groups = (kmax + 7) / 8;
  int nw = 1;
  while (nw < 16 && nw * 2 <= groups) nw *= 2;   // >= 1 group per wave... up to 16 waves
  // a 16-wave workgroup holds a whole CU (VGPRs); past 256 tiles the grid
  // would run in two rounds, so take 8 waves (two workgroups per CU)
  if (nw == 16 && b.total_tiles > 256) nw = 8;
  for (int i = 0; i < b.ntasks; ++i)   // the computed fresh-action operand takes 16 waves
    if (b.t[i].a_mode == A_HEAD_FWD) nw = 16;
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

static int SmallLdsFloats(int nw) {
  switch (nw) {
    case 1: return SmallLds<1>::N;
    case 2: return SmallLds<2>::N;
    case 4: return SmallLds<4>::N;
    case 8: return SmallLds<8>::N;
    default: return SmallLds<16>::N;
  }
}
constexpr int kLdsBytesPerCu = 160 * 1024;
static bool small_stage_on() {
  static const bool on = [] { const char* e = getenv("OAC_SMALL_STAGE"); return e && atoi(e) == 1; }();
  return on;
}

hipError_t gemm_small_launch(const GemmBatch& b0, hipStream_t s) {
  if (b0.total_tiles <= 0) return hipSuccess;
  GemmBatch b = b0;
  for (int i = 0; i < b.ntasks; ++i) {   // second products: plain unsplit dX tasks
    const GemmTask& t = b.t[i];
    if (t.K2 > 0 && (t.ksplit > 1 || !t.a_kc || t.b_kc || t.a_mode != A_PLAIN))
      return hipErrorInvalidValue;
    // the computed head-backward operand: an unsplit dX with K = 2 Da, <= kHeadParts parts
    if (t.a_mode == A_HEAD_BWD && (!t.a_kc || t.b_kc || t.ksplit > 1 || (t.K & 1) || t.K2 > 0 ||
                                    t.R < 1 || t.R > kHeadParts || 32 * stage_stride(t.K) > 2 * 32 * 65))
      return hipErrorInvalidValue;
    if (t.epi == EPI_MASK_DA && (t.R < 1 || t.R > 32 || t.ksplit > 1 || !t.C2 || !t.V))
      return hipErrorInvalidValue;
  }
  const int nw = b.force_nw > 0 ? b.force_nw : gemm_small_waves(b);
  int gpw = b.force_gpw > 0 ? b.force_gpw : (nw >= 16 ? 4 : 5);
  b.adam_blocks = 0;
  if (b.fuse_adam) {
    long n4 = 0;
    for (int i = 0; i < b.nseg; ++i) {
      if ((b.seg_n[i] | b.seg_off[i]) & 3) return hipErrorInvalidValue;
      n4 = std::max(n4, b.seg_n[i] >> 2);
    }
    b.adam_blocks = (int)std::min<long>((n4 + 64 * nw - 1) / (64 * nw), 1024);
    if (b.adam_blocks < 1) b.adam_blocks = 1;
  }
  const int grid = b.total_tiles + b.adam_blocks + (b.rg.ring ? b.rg.blocks : 0);
  const GemmHead h = gemm_head(b);
  // staged k-contiguous operands (OAC_SMALL_STAGE=1): when the images fit
  // beside the workgroups per CU the grid needs (1 at >= 16 waves)
  int lds = SmallLdsFloats(nw);
  for (int i = 0; i < b.ntasks; ++i) {   // the computed fresh-action operand: 16 waves, its LDS
    const GemmTask& t = b.t[i];
    if (t.a_mode != A_HEAD_FWD) continue;
    const HeadFwd& hf = b.hf[t.a_aux & 1];
    if (nw != 16 || !t.b_kc || t.ksplit > 1 || t.K2 > 0 || t.K % 32 || (64 * nw) % t.K ||
        hf.Da < 1 || hf.Da > 32 || !hf.h2 || !hf.wh || !hf.bh || !hf.eps || !t.a_v)
      return hipErrorInvalidValue;
    lds = std::max(lds, stage_floats(t));
  }
  if (4 * lds > kLdsBytesPerCu) return hipErrorInvalidValue;
  bool stg = false;
  if (small_stage_on() && b.force_gpw <= 0 && (nw == 8 || nw == 16)) {
    int need = 0;
    for (int i = 0; i < b.ntasks; ++i) need = std::max(need, stage_floats(b.t[i]));
    const int per_cu = nw >= 16 ? 1 : std::max(1, (grid + 255) / 256);
    if (need > 0 && 4 * std::max(need, lds) * per_cu <= kLdsBytesPerCu) {
      stg = true;
      lds = std::max(need, lds);
      if (nw == 8) gpw = 4;
    }
  }
  const size_t shm = 4 * (size_t)lds;
#define OAC_GS(NW_, G_) \
  if (nw == NW_ && gpw == G_ && !stg) { \
    if (shm > 64 * 1024) { \
      const hipError_t ea = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_small_kernel<NW_, G_, false>), \
          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm); \
      if (ea != hipSuccess) return ea; } \
    OAC_LAUNCH((gemm_small_kernel<NW_, G_, false>), dim3(grid), dim3(64 * NW_), shm, s, h.total_tiles, h.publish, \
               h.tb1, h.tb2, h.tb3, h.tb4, h.tb5, h.tb6, h.tb7, b); \
    return hipGetLastError(); }
#define OAC_GSS(NW_, G_) \
  if (nw == NW_ && gpw == G_ && stg) { \
    if (shm > 64 * 1024) { \
      const hipError_t ea = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_small_kernel<NW_, G_, true>), \
          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm); \
      if (ea != hipSuccess) return ea; } \
    OAC_LAUNCH((gemm_small_kernel<NW_, G_, true>), dim3(grid), dim3(64 * NW_), shm, s, h.total_tiles, h.publish, \
               h.tb1, h.tb2, h.tb3, h.tb4, h.tb5, h.tb6, h.tb7, b); \
    return hipGetLastError(); }
  // staged operands: LDS fragment reads need fewer k-groups in flight (8 waves: 4)
  OAC_GSS(8, 4) OAC_GSS(16, 4)
#undef OAC_GSS
  OAC_GS(1, 5) OAC_GS(2, 5) OAC_GS(4, 5) OAC_GS(8, 5) OAC_GS(16, 4)
  OAC_GS(4, 3) OAC_GS(4, 4) OAC_GS(4, 6) OAC_GS(4, 8)
  OAC_GS(8, 3) OAC_GS(8, 4) OAC_GS(8, 6) OAC_GS(8, 8)
  OAC_GS(16, 2) OAC_GS(16, 3) OAC_GS(16, 5) OAC_GS(16, 6)
#undef OAC_GS
  return hipErrorInvalidValue;
}

}  // namespace oac
