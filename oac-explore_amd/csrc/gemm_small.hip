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
// * The dL/da launch's head-backward tiles (EPI_HEAD_BWD with C2, the HD2
//   instance) go on from their dhead rows to a 64-column chunk of the head's
//   dX as v_mfma_f32_16x16x4_f32 tiles: one launch fewer in the step.
#include "oac_common.h"
#include "kernels.h"
#include "adam_common.h"
#include "policy_math.h"
#include "gemm_operand.h"

#include <algorithm>
#include <cstddef>
#include <cstring>

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

#ifdef OAC_STAGE_CLOCK   // per-stage wall clock of thread 0 of each block (tools/micro only)
__device__ long long g_gs_clock[4096 * 8];
#define GS_STAGE(i) do { __builtin_amdgcn_s_waitcnt(0); \
  if (threadIdx.x == 0 && blockIdx.x < 4096) g_gs_clock[blockIdx.x * 8 + (i)] = wall_clock64(); } while (0)
#else
#define GS_STAGE(i)
#endif

// GemmTask::fold's per-lane sums (row m = lane & 31 over the k of this lane's
// k-groups): inside the k loop at 16 waves (105 -> 119 VGPRs, four waves per
// SIMD either way); below that in a pass of its own after the k loop, whose
// operands come back from the cache -- accumulating in the 8-wave k loop took
// that kernel from 123 to 137 VGPRs, past the 128 of two workgroups per CU
struct FoldAcc { float rs, gs, ss; };
__device__ __forceinline__ void fold_add(FoldAcc& fa, const Lane& la, int k, int k_hi, float a,
                                         float x, float y) {
  const bool kin = k < k_hi;
  fa.rs += a;                                // the k loop's A value (fix1)
  fa.gs += (la.valid && kin) ? y * x : 0.f;  // s[k] x(k, m)
  fa.ss += kin ? y : 0.f;                    // s[k]
}
// acc += A[m0.., k_lo..k_hi) . B[k_lo..k_hi), n0..]  for this wave's k-groups
// arow >= 0: this lane's A row is buffer row arow (the direct gather's index,
// loaded by the caller ahead of everything else)
template <int NW>
__device__ __forceinline__ FoldAcc fold_pass(const GemmTask& t, int m0, int k_lo, int k_hi) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l32 = lane & 31, half = lane >> 5;
  const Lane la = lane_init<OP_MN_R1>(m0 + l32, t.M, false, t.a_mask, t.ld_mask, t.a_s, t.a_v);
  const int g_lo = k_lo >> 3, g_hi = (k_hi + 7) >> 3, kmax = k_hi - 1;
  FoldAcc fa{0.f, 0.f, 0.f};
#pragma unroll 1
  for (int g0 = g_lo + wave; g0 < g_hi; g0 += 2 * NW) {   // two groups in flight
    float x0[4], y0[4], x1[4], y1[4];
    const int kb0 = 8 * g0 + 4 * half, kb1 = kb0 + 8 * NW;
    const bool two = g0 + NW < g_hi;
    load4<OP_MN_R1>(la, kb0, kmax, x0, y0);
    if (two) load4<OP_MN_R1>(la, kb1, kmax, x1, y1);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      fold_add(fa, la, kb0 + c, k_hi, fix1<OP_MN_R1>(la, kb0 + c, k_hi, x0[c], y0[c]), x0[c], y0[c]);
    if (two) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        fold_add(fa, la, kb1 + c, k_hi, fix1<OP_MN_R1>(la, kb1 + c, k_hi, x1[c], y1[c]), x1[c], y1[c]);
    }
  }
  return fa;
}

template <int NW, int AK, int BK, int GPW = (NW >= 16 ? 4 : 5), bool FOLD = false>
__device__ __forceinline__ void k_loop(const GemmTask& t, int m0, int n0, int k_lo, int k_hi,
                                       floatx16& acc, int arow, FoldAcc& fa) {
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
  // direct rows (the drop-in layer-0 launch: random replay rows, from HBM):
  // the A fragment of the wave's first group of its second pass, requested
  // with the first pass's loads, so that pass waits on one row fetch, not two
  const int g_pf = g_lo + wave + kGPW * NW;
  const bool pf = (AK == OP_KC) && arow >= 0 && g_pf < g_hi;   // (wave-uniform)
  float px[4] = {0.f, 0.f, 0.f, 0.f}, py[4];
  if (pf) load4<AK>(la, 8 * g_pf + 4 * half, kmax, px, py);
#pragma unroll 1
  for (int g0 = g_lo + wave; g0 < g_hi; g0 += kGPW * NW) {
    float ax[kGPW][4], ay[kGPW][4], bx[kGPW][4], by[kGPW][4];
#pragma unroll
    for (int j = 0; j < kGPW; ++j)
      if (g0 + j * NW < g_hi) {
        const int kb = 8 * (g0 + j * NW) + 4 * half;
        load4<BK>(lb, kb, kmax, bx[j], by[j]);   // B first: it never waits on a row index
        if (j == 0 && pf && g0 == g_pf) {
#pragma unroll
          for (int c = 0; c < 4; ++c) ax[j][c] = px[c];
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
          if constexpr (FOLD) fold_add(fa, la, kb + c, k_hi, a, ax[j][c], ay[j][c]);
        }
      }
  }
}

template <int NW, int GPW, bool FOLDK>
__device__ __forceinline__ void k_dispatch(const GemmTask& t, int m0, int n0, int k_lo, int k_hi,
                                           floatx16& acc, int arow, bool fold, FoldAcc& fa) {
  const bool r1 = t.a_mode == A_RANK1_MASK;
  if (t.a_kc && t.b_kc)        k_loop<NW, OP_KC, OP_KC, GPW>(t, m0, n0, k_lo, k_hi, acc, arow, fa);   // forward
  else if (t.a_kc && !r1)      k_loop<NW, OP_KC, OP_MN, GPW>(t, m0, n0, k_lo, k_hi, acc, -1, fa);      // dX
  else if (t.a_kc)             k_loop<NW, OP_KC_R1, OP_MN, GPW>(t, m0, n0, k_lo, k_hi, acc, -1, fa);   // dX, rank-1 seed
  else if (!r1)                k_loop<NW, OP_MN, OP_MN, GPW>(t, m0, n0, k_lo, k_hi, acc, -1, fa);      // dW
  else if (FOLDK && NW >= 16 && fold)
    k_loop<NW, OP_MN_R1, OP_MN, GPW, FOLDK>(t, m0, n0, k_lo, k_hi, acc, -1, fa);   // dW + fold
  else                         k_loop<NW, OP_MN_R1, OP_MN, GPW>(t, m0, n0, k_lo, k_hi, acc, -1, fa);   // dW, rank-1 seed
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
      if (batch.fuse_adam && !t.no_adam) {
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
    case EPI_ADD_RELU: case EPI_MASK:
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
      if (batch.fuse_adam && !t.no_adam) {   // adam_elem on the prefetched p, m, v, target
        const long i = g - batch.adam.g;
        float p = x.xb, m = x.am, v = x.av;
        adam1(ac, p, acc, m, v);
        (batch.adam.p_out ? batch.adam.p_out : batch.adam.p)[i] = p;
        if (!batch.adam.preview) {
          batch.adam.m[i] = m; batch.adam.v[i] = v;
          if (ac.polyak) batch.adam.target[i] = polyak1(ac, x.at, p);
        }
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
    case EPI_MASK: t.C[o] = x.xa > 0.f ? acc : 0.f; break;
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
template <int NW, bool FOLDK = false>
struct SmallLds {
  static constexpr int RED = NW * 16 * 64;   // partial tiles: NW x 16 regs x 64 lanes
  static constexpr int FOLD = RED > 2 * 32 * 65 ? RED : 2 * 32 * 65;   // (before: the epilogue operands)
  static constexpr int N = FOLD + (FOLDK ? NW * 65 : 0);   // + the fold's per-wave sums [rs 32 | gs 32 | ss 1]
};

// GemmTask::fold: one folded gradient element's value -> the gradient arena,
// and with the fused optimizer its Adam (+ Polyak) on the prefetched p, m, v, t
// (as epi_one's EPI_GRAD elements)
struct FoldIn { float p, m, v, t; };
__device__ __forceinline__ FoldIn fold_prefetch(const GemmBatch& batch, const float* g) {
  FoldIn x{0.f, 0.f, 0.f, 0.f};
  const long i = g - batch.adam.g;
  x.p = batch.adam.p[i]; x.m = batch.adam.m[i]; x.v = batch.adam.v[i];
  if (batch.adam.target) x.t = batch.adam.target[i];
  return x;
}
__device__ __forceinline__ void fold_store(const GemmBatch& batch, const AdamConsts& ac, bool adam,
                                           float* g, float val, FoldIn x) {
  *g = val;
  if (!adam) return;
  const long i = g - batch.adam.g;
  float p = x.p, m = x.m, v = x.v;
  adam1(ac, p, val, m, v);
  (batch.adam.p_out ? batch.adam.p_out : batch.adam.p)[i] = p;
  if (!batch.adam.preview) {
    batch.adam.m[i] = m; batch.adam.v[i] = v;
    if (ac.polyak) batch.adam.target[i] = polyak1(ac, x.t, p);
  }
}

constexpr int kGatherU = 4;   // float4s per lane of a side block's row copy (rows <= 1 KB)

// one 16x16 tile of the head's dX over KS k-steps of 4: A from the dhead rows
// in LDS (arow: the lane's row at its k-group; zeros past 2N), B the lane's
// prefetched weights (k-step order, a fixed order per output)
template <int KS>
__device__ __forceinline__ floatx4 hd_mfma(const float* arow, const float (&hb)[12]) {
  float a[KS];
#pragma unroll
  for (int st = 0; st < KS; ++st) a[st] = arow[4 * st];
  floatx4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < KS; ++st) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[st], hb[st], c, 0, 0, 0);
  return c;
}

// FOLDK: the kernel that takes GemmTask::fold tasks (a variant of its own, so
// the other launches keep the registers and schedule of the plain kernel:
// with the fold in every kernel, launches without a fold task came out
// 0.2-0.4 us slower)
// HD2: the kernel that takes EPI_HEAD_BWD tasks with the head's dX chunk
// (GemmTask::C2; its own instance, as FOLDK, so the other launches keep
// their registers and schedule)
template <int NW, int GPW, bool FOLDK = false, bool HD2 = false>
__device__ __forceinline__ void gemm_small_block(int bid, int total_tiles, int publish, int tb1,
                                                 int tb2, int tb3, int tb4, int tb5, int tb6,
                                                 int tb7, const GemmBatch& batch, float* red,
                                                 const int* inl = nullptr) {
  constexpr int PER = 1024 / (64 * NW);   // epilogue elements per thread
  GS_STAGE(0);
  if (publish && bid == 0 && threadIdx.x == 0)
    publish_step_consts(batch.publish, batch.pub_beta1, batch.pub_beta2);
  const int* rows = nullptr;   // direct drop-in gather: this step's index slot (host memory)
  long long bc = 0;
  if (inl) {   // the indices in the kernel arguments (gemm_small_kernel_inl)
    bc = batch.rg.state->batch_counter;
    rows = inl;
  } else if (batch.rg.ring) {
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
    if (a.copy_src) {   // (or the copy of updates an earlier launch computed into a.copy_src)
      const long stride = (long)batch.adam_blocks * 64 * NW;
      for (int sgi = 0; sgi < batch.nseg; ++sgi) {
        const float4* src = reinterpret_cast<const float4*>(a.copy_src + batch.seg_off[sgi]);
        float4* dst = reinterpret_cast<float4*>(a.p + batch.seg_off[sgi]);
        const long n4 = batch.seg_n[sgi] >> 2;
        for (long i = (long)(bid - total_tiles) * 64 * NW + threadIdx.x; i < n4; i += stride)
          dst[i] = src[i];
      }
      return;
    }
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
    __shared__ int tile_rows[32];
    if (wave == 0 && lane < 32) tile_rows[lane] = rows[min(m0 + lane, t.M - 1)];
    __syncthreads();
    arow = tile_rows[lane & 31];
  }

  EpiIn xin[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * 64 * NW;
    const int r = e >> 6, l = e & 63;
    xin[i] = epi_prefetch(batch, t, m0 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), n0 + (l & 31));
  }
  // GemmTask::fold (first column block): thread f < 32 finishes row m0 + f's
  // bias-column and width-1-layer sums, thread 32 (tile m0 = 0) the seed sum
  const bool fold = FOLDK && t.fold && n0 == 0;   // (workgroup-uniform)
  const bool fold_adam = fold && batch.fuse_adam && !t.no_adam;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  // EPI_HEAD_BWD with C2: the head's dX for the task's R hidden columns from
  // this tile's own dhead rows, as v_mfma_f32_16x16x4_f32 tiles (lane l:
  // A[l&15][k=l>>4], B[k=l>>4][l&15]; D reg r: row 4*(l>>4)+r, col l&15):
  // wave w takes row tile w & 1 and column tile w >> 1 (R <= 8 NW).  Its B
  // operands (the head weights, 2N <= 48 k) and the ReLU mask of its outputs
  // are requested ahead: before the k loop on 16 waves (122 VGPRs), after it
  // on 8 (held across the 8-wave loop they took it to 141, one workgroup per CU)
  constexpr int kHdS = 12;   // k-steps of 4 (2N <= 48)
  const bool hd = HD2 && t.epi == EPI_HEAD_BWD && t.C2 != nullptr;   // (workgroup-uniform)
  float hb[HD2 ? kHdS : 1], hm[4];
  auto hd_prefetch = [&]() {
    const int l16 = lane & 15, g4 = lane >> 4, n2 = 2 * t.N;
    const int col = (wave >> 1) * 16 + l16;
    const bool cv = col < t.R;
#pragma unroll
    for (int st = 0; st < kHdS; ++st) {
      const int k = 4 * st + g4;
      hb[st] = (cv && k < n2) ? t.U[(long)k * t.ldu + col] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 16 * (wave & 1) + 4 * g4 + r;
      hm[r] = (cv && m < t.M) ? t.aux[(long)m * t.ld_aux + col] : 0.f;
    }
  };
  if constexpr (HD2 && NW >= 16)
    if (hd) hd_prefetch();

  FoldAcc fa{0.f, 0.f, 0.f};
  k_dispatch<NW, GPW, FOLDK>(t, m0, n0, k_lo, k_hi, acc, arow, fold, fa);
  if constexpr (FOLDK && NW < 16)
    if (fold) fa = fold_pass<NW>(t, m0, k_lo, k_hi);
  // the folded elements' optimizer operands, requested now: their latency
  // behind the LDS reduction (held across the k loop they cost registers)
  FoldIn fb{}, fw{};
  if (fold_adam && threadIdx.x < 33) {
    const int fm = min(m0 + (int)threadIdx.x, t.M - 1);
    fb = fold_prefetch(batch, threadIdx.x < 32 ? t.bias_grad + fm : t.C2 + t.ldc2);
    fw = fold_prefetch(batch, t.C2 + fm);
  }

  if (t.K2 > 0) {   // second product into the same accumulator (unsplit dX tasks only)
    GemmTask t2 = t;
    t2.A = t.A2; t2.B = t.B2; t2.K = t.K2;
    k_loop<NW, OP_KC, OP_MN, GPW>(t2, m0, n0, 0, t.K2, acc, -1, fa);
  }
  if constexpr (HD2 && NW < 16)
    if (hd) hd_prefetch();
  GS_STAGE(2);
  // fixed-order split-K reduction through LDS
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(wave * 16 + r) * 64 + lane] = acc[r];
  float* fred = red + SmallLds<NW, FOLDK>::FOLD;
  if (fold) {   // the two halves' k, then one slot per wave
    fa.rs += __shfl_xor(fa.rs, 32);
    fa.gs += __shfl_xor(fa.gs, 32);
    fa.ss += __shfl_xor(fa.ss, 32);
    if (lane < 32) { fred[wave * 65 + lane] = fa.rs; fred[wave * 65 + 32 + lane] = fa.gs; }
    if (lane == 0) fred[wave * 65 + 64] = fa.ss;
  }
  __syncthreads();
  float fsum_a = 0.f, fsum_b = 0.f;   // (waves in order)
  if (fold && threadIdx.x < 33) {
    const int f = threadIdx.x;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      fsum_a += fred[w * 65 + (f < 32 ? f : 64)];
      if (f < 32) fsum_b += fred[w * 65 + 32 + f];
    }
  }
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
  if constexpr (HD2) {
    if (hd) {   // the head backward, then its dX columns
      __syncthreads();   // (every wave's reads of the partial tiles are done: the LDS is reused)
      constexpr int kDh = 65;   // dhead row stride in LDS (odd: a column read is conflict-free)
      float* dh = red;          // [32][kDh]: dmean | dls_raw of the tile's rows
      const int N = t.N;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = threadIdx.x + i * 64 * NW;
        const int r = e >> 6, l = e & 63;
        const int mt = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), nt = l & 31;
        const int m = m0 + mt, n = n0 + nt;
        float dmean = 0.f, dls = 0.f;
        if (m < t.M && n < N) {
          const EpiIn x = xin[i];
          tanh_gauss_backward(vals[i], x.xb, x.xa, x.am, x.av, x.at, x.s * (1.f / (float)t.M), dmean,
                              dls);
          if (!t.dup) {
            const long o = (long)m * t.ldc + n;
            t.C[o] = dmean;
            t.C[o + N] = dls;
          }
        }
        if (n < N) { dh[mt * kDh + n] = dmean; dh[mt * kDh + N + n] = dls; }
      }
      for (int e = threadIdx.x; e < 32 * 64; e += 64 * NW)   // k past 2N: zeros (fixed-length MFMA runs)
        if ((e & 63) >= 2 * N) dh[(e >> 6) * kDh + (e & 63)] = 0.f;
      __syncthreads();
      const int l16 = lane & 15, g4 = lane >> 4, ksteps = (2 * N + 3) >> 2;
      const int rt = 16 * (wave & 1), col = (wave >> 1) * 16 + l16;
      if ((wave >> 1) * 16 < t.R) {   // (wave-uniform)
        const float* arow = dh + (rt + l16) * kDh + g4;
        const floatx4 c = ksteps <= 8 ? hd_mfma<8>(arow, hb) : hd_mfma<12>(arow, hb);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float mk = hm[r];
          asm volatile("" : "+v"(mk));   // (the mask's wait here, after the MFMAs, not at its load)
          const int m = m0 + rt + 4 * g4 + r;
          if (col < t.R && m < t.M) t.C2[(long)m * t.ldc2 + col] = mk > 0.f ? c[r] : 0.f;
        }
      }
      if (batch.fuse_adam && !batch.adam.no_book && bid == 0 && threadIdx.x == 0)
        step_bookkeeping(batch.adam.state, batch.adam.alpha, batch.adam.advance);
      return;
    }
  }
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
  if (fold && threadIdx.x < 32 && m0 + (int)threadIdx.x < t.M) {
    const int m = m0 + threadIdx.x;
    fold_store(batch, ac, fold_adam, t.bias_grad + m, fsum_a, fb);
    fold_store(batch, ac, fold_adam, t.C2 + m, fsum_b, fw);
  } else if (fold && threadIdx.x == 32 && m0 == 0) {
    fold_store(batch, ac, fold_adam, t.C2 + t.ldc2, fsum_a, fb);
  }
  if (batch.fuse_adam && !batch.adam.no_book && bid == 0 && threadIdx.x == 0)
    step_bookkeeping(batch.adam.state, batch.adam.alpha, batch.adam.advance);
  GS_STAGE(4);
}

template <int NW, int GPW, bool FOLDK = false, bool HD2 = false>
__global__ void __launch_bounds__(64 * NW)
gemm_small_kernel(int total_tiles, int publish, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6,
                  int tb7, const GemmBatch batch) {
  static_assert(!HD2 || (NW >= 8 && SmallLds<NW, FOLDK>::N >= 32 * 65), "HD2: 8+ waves, dhead in LDS");
  __shared__ __attribute__((aligned(16))) float red[SmallLds<NW, FOLDK>::N];
  gemm_small_block<NW, GPW, FOLDK, HD2>(blockIdx.x, total_tiles, publish, tb1, tb2, tb3, tb4, tb5,
                                        tb6, tb7, batch, red);
}

// The direct drop-in layer-0 launch with the step's B <= 256 indices in the
// kernel arguments: no dependent read of the host-coherent slot before the
// tiles can request their rows.
struct InlineRows { int r[kInlineRows]; };
// (read in place in the kernel-argument segment: taking the address of the
// by-value argument made the compiler copy its 1 KB into every thread's
// scratch -- 1,028 bytes of private segment, that launch 11.7 -> 45.8 us)
// The kernel-argument segment lays the arguments out as this struct does
// (each at its own alignment, in order): it mirrors gemm_small_kernel_inl's
// parameter list, which must change with it.
struct InlineKernArgs {
  int total_tiles, publish, tb1, tb2, tb3, tb4, tb5, tb6, tb7;
  GemmBatch batch;
  InlineRows ir;
};
constexpr size_t kInlineRowsOff = offsetof(InlineKernArgs, ir);
static_assert(offsetof(InlineKernArgs, batch) % alignof(GemmBatch) == 0 &&
                  kInlineRowsOff == offsetof(InlineKernArgs, batch) + sizeof(GemmBatch),
              "inline rows must follow the batch argument directly");
template <int NW, int GPW>
__global__ void __launch_bounds__(64 * NW)
gemm_small_kernel_inl(int total_tiles, int publish, int tb1, int tb2, int tb3, int tb4, int tb5,
                      int tb6, int tb7, const GemmBatch batch, const InlineRows ir) {
  __shared__ __attribute__((aligned(16))) float red[SmallLds<NW>::N];
  (void)ir;
  const __attribute__((address_space(4))) char* ka =
      (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
  const int* rows = (const int*)(ka + kInlineRowsOff);
  gemm_small_block<NW, GPW>(blockIdx.x, total_tiles, publish, tb1, tb2, tb3, tb4, tb5, tb6, tb7,
                            batch, red, rows);
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

// (bc / pos: the launch records in device memory, kernels.h BatchCache -- not
// taken here: at B=256 the small kernel's launches measured the same either way,
// some launches 0.3-0.6 us faster and others as much slower, where the
// pipelined large-batch kernels gained, tools/gpu_r5_t14.sh)
hipError_t gemm_small_launch(const GemmBatch& b0, hipStream_t s, BatchCache* bc = nullptr, int pos = -1) {
  (void)bc; (void)pos;
  if (b0.total_tiles <= 0) return hipSuccess;
  GemmBatch b = b0;
  for (int i = 0; i < b.ntasks; ++i)   // second products: plain unsplit dX tasks
    if (b.t[i].K2 > 0 && (b.t[i].ksplit > 1 || !b.t[i].a_kc || b.t[i].b_kc ||
                          b.t[i].a_mode != A_PLAIN))
      return hipErrorInvalidValue;
  int nw = b.force_nw > 0 ? b.force_nw : gemm_small_waves(b);
  int gpw = b.force_gpw > 0 ? b.force_gpw : (nw >= 16 ? 4 : 5);
  b.adam_blocks = 0;
  if (b.fuse_adam) {
    long n4 = 0;
    for (int i = 0; i < b.nseg; ++i) {
      if ((b.seg_n[i] | b.seg_off[i]) & 3) return hipErrorInvalidValue;
      n4 = std::max(n4, b.seg_n[i] >> 2);
    }
    b.adam_blocks = (int)std::min<long>((n4 + 64 * nw - 1) / (64 * nw), 1024);
    if (b.adam_blocks < 1 && b.nseg > 0) b.adam_blocks = 1;
  }
  const int grid = b.total_tiles + b.adam_blocks + (b.rg.ring ? b.rg.blocks : 0);
  const GemmHead h = gemm_head(b);
  const bool inl = b.rg.inl && b.rg.ring && b.rg.B <= kInlineRows &&
                   ((nw == 16 && gpw == 4) || (nw == 8 && gpw == 5));
  bool has_fold = false, has_hd = false;
  for (int i = 0; i < b.ntasks; ++i) {
    has_fold = has_fold || b.t[i].fold;
    const GemmTask& t = b.t[i];
    if (t.epi == EPI_HEAD_BWD && t.C2) {   // the head's dX chunk: dhead and the weights in LDS
      if (t.N > 24 || t.R < 1 || t.R > 256 || t.tiles_n != 1 || t.ksplit > 1)
        return hipErrorInvalidValue;
      has_hd = true;
    }
  }
  if (has_fold && inl) return hipErrorInvalidValue;   // (no fold task in a row-gathering launch)
  if (has_hd && (has_fold || inl)) return hipErrorInvalidValue;
  if (has_hd) {   // the head-dX kernels: 8 or 16 waves (a thread's share of the chunk)
    // (a 16-column tile per wave, NW / 2 waves per row tile -> R <= 8 NW)
    int rmax = 0;
    for (int i = 0; i < b.ntasks; ++i)
      if (b.t[i].epi == EPI_HEAD_BWD && b.t[i].C2) rmax = std::max(rmax, b.t[i].R);
    if (b0.force_nw <= 0 && (nw < 8 || (nw < 16 && rmax > 8 * nw))) {
      nw = rmax > 64 ? 16 : 8;
      gpw = b0.force_gpw > 0 ? b0.force_gpw : (nw >= 16 ? 4 : 5);
    }
    if (rmax > 8 * nw) return hipErrorInvalidValue;
    if (nw == 16 && gpw == 4)
      OAC_LAUNCH((gemm_small_kernel<16, 4, false, true>), dim3(grid), dim3(64 * 16), 0, s, h.total_tiles,
                 h.publish, h.tb1, h.tb2, h.tb3, h.tb4, h.tb5, h.tb6, h.tb7, b);
    else if (nw == 8 && gpw == 5)
      OAC_LAUNCH((gemm_small_kernel<8, 5, false, true>), dim3(grid), dim3(64 * 8), 0, s, h.total_tiles,
                 h.publish, h.tb1, h.tb2, h.tb3, h.tb4, h.tb5, h.tb6, h.tb7, b);
    else
      return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (inl) {
    InlineRows ir;
    std::memcpy(ir.r, b.rg.inl, sizeof(int) * b.rg.B);
    if (nw == 16)
      OAC_LAUNCH((gemm_small_kernel_inl<16, 4>), dim3(grid), dim3(64 * 16), 0, s, h.total_tiles, h.publish,
                 h.tb1, h.tb2, h.tb3, h.tb4, h.tb5, h.tb6, h.tb7, b, ir);
    else
      OAC_LAUNCH((gemm_small_kernel_inl<8, 5>), dim3(grid), dim3(64 * 8), 0, s, h.total_tiles, h.publish,
                 h.tb1, h.tb2, h.tb3, h.tb4, h.tb5, h.tb6, h.tb7, b, ir);
    return hipGetLastError();
  }
  if (has_fold) {   // the fold kernels: the default wave / k-group pairs only
#define OAC_GSF(NW_, G_) \
    if (nw == NW_ && gpw == G_) { \
      OAC_LAUNCH((gemm_small_kernel<NW_, G_, true>), dim3(grid), dim3(64 * NW_), 0, s, h.total_tiles, \
                 h.publish, h.tb1, h.tb2, h.tb3, h.tb4, h.tb5, h.tb6, h.tb7, b); \
      return hipGetLastError(); }
    OAC_GSF(1, 5) OAC_GSF(2, 5) OAC_GSF(4, 5) OAC_GSF(8, 5) OAC_GSF(16, 4)
#undef OAC_GSF
    return hipErrorInvalidValue;
  }
#define OAC_GS(NW_, G_) \
  if (nw == NW_ && gpw == G_) { \
    OAC_LAUNCH((gemm_small_kernel<NW_, G_>), dim3(grid), dim3(64 * NW_), 0, s, h.total_tiles, h.publish, \
               h.tb1, h.tb2, h.tb3, h.tb4, h.tb5, h.tb6, h.tb7, b); \
    return hipGetLastError(); }
  OAC_GS(1, 5) OAC_GS(2, 5) OAC_GS(4, 5) OAC_GS(8, 5) OAC_GS(16, 4)
  OAC_GS(4, 3) OAC_GS(4, 4) OAC_GS(4, 6) OAC_GS(4, 8)
  OAC_GS(8, 3) OAC_GS(8, 4) OAC_GS(8, 6) OAC_GS(8, 8)
  OAC_GS(16, 2) OAC_GS(16, 3) OAC_GS(16, 5) OAC_GS(16, 6)
#undef OAC_GS
  return hipErrorInvalidValue;
}

}  // namespace oac
