// Per-sample (row-parallel) kernels of the SAC/OAC step: the tanh-Gaussian
// sample + log-prob, the alpha update, the twin-min TD target and MSE
// gradients, and the policy-head backward.  All fp32, one thread per row (or
// per row x action-dim), deterministic fixed-order reductions.
#include "oac_common.h"
#include "kernels.h"
#include "adam_common.h"
#include "policy_math.h"
#include "target_math.h"

namespace oac {

__device__ __forceinline__ float mul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float add_rn(float a, float b) { return __fadd_rn(a, b); }

// --------------------------------------------------------------------------
// TanhGaussianPolicy.forward tail (trainer/policies.py:275-304):
//   log_std = clamp(ls_raw, -20, 2); std = exp(log_std); z = mean + std*eps;
//   a = tanh(z);  logp = sum_j [ -(z-mean)^2/(2 std^2) - log std - log sqrt(2pi)
//                                - log(1 - a^2 + 1e-6) ]
// One half-wave (32 lanes) per row, lane j = action dim j (act_dim <= 32);
// the sum over j is a 5-step shuffle reduction.  y-dimension 0: obs batch
// (eps1), 1: next_obs batch (eps2).
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) policy_sample_kernel(PolicySampleArgs p) {
  const PolicySampleSeg& s = p.seg[blockIdx.y];
  const int Da = p.act_dim;
  const int r = (blockIdx.x * 256 + threadIdx.x) >> 5;
  const int j = threadIdx.x & 31;
  float l = 0.f;
  if (r < p.B && j < Da) {
    const long e = (long)r * Da + j;
    const float* hd = s.head + (long)r * (2 * Da);
    float a, sd, u;
    l = tanh_gauss_sample(hd[j], hd[Da + j], s.eps[e], a, sd, u);
    s.act[e] = a;
    s.stdv[e] = sd;
    s.u[e] = u;
    if (s.act_row) s.act_row[(long)r * s.ld_act_row + j] = a;
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) l += __shfl_xor(l, o, 32);
  if (j == 0 && r < p.B) s.logp[r] = l;
}

// Deterministic block sum of (logp + target_entropy) over all B rows (every
// block computes the same value in the same order).
__device__ float block_logp_sum(const float* logp, int B, float te, float* red) {
  // the same per-thread order, loads issued 16 at a time (target_math.h logp_sum256)
  float acc = 0.f;
  const int st = blockDim.x;
  int i = threadIdx.x;
  for (; i + 15 * st < B; i += 16 * st) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = logp[i + st * k];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += v[k] + te;
  }
  for (; i < B; i += st) acc += logp[i] + te;
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float sum = red[0];
  __syncthreads();
  return sum;
}

// Data-parallel: the all-reduced per-row-block partials of the head launch
// (HeadArgs::logp_part), summed by the whole block (one load per thread for
// n <= blockDim, then the fixed tree of block_logp_sum); every block and
// every thread gets the same value
__device__ float block_part_sum(const float* part, int n, float* red) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float sum = red[0];
  __syncthreads();
  return sum;
}

// Data-parallel: local sum(logp + target_entropy) into alpha->sum (all-reduced
// by the caller before phase 1).
__global__ void __launch_bounds__(256) logp_sum_kernel(LogpSumArgs a) {
  __shared__ float red[256];
  const float s = block_logp_sum(a.logp, a.B, a.target_entropy, red);
  if (threadIdx.x == 0) a.alpha->sum = s;
}

// --------------------------------------------------------------------------
// Twin-min TD target and critic MSE gradients (trainer/trainer.py:151-196):
//   y  = reward_scale*r + (1-d)*gamma*(min(tq1,tq2) - alpha*logp')
//   dq_i = 2 (q_i - y) / B ;  policy seed g_i = -1/B on the min critic
//   (torch-1.4 min() backward: ties go to the first argument).
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) critic_targets_kernel(CriticTargetArgs p) {
  __shared__ float red[256];
  // this row's inputs first (clamped row, all loads in flight together), so
  // their latency overlaps the alpha reduction below
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  TargetRowIn x;
  target_row_load(p, min(r, p.B - 1), x);
  // last-layer dW (p.wl_h2): thread t owns column 32 blockIdx.y + (t & 31) of
  // critic (t >> 5) & 1 over the 64 rows 64 (t >> 6) .. + 63 of this block;
  // those h2 values are requested with the row's inputs
  const bool wl = p.wl_h2[0] != nullptr;
  const int t = threadIdx.x, wi = (t >> 5) & 1, wpart = t >> 6;
  const int wn = blockIdx.y * 32 + (t & 31);
  float h2v[64];
  if (wl) {
    const float* hp = (wi ? p.wl_h2[1] : p.wl_h2[0]) + (long)(blockIdx.x * 256 + 64 * wpart) * p.wl_H + wn;
#pragma unroll
    for (int j = 0; j < 64; ++j) h2v[j] = hp[(long)j * p.wl_H];
  }
  float alpha = 0.f;
  if (p.alpha) {
    // every block computes the update identically; block 0 publishes next_*
    // (the critic Adam commits them), so no block reads what another writes
    const float S = (p.world_size > 1) ? (p.logp_part ? block_part_sum(p.logp_part, p.n_logp_part, red)
                                                      : p.alpha->sum)
                                       : logp_sum256(p.logp1, p.B, p.target_entropy, red);
    alpha = alpha_update(p, S, blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0);
  }
  if (!wl) {
    if (r >= p.B) return;
    float dq1, dq2;
    target_row(p, r, x, alpha, true, dq1, dq2);
    return;
  }
  // (wl: B % 256 == 0, every thread has a row; column group 0 writes the rows)
  __shared__ float sdq[2][256];
  __shared__ float spart[4][65];
  __shared__ float sbias[2][4];
  float dq1, dq2;
  target_row(p, r, x, alpha, blockIdx.y == 0, dq1, dq2);
  sdq[0][t] = dq1;
  sdq[1][t] = dq2;
  __syncthreads();
  {
    float s = 0.f;   // rows in order within the 64-row part
#pragma unroll
    for (int j = 0; j < 64; ++j) s = fmaf(sdq[wi][64 * wpart + j], h2v[j], s);
    spart[wpart][wi * 32 + (t & 31)] = s;
  }
  if (blockIdx.y == 0 && t < 8) {   // the bias: sum of dq_i over the part
    const int bi = t >> 2, bp = t & 3;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 64; ++j) s += sdq[bi][64 * bp + j];
    sbias[bi][bp] = s;
  }
  __syncthreads();
  const long so = (long)blockIdx.x * p.wl_slab_stride;   // this block's slab
  if (t < 64) {   // parts in order
    float s = spart[0][t];
#pragma unroll
    for (int q = 1; q < 4; ++q) s += spart[q][t];
    ((t >> 5) ? p.wl_g[1] : p.wl_g[0])[so + blockIdx.y * 32 + (t & 31)] = s;
  } else if (blockIdx.y == 0 && t < 66) {
    const int bi = t - 64;
    float s = sbias[bi][0];
#pragma unroll
    for (int q = 1; q < 4; ++q) s += sbias[bi][q];
    (bi ? p.wl_gb[1] : p.wl_gb[0])[so] = s;
  }
}

// --------------------------------------------------------------------------
// Policy-head backward: upstream dL/da from the critics (da1 + da2) and
// dL/dlogp = alpha/B, through log_prob (policies.py:154-160), tanh,
// z = mean + std*eps, std = exp(clamp(ls_raw)) (clamp passes the gradient
// where -20 <= ls_raw <= 2).  Writes [dmean | dls_raw] per row.
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) policy_head_backward_kernel(PolicyHeadBwdArgs p) {
  const int Da = p.act_dim;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= p.B * Da) return;
  const int r = idx / Da, j = idx % Da;
  const float alpha = p.alpha ? p.alpha->alpha : 0.f;
  const float G = alpha * (1.f / (float)p.B);
  const long e = (long)r * Da + j;
  float ga = p.da1[e];
  if (p.da2) ga += p.da2[e];
  float dmean, dls;
  tanh_gauss_backward(ga, p.act[e], p.stdv[e], p.u[e], p.eps[e], p.head[(long)r * 2 * Da + Da + j], G,
                      dmean, dls);
  p.dhead[(long)r * 2 * Da + j] = dmean;
  p.dhead[(long)r * 2 * Da + Da + j] = dls;
}

}  // namespace oac

namespace oac {

hipError_t launch_policy_sample(const PolicySampleArgs& a, int nseg, hipStream_t s) {
  OAC_LAUNCH(policy_sample_kernel, dim3((a.B + 7) / 8, nseg), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_logp_sum(const LogpSumArgs& a, hipStream_t s) {
  OAC_LAUNCH(logp_sum_kernel, dim3(1), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_critic_targets(const CriticTargetArgs& a, hipStream_t s) {
  // 256 rows per block: the per-row work spreads over CUs (every block redoes
  // the 4-byte-per-row alpha reduction, which is cheap)
  if (a.wl_h2[0] && (a.B % 256 || a.wl_H % 32 || !a.wl_h2[1] || !a.wl_g[0] || !a.wl_g[1] ||
                    !a.wl_gb[0] || !a.wl_gb[1]))
    return hipErrorInvalidValue;
  OAC_LAUNCH(critic_targets_kernel, dim3((a.B + 255) / 256, a.wl_h2[0] ? a.wl_H / 32 : 1), dim3(256), 0,
             s, a);
  return hipGetLastError();
}
hipError_t launch_policy_head_backward(const PolicyHeadBwdArgs& a, hipStream_t s) {
  OAC_LAUNCH(policy_head_backward_kernel, dim3((a.B * a.act_dim + 255) / 256), dim3(256),
                     0, s, a);
  return hipGetLastError();
}

}  // namespace oac

namespace oac {

// --------------------------------------------------------------------------
// ParticleTrainer (OAC flavour, share_layers=True),
// /root/reference/trainer/particle_trainer_oac.py:185-256:
//   sorted_qs = sort_K(Q(obs, a));  tq_sorted = sort_K(TQ(next_obs, a'))
//   y_i = scale*r + (1-d)*gamma*tq_sorted_i                      (207-208)
//   qf_loss = sum_i MSE(sorted_qs_i, y_i)   (NOT divided by K)   (247-251)
// The per-sample sort over K (<= 16) is a 16-wide bitonic network on
// (value, head index) pairs -- every array index static, so the rows stay in
// registers (an insertion sort's data-dependent indexing put them in scratch:
// 11.6 us for 256 rows) -- ordering ties by head index, i.e. a stable sort;
// the gradient is scattered back through the sort permutation.
// --------------------------------------------------------------------------
constexpr int kMaxHeads = 16;

__device__ __forceinline__ void cas_kv(float& va, int& ia, float& vb, int& ib, bool up) {
  const bool gt = va > vb || (va == vb && ia > ib);
  if (gt == up) {
    const float tv = va; va = vb; vb = tv;
    const int ti = ia; ia = ib; ib = ti;
  }
}

// ascending sort of (v, ix); entries K..15 must hold +inf (and indices >= K)
__device__ __forceinline__ void sort16(float (&v)[kMaxHeads], int (&ix)[kMaxHeads]) {
#pragma unroll
  for (int k = 2; k <= kMaxHeads; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < kMaxHeads; ++i) {
        const int l = i ^ j;
        if (l > i) cas_kv(v[i], ix[i], v[l], ix[l], (i & k) == 0);
      }
}

// row r's K values (padded with +inf) and their head indices
__device__ __forceinline__ void load_row16(const float* src, int K, float (&v)[kMaxHeads],
                                           int (&ix)[kMaxHeads]) {
#pragma unroll
  for (int i = 0; i < kMaxHeads; ++i) {
    v[i] = i < K ? src[i] : __builtin_huge_valf();
    ix[i] = i;
  }
}

// Row kernels of the particle / g-oac targets and seeds: 16 rows per
// 256-thread block (thread t < 16 owns row 16 b + t).  With a RowHead set, the
// block first evaluates the critic's K-output last layer for its 16 rows as
// one 16x16 output tile of v_mfma_f32_16x16x4_f32: the hidden width is split
// over the 4 waves in 16-wide k-chunks (one 16-byte load per lane and
// operand, MFMA j of a chunk multiplies element j, as in head.hip), the wave
// partials are summed through LDS in fixed order, and the result goes to LDS
// for the row logic and to the workspace view.  This replaces the last-layer
// GEMM launch that otherwise sits between the hidden layer and this kernel.
constexpr int kRowBlock = 16;
static bool head_ok(const RowHead& h) { return !h.h || (h.w && h.b && h.out && h.H >= 1); }
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float f4a __attribute__((ext_vector_type(4), aligned(4)));

struct RowHeadLds {
  float red[4][4][64];          // wave partials
  float out[kRowBlock][kMaxHeads];
};

__device__ __forceinline__ void row_heads(const RowHead& hd, int K, int B, int r0, RowHeadLds& sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l16 = lane & 15, g4 = lane >> 4;
  const float* arow = hd.h + (long)min(r0 + l16, B - 1) * hd.H;
  const float* brow = hd.w + (long)min(l16, K - 1) * hd.H;
  const bool bv = l16 < K;
  floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
  const int chunks = (hd.H + 15) >> 4;
  if ((hd.H & 15) == 0 && hd.H <= 256) {
    // one k-batch per wave, unpredicated (clamped chunk) loads: a per-lane
    // branch between the loads and the MFMAs made them wait for every load
    constexpr int kQ = 4;
    f4a xa[kQ], xb[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const int kb = 16 * min(wave + 4 * q, chunks - 1) + 4 * g4;
      xa[q] = *reinterpret_cast<const f4a*>(arow + kb);
      xb[q] = *reinterpret_cast<const f4a*>(brow + kb);
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q)
      if (wave + 4 * q < chunks) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[q][e], bv ? xb[q][e] : 0.f, acc, 0, 0, 0);
      }
  } else {
    // up to 4 chunks per wave in flight (all of them for H <= 256): the loads
    // of a batch are issued together, then its 16 MFMAs
    constexpr int kQ = 4;
#pragma unroll 1
    for (int c0 = wave; c0 < chunks; c0 += 4 * kQ) {
      float xa[kQ][4], xb[kQ][4];
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
        const int kb = 16 * (c0 + 4 * q) + 4 * g4;
        if (kb + 3 < hd.H) {
          const f4a a = *reinterpret_cast<const f4a*>(arow + kb);
          const f4a b = *reinterpret_cast<const f4a*>(brow + kb);
          xa[q][0] = a.x; xa[q][1] = a.y; xa[q][2] = a.z; xa[q][3] = a.w;
          xb[q][0] = b.x; xb[q][1] = b.y; xb[q][2] = b.z; xb[q][3] = b.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            xa[q][e] = kb + e < hd.H ? arow[kb + e] : 0.f;
            xb[q][e] = kb + e < hd.H ? brow[kb + e] : 0.f;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < kQ; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[q][e], bv ? xb[q][e] : 0.f, acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) sh.red[wave][r][lane] = acc[r];
  __syncthreads();
  {
    const int r = threadIdx.x >> 6, l = threadIdx.x & 63;   // D reg r of lane l
    const int row = 4 * (l >> 4) + r, col = l & 15;
    const float v = ((sh.red[0][r][l] + sh.red[1][r][l]) + sh.red[2][r][l]) + sh.red[3][r][l];
    if (col < K) {
      const float o = v + hd.b[col];
      sh.out[row][col] = o;
      if (r0 + row < B) hd.out[(long)(r0 + row) * K + col] = o;
    }
  }
}

// Two K-output heads of the same hidden width for the same 16 rows (the
// targets kernel's target critic and critic): all loads of both issued
// before the first MFMA, one LDS round.  Same per-head MFMA order as
// row_heads.  H % 16 == 0 and H <= 256 (one k-batch per wave).
__device__ __forceinline__ void row_heads2(const RowHead& h0, const RowHead& h1, int K, int B, int r0,
                                           RowHeadLds& s0, RowHeadLds& s1) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int H = h0.H, chunks = H >> 4;
  const long ra = (long)min(r0 + l16, B - 1) * H, rb = (long)min(l16, K - 1) * H;
  const bool bv = l16 < K;
  constexpr int kQ = 4;
  f4a x0[kQ], w0[kQ], x1[kQ], w1[kQ];
#pragma unroll
  for (int q = 0; q < kQ; ++q) {   // unpredicated (clamped chunk): no branch before the MFMAs
    const int kb = 16 * min(wave + 4 * q, chunks - 1) + 4 * g4;
    x0[q] = *reinterpret_cast<const f4a*>(h0.h + ra + kb);
    w0[q] = *reinterpret_cast<const f4a*>(h0.w + rb + kb);
    x1[q] = *reinterpret_cast<const f4a*>(h1.h + ra + kb);
    w1[q] = *reinterpret_cast<const f4a*>(h1.w + rb + kb);
  }
  floatx4 acc0 = floatx4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
  for (int q = 0; q < kQ; ++q)
    if (wave + 4 * q < chunks) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[q][e], bv ? w0[q][e] : 0.f, acc0, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[q][e], bv ? w1[q][e] : 0.f, acc1, 0, 0, 0);
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) { s0.red[wave][r][lane] = acc0[r]; s1.red[wave][r][lane] = acc1[r]; }
  __syncthreads();
  const int r = threadIdx.x >> 6, l = threadIdx.x & 63;   // D reg r of lane l
  const int row = 4 * (l >> 4) + r, col = l & 15;
  if (col < K) {
    const float v0 = ((s0.red[0][r][l] + s0.red[1][r][l]) + s0.red[2][r][l]) + s0.red[3][r][l];
    const float v1 = ((s1.red[0][r][l] + s1.red[1][r][l]) + s1.red[2][r][l]) + s1.red[3][r][l];
    const float o0 = v0 + h0.b[col], o1 = v1 + h1.b[col];
    s0.out[row][col] = o0;
    s1.out[row][col] = o1;
    if (r0 + row < B) {
      h0.out[(long)(r0 + row) * K + col] = o0;
      h1.out[(long)(r0 + row) * K + col] = o1;
    }
  }
}

__device__ __forceinline__ void particle_targets_rows(const ParticleTargetArgs& p, RowHeadLds& hs,
                                                      RowHeadLds& qs,
                                                      float (&sdq)[kRowBlock][kMaxHeads]) {
  const int r0 = blockIdx.x * kRowBlock, r = r0 + threadIdx.x;
  const int K = p.K;
  if (p.th.h && p.qh.h && p.th.H == p.qh.H && (p.th.H & 15) == 0 && p.th.H <= 256) {
    row_heads2(p.th, p.qh, K, p.B, r0, hs, qs);   // both heads, loads issued together
    __syncthreads();
  } else {
    if (p.th.h) {
      row_heads(p.th, K, p.B, r0, hs);
      __syncthreads();
    }
    if (p.qh.h) {   // the critic's own last layer on (obs, a) (particle_trainer_oac.py:185-191)
      row_heads(p.qh, K, p.B, r0, qs);
      __syncthreads();
    }
  }
  // both sorts by the whole block: 16 lanes per row, lane k ranks its value
  // against the row's 16 (ties by head index, the padding slots past K last)
  // -- the order sort16's comparator defines, so the same permutation -- and
  // scatters it into LDS; a row thread's bitonic network was ~1,000 dependent
  // VALU ops.  The order is total: NaN ranks after every number, as in
  // torch.sort (a diverged critic then gives NaN losses, and every rank is
  // still taken exactly once, so the scatters below stay inside [0, K)).
  __shared__ float s_qv[kRowBlock][kMaxHeads], s_tv[kRowBlock][kMaxHeads];
  __shared__ int s_qi[kRowBlock][kMaxHeads], s_ti[kRowBlock][kMaxHeads];
  {
    static_assert(kRowBlock * kMaxHeads == 256, "one thread per (row, head slot)");
    const int row = threadIdx.x >> 4, k = threadIdx.x & 15, m = min(r0 + row, p.B - 1);
    const int base = (threadIdx.x & 63) & ~15;
    const float inf = __builtin_huge_valf();
    const float qv = k < K ? (p.qh.h ? qs.out[row][k] : p.q[(long)m * K + k]) : inf;
    const float tv = k < K ? (p.th.h ? hs.out[row][k] : p.tq[(long)m * K + k]) : inf;
    // order-preserving integer keys, computed once per lane: a number's bits
    // mapped monotonically (-0 as +0: they compare equal), NaN above +inf,
    // the padding above NaN; ties (equal keys) by index
    auto key = [](float v, bool pad) -> unsigned {
      if (pad) return 0xFFFFFFFFu;
      if (v != v) return 0xFFFFFFFEu;
      const unsigned u = __float_as_uint(v == 0.f ? 0.f : v);
      return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    };
    const unsigned kq = key(qv, k >= K), kt = key(tv, k >= K);
    int rq = 0, rt = 0;
#pragma unroll
    for (int j = 0; j < kMaxHeads; ++j) {
      const unsigned qj = (unsigned)__shfl((int)kq, base | j, 64);
      const unsigned tj = (unsigned)__shfl((int)kt, base | j, 64);
      rq += (qj < kq || (qj == kq && j < k)) ? 1 : 0;
      rt += (tj < kt || (tj == kt && j < k)) ? 1 : 0;
    }
    s_qv[row][rq] = qv; s_qi[row][rq] = k;
    s_tv[row][rt] = tv; s_ti[row][rt] = k;
  }
  __syncthreads();
  if (threadIdx.x >= kRowBlock || r >= p.B) return;
  const float fK = (float)K;
  float q[kMaxHeads], t[kMaxHeads];
  int qi[kMaxHeads], tix[kMaxHeads];
#pragma unroll
  for (int i = 0; i < kMaxHeads; ++i) {
    q[i] = s_qv[threadIdx.x][i]; qi[i] = s_qi[threadIdx.x][i];
    t[i] = s_tv[threadIdx.x][i]; tix[i] = s_ti[threadIdx.x][i];
  }
  const float rew = p.batch[(long)r * p.ld_batch + p.off_rew];
  const float term = p.batch[(long)r * p.ld_batch + p.off_term];
  const float invB = 1.f / (float)p.B;
  const float sr = __fmul_rn(p.reward_scale, rew);
  const float gd = __fmul_rn(1.f - term, p.discount);
  float y[kMaxHeads];
#pragma unroll
  for (int i = 0; i < kMaxHeads; ++i) y[i] = __fadd_rn(sr, __fmul_rn(gd, t[i]));
  // sums over the K valid slots, in slot order
  auto mean_k = [&](const float (&a)[kMaxHeads]) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kMaxHeads; ++i) if (i < K) s += a[i];
    return s / fK;
  };
  // std_soft_update (particle_trainer.py:222-231): current sorted predictions
  // re-centred on the next-value mean, mixed with the next values
  if (p.soft_prob >= 0.f) {
    const float mq = mean_k(q), my = mean_k(y);
    const float w = 1.f - p.soft_prob;
#pragma unroll
    for (int i = 0; i < kMaxHeads; ++i)
      if (i < K) y[i] = __fadd_rn(__fmul_rn(p.soft_prob, y[i]), __fmul_rn(w, (q[i] - mq) + my));
  }
  // counts=True (particle_trainer_oac.py:220-224, particle_trainer.py:236-241):
  // a row drawn before (count > 0) gets the sorted predictions re-centred on
  // the target mean, y_i <- (sorted_q_i - mean_k sorted_q) + mean_k y
  if (p.counts && p.counts[r] != 0.f) {
    const float mq = mean_k(q), my = mean_k(y);
#pragma unroll
    for (int i = 0; i < kMaxHeads; ++i)
      if (i < K) y[i] = (q[i] - mq) + my;
  }
  // rescale_targets_around_mean (particle_trainer.py:254-262): a target spread
  // wider than q_max - q_min is shrunk around its mean to that width
  if (p.rescale_spread > 0.f) {
    float ylast = y[0];
#pragma unroll
    for (int i = 1; i < kMaxHeads; ++i) if (i == K - 1) ylast = y[i];
    const float range = ylast - y[0];
    if (range > p.rescale_spread) {
      const float my = mean_k(y);
      const float f = p.rescale_spread / (range + 1e-6f);
#pragma unroll
      for (int i = 0; i < kMaxHeads; ++i)
        if (i < K) y[i] = __fadd_rn(__fmul_rn(y[i] - my, f), my);
    }
  }
  const float g2 = p.loss_scale > 0.f ? __fmul_rn(2.f, p.loss_scale) : 2.f;
#pragma unroll
  for (int i = 0; i < kMaxHeads; ++i) {
    if (i < K) {
      const float d = q[i] - y[i];
      const float g = __fmul_rn(g2 * d, invB);
      p.y[(long)r * K + i] = y[i];
      p.sqe[(long)r * K + i] = d * d;
      p.dq[(long)r * K + qi[i]] = g;
      if (p.dh2) sdq[threadIdx.x][qi[i]] = g;
    }
  }
}

// threads of the prefetching dh2 pass: rows_per_pass(n4) rows of n4 float4s
// per 256 threads (n4 <= 64), four passes over a 16-row block
__device__ __forceinline__ int rows_per_pass(int n4) { return 256 / n4; }

// the targets kernel's row logic, then (p.dh2) the 16 rows' backward into
// the last hidden layer by the whole block
__global__ void __launch_bounds__(256) particle_targets_kernel(ParticleTargetArgs p) {
  __shared__ RowHeadLds hs, qs;
  __shared__ float sdq[kRowBlock][kMaxHeads];
  const int r0 = blockIdx.x * kRowBlock;
  const int K = p.K, H = p.qh.H, n4 = H >> 2;
  // the backward's operands need nothing the row logic computes: with H <= 256
  // a thread's 4 elements share one float4 column c of the K weight rows, so
  // those and the 4 hidden-row float4s are requested before the heads (the
  // dh2 pass then starts on registers, not on a round trip after the rows)
  const bool pre = p.dh2 && n4 <= 64 && n4 * kRowBlock <= 1024 && K <= kMaxHeads;
  float4 hpf[4], wpf[kMaxHeads];
  if (pre) {
    const int c = 4 * (threadIdx.x % n4), rr0 = threadIdx.x / n4, rstep = 256 / n4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = min(r0 + rr0 + j * rstep, p.B - 1);
      hpf[j] = *reinterpret_cast<const float4*>(p.qh.h + (long)m * H + c);
    }
#pragma unroll
    for (int k = 0; k < kMaxHeads; ++k)
      wpf[k] = *reinterpret_cast<const float4*>(p.qh.w + (long)min(k, K - 1) * H + c);
  }
  particle_targets_rows(p, hs, qs, sdq);
  if (!p.dh2) return;
  __syncthreads();
  if (pre && threadIdx.x < rows_per_pass(n4) * n4) {
    const int c = 4 * (threadIdx.x % n4), rr0 = threadIdx.x / n4, rstep = 256 / n4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rr = min(rr0 + j * rstep, kRowBlock - 1), m = r0 + rr;
      if (rr0 + j * rstep >= kRowBlock || m >= p.B) continue;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < kMaxHeads; ++k) {   // k order, as the GEMM's accumulation
        const float g = k < K ? sdq[rr][k] : 0.f;   // (+0 past K: the sum is unchanged)
        a.x = fmaf(g, wpf[k].x, a.x); a.y = fmaf(g, wpf[k].y, a.y);
        a.z = fmaf(g, wpf[k].z, a.z); a.w = fmaf(g, wpf[k].w, a.w);
      }
      const float4 h = hpf[j];
      float4 o;
      o.x = h.x > 0.f ? a.x : 0.f; o.y = h.y > 0.f ? a.y : 0.f;
      o.z = h.z > 0.f ? a.z : 0.f; o.w = h.w > 0.f ? a.w : 0.f;
      *reinterpret_cast<float4*>(p.dh2 + (long)m * H + c) = o;
    }
    return;
  }
  if (pre) return;
  for (int e = threadIdx.x; e < kRowBlock * n4; e += 256) {
    const int rr = e / n4, c = 4 * (e - rr * n4), m = r0 + rr;
    if (m >= p.B) continue;
    const float4 h = *reinterpret_cast<const float4*>(p.qh.h + (long)m * H + c);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < K; ++k) {   // k order, as the GEMM's accumulation
      const float4 w = *reinterpret_cast<const float4*>(p.qh.w + (long)k * H + c);
      const float g = sdq[rr][k];
      a.x = fmaf(g, w.x, a.x); a.y = fmaf(g, w.y, a.y);
      a.z = fmaf(g, w.z, a.z); a.w = fmaf(g, w.w, a.w);
    }
    float4 o;
    o.x = h.x > 0.f ? a.x : 0.f; o.y = h.y > 0.f ? a.y : 0.f;
    o.z = h.z > 0.f ? a.z : 0.f; o.w = h.w > 0.f ? a.w : 0.f;
    *reinterpret_cast<float4*>(p.dh2 + (long)m * H + c) = o;
  }
}

// sorted_qs[0] of Q(obs, a~) with the post-step critic (particle_trainer_oac.py:286-295)
// -> gradient seed -1/B on the argmin head; plus the alpha update (274-281)
// on a block of its own after the row blocks (committed by the policy Adam,
// which reads no alpha field).
__global__ void __launch_bounds__(256) particle_min_kernel(ParticleMinArgs p) {
  __shared__ float red[256];
  const int nrb = (p.B + kRowBlock - 1) / kRowBlock;
  if ((int)blockIdx.x == nrb) {   // the alpha update: its own block, beside the row blocks
    if (!p.alpha) return;
    const float S = (p.world_size > 1) ? (p.logp_part ? block_part_sum(p.logp_part, p.n_logp_part, red)
                                                      : p.alpha->sum)
                                       : block_logp_sum(p.logp, p.B, p.target_entropy, red);
    if (threadIdx.x == 0) {
      AlphaState* as = p.alpha;
      const float n = (float)((long long)p.B * (p.world_size > 1 ? p.world_size : 1));
      const float la_old = as->log_alpha;
      const float g = -(S / n);
      double bc1, sbc2;
      bias_corrections(p.state, p.state->n_steps + 1, p.beta1, p.beta2, bc1, sbc2);
      const float m = __fadd_rn(__fmul_rn(as->m, (float)p.beta1), __fmul_rn((float)(1.0 - p.beta1), g));
      const float v = __fadd_rn(__fmul_rn(as->v, (float)p.beta2),
                                __fmul_rn(__fmul_rn((float)(1.0 - p.beta2), g), g));
      const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), (float)sbc2), (float)p.adam_eps);
      const float la = __fadd_rn(la_old, __fdiv_rn(__fmul_rn(-(float)(p.lr / bc1), m), denom));
      as->next_log_alpha = la; as->next_m = m; as->next_v = v;
      as->alpha = expf(la); as->grad = g; as->alpha_loss = -(la_old * S) / n;
    }
    return;
  }
  __shared__ RowHeadLds hs;
  const int r0 = blockIdx.x * kRowBlock, r = r0 + threadIdx.x;
  const int K = p.K;
  const int H = p.hn.H, n4 = H >> 2;
  // the backward's operands (the 4 hidden-row float4s of this thread and the
  // K weight rows' float4 of its column) requested before the heads, as in
  // particle_targets_kernel
  const bool pre = p.dh2 && n4 <= 64;
  float4 hpf[4], wpf[kMaxHeads];
  if (pre) {
    const int c = 4 * (threadIdx.x % n4), rr0 = threadIdx.x / n4, rstep = 256 / n4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = min(r0 + rr0 + j * rstep, p.B - 1);
      hpf[j] = *reinterpret_cast<const float4*>(p.hn.h + (long)m * H + c);
    }
#pragma unroll
    for (int k = 0; k < kMaxHeads; ++k)
      wpf[k] = *reinterpret_cast<const float4*>(p.hn.w + (long)min(k, K - 1) * H + c);
  }
  if (p.hn.h) {
    row_heads(p.hn, K, p.B, r0, hs);
    __syncthreads();
  }
  __shared__ int sbest[kRowBlock];
  const float invB = 1.f / (float)p.B;
  if (threadIdx.x < kRowBlock && r < p.B) {
    const float* qn = p.hn.h ? &hs.out[threadIdx.x][0] : p.qn + (long)r * K;
    int best = 0;
    float bv = qn[0];
    for (int i = 1; i < K; ++i) {
      const float x = qn[i];
      if (x < bv || (bv != bv && x == x)) { bv = x; best = i; }   // (NaN last, as torch.sort)
    }
    for (int i = 0; i < K; ++i) p.gq[(long)r * K + i] = (i == best) ? -invB : 0.f;
    p.qmin[r] = bv;
    sbest[threadIdx.x] = best;
  }
  if (!p.dh2) return;
  // -min Q backward into the last hidden layer (the dX launch it replaces
  // summed gq[r, k] W[k, n] over k: one nonzero product, the rest +0)
  __syncthreads();
  if (pre) {
    if (threadIdx.x >= rows_per_pass(n4) * n4) return;
    const int c = 4 * (threadIdx.x % n4), rr0 = threadIdx.x / n4, rstep = 256 / n4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rr = min(rr0 + j * rstep, kRowBlock - 1), m = r0 + rr;
      if (rr0 + j * rstep >= kRowBlock || m >= p.B) continue;
      const int b = sbest[rr];
      // the argmin head's row as a masked sum (exact: one term is w, the rest
      // +-0), so the prefetched rows stay in registers.  Not exact if another
      // head's weight is +-inf (0 * inf): a critic that far diverged has
      // inf / NaN Q values in the reference too.  Exact forms measured slower
      // (round 5, configs[4], this launch 6.2 us): a select chain 7.9, the
      // rows staged through LDS 9.3.
      float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < kMaxHeads; ++k) {
        const float sel = b == k ? 1.f : 0.f;
        w.x = fmaf(sel, wpf[k].x, w.x); w.y = fmaf(sel, wpf[k].y, w.y);
        w.z = fmaf(sel, wpf[k].z, w.z); w.w = fmaf(sel, wpf[k].w, w.w);
      }
      const float4 h = hpf[j];
      float4 o;
      o.x = h.x > 0.f ? -invB * w.x : 0.f; o.y = h.y > 0.f ? -invB * w.y : 0.f;
      o.z = h.z > 0.f ? -invB * w.z : 0.f; o.w = h.w > 0.f ? -invB * w.w : 0.f;
      *reinterpret_cast<float4*>(p.dh2 + (long)m * H + c) = o;
    }
    return;
  }
  for (int e = threadIdx.x; e < kRowBlock * n4; e += 256) {
    const int rr = e / n4, c = 4 * (e - rr * n4), m = r0 + rr;
    if (m >= p.B) continue;
    const float4 h = *reinterpret_cast<const float4*>(p.hn.h + (long)m * H + c);
    const float4 w = *reinterpret_cast<const float4*>(p.hn.w + (long)sbest[rr] * H + c);
    float4 o;
    o.x = h.x > 0.f ? -invB * w.x : 0.f; o.y = h.y > 0.f ? -invB * w.y : 0.f;
    o.z = h.z > 0.f ? -invB * w.z : 0.f; o.w = h.w > 0.f ? -invB * w.w : 0.f;
    *reinterpret_cast<float4*>(p.dh2 + (long)m * H + c) = o;
  }
}

hipError_t launch_particle_targets(const ParticleTargetArgs& a, hipStream_t s) {
  if (a.K > kMaxHeads || !head_ok(a.th) || !head_ok(a.qh)) return hipErrorInvalidValue;
  if (a.dh2 && (!a.qh.h || (a.qh.H & 3))) return hipErrorInvalidValue;
  OAC_LAUNCH(particle_targets_kernel, dim3((a.B + kRowBlock - 1) / kRowBlock), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_particle_min(const ParticleMinArgs& a, hipStream_t s) {
  if (a.dh2 && (!a.hn.h || (a.hn.H & 3))) return hipErrorInvalidValue;
  if (a.K > kMaxHeads || !head_ok(a.hn)) return hipErrorInvalidValue;
  // the row blocks, then one block for the alpha update
  OAC_LAUNCH(particle_min_kernel, dim3((a.B + kRowBlock - 1) / kRowBlock + 1), dim3(256), 0, s, a);
  return hipGetLastError();
}

// --------------------------------------------------------------------------
// g-oac GaussianTrainer, share_layers=True (trainer/gaussian_trainer.py).
// The critic's raw outputs are [mean | log std]; std = exp(log std) is the
// FlattenMlp positive=[False, True] output (networks.py:69-75).
// --------------------------------------------------------------------------

// TD targets and the critic gradient (gaussian_trainer.py:199-242 with the
// share_layers branch 205-237):
//   std_target = (1-d)*gamma*exp(tq1)   [soft update: p*next + (1-p)*std]
//   counts=True: std_target <- std where count != 0 (factor, 238-242 / 219-223)
//   q_target   = scale*r + (1-d)*gamma*tq0 ; std_target = clamp(., 0, std_init)
//   loss = MSE(q0, q_target) + MSE(std, std_target)
//   dL/dq0 = 2 (q0 - y_q) / B ;  dL/dq1 = 2 (std - y_s) / B * std  (exp backward)
__global__ void __launch_bounds__(256) gauss_targets_kernel(GaussTargetArgs p) {
  __shared__ RowHeadLds hs;
  const int r0 = blockIdx.x * kRowBlock, r = r0 + threadIdx.x;
  if (p.th.h) {
    row_heads(p.th, 2, p.B, r0, hs);
    __syncthreads();
  }
  if (threadIdx.x >= kRowBlock || r >= p.B) return;
  const float* tq = p.th.h ? &hs.out[threadIdx.x][0] : p.tq + 2L * r;
  const float q0 = p.q[2L * r], sd = expf(p.q[2L * r + 1]);
  const float t0 = tq[0], tsd = expf(tq[1]);
  const float rew = p.batch[(long)r * p.ld_batch + p.off_rew];
  const float term = p.batch[(long)r * p.ld_batch + p.off_term];
  const float gd = __fmul_rn(1.f - term, p.discount);
  float ys = __fmul_rn(gd, tsd);
  if (p.soft_prob >= 0.f)
    ys = __fadd_rn(__fmul_rn(p.soft_prob, ys), __fmul_rn(1.f - p.soft_prob, sd));
  if (p.counts && p.counts[r] != 0.f) ys = sd;
  ys = fminf(fmaxf(ys, 0.f), p.std_init);
  const float yq = __fadd_rn(__fmul_rn(p.reward_scale, rew), __fmul_rn(gd, t0));
  const float invB = 1.f / (float)p.B;
  const float d0 = q0 - yq, d1 = sd - ys;
  p.dq[2L * r] = __fmul_rn(2.f * d0, invB);
  p.dq[2L * r + 1] = __fmul_rn(__fmul_rn(2.f * d1, invB), sd);
  p.y[2L * r] = yq;
  p.y[2L * r + 1] = ys;
  p.sqe[2L * r] = d0 * d0;
  p.sqe[2L * r + 1] = d1 * d1;
}

// Policy-loss seeds through the post-step critic (gaussian_trainer.py:323-336,
// 338-350): policy: L = -mean(q0 + z*exp(q1)) -> [-1/B, -z/B * std];
// target policy: L = -mean(q0) -> [-1/B, 0]
__global__ void __launch_bounds__(256) gauss_seed_kernel(GaussSeedArgs p) {
  __shared__ RowHeadLds hs;
  const int r0 = blockIdx.x * kRowBlock, r = r0 + threadIdx.x;
  if (p.hn.h) {   // (the target policy's seed is constant: qt is never read)
    row_heads(p.hn, 2, p.B, r0, hs);
    __syncthreads();
  }
  if (threadIdx.x >= kRowBlock || r >= p.B) return;
  const float* qn = p.hn.h ? &hs.out[threadIdx.x][0] : p.qn + 2L * r;
  const float g0 = -(1.f / (float)p.B);
  const float sd = expf(qn[1]);
  p.ub[r] = __fadd_rn(qn[0], __fmul_rn(p.std_bound, sd));
  p.g[2L * r] = g0;
  p.g[2L * r + 1] = __fmul_rn(__fmul_rn(g0, p.std_bound), sd);
  p.gt[2L * r] = g0;
  p.gt[2L * r + 1] = 0.f;
}

// particle_trainer.py policy losses through the post-step critic: the
// policy maximises the delta_index-th sorted particle (:317-330; gradient to
// the head sort placed there), the target policy the particle mean (:339-348)
__global__ void __launch_bounds__(256) particle_ub_seed_kernel(ParticleUbSeedArgs p) {
  __shared__ RowHeadLds hs;
  const int r0 = blockIdx.x * kRowBlock, r = r0 + threadIdx.x;
  const int K = p.K;
  if (p.hn.h) {   // (the target policy's seed is constant: qt is never read)
    row_heads(p.hn, K, p.B, r0, hs);
    __syncthreads();
  }
  if (threadIdx.x >= kRowBlock || r >= p.B) return;
  float v[kMaxHeads];
  int ix[kMaxHeads];
  load_row16(p.hn.h ? &hs.out[threadIdx.x][0] : p.qn + (long)r * K, K, v, ix);
  sort16(v, ix);
  const float g0 = -(1.f / (float)p.B);
  int sel = ix[0];
  float ub = v[0];
#pragma unroll
  for (int i = 1; i < kMaxHeads; ++i)
    if (i == p.delta_index) { sel = ix[i]; ub = v[i]; }
#pragma unroll
  for (int i = 0; i < kMaxHeads; ++i) {
    if (i < K) {
      p.g[(long)r * K + i] = (i == sel) ? g0 : 0.f;
      p.gt[(long)r * K + i] = g0 / (float)K;
    }
  }
  p.ub[r] = ub;
}

__global__ void __launch_bounds__(256) det_head_backward_kernel(DetHeadBwdArgs p) {
  const int Da = p.act_dim;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= p.B * Da) return;
  const int r = idx / Da, j = idx % Da;
  const int g = blockIdx.y;
  const float a = p.act[g][idx];
  float* dh = p.dhead[g] + (long)r * 2 * Da;
  dh[j] = __fmul_rn(p.da[g][idx], __fsub_rn(1.f, __fmul_rn(a, a)));
  dh[Da + j] = 0.f;
}

hipError_t launch_gauss_targets(const GaussTargetArgs& a, hipStream_t s) {
  if (!head_ok(a.th)) return hipErrorInvalidValue;
  OAC_LAUNCH(gauss_targets_kernel, dim3((a.B + kRowBlock - 1) / kRowBlock), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_gauss_seed(const GaussSeedArgs& a, hipStream_t s) {
  if (!head_ok(a.hn)) return hipErrorInvalidValue;
  OAC_LAUNCH(gauss_seed_kernel, dim3((a.B + kRowBlock - 1) / kRowBlock), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_particle_ub_seed(const ParticleUbSeedArgs& a, hipStream_t s) {
  if (a.K > kMaxHeads || !head_ok(a.hn)) return hipErrorInvalidValue;
  OAC_LAUNCH(particle_ub_seed_kernel, dim3((a.B + kRowBlock - 1) / kRowBlock), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_det_head_backward(const DetHeadBwdArgs& a, hipStream_t s) {
  OAC_LAUNCH(det_head_backward_kernel, dim3((a.B * a.act_dim + 255) / 256, a.nseg), dim3(256), 0,
             s, a);
  return hipGetLastError();
}

}  // namespace oac
