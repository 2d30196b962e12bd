// Policy head + tanh-Gaussian sample + the critics' action columns, one launch.
//
// For a 32-row block of one policy batch (obs or next_obs) a workgroup
//   1. computes the stacked heads  [mean | ls_raw] = h2 . W_head^T + b
//      (TanhGaussianPolicy.forward, /root/reference/trainer/policies.py:275-283;
//      K = hidden split over the 8 waves, fixed-order LDS reduction),
//   2. samples a = tanh(mean + std*eps) and its log-prob (policies.py:175-192,
//      147-160) exactly as policy_sample_kernel (rows.hip) does,
//   3. finishes layer 0 of the critics that consume this action:
//      h1 = relu(P + a . W0[:, Do:]^T) with P = obs . W0[:, :Do]^T + b0 saved
//      by the layer-0 launch (FlattenMlp on cat([obs, a]), networks.py:159-161)
//      -- for Q1/Q2(obs, a~) on the obs batch and TQ1/TQ2(next_obs, a') on the
//      next_obs batch (trainer.py:151-153, 172-177).
// Step 3 only needs this block's own 32 actions, so the three stages that were
// separate launches (head GEMM, sample, K = act_dim GEMM) have no inter-
// workgroup seam.  The hidden columns of step 3 are split over `col_chunks`
// workgroups per row block; each recomputes steps 1-2 (cheap) and chunk 0
// writes the per-row outputs.
#include "oac_common.h"
#include "kernels.h"

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

constexpr int kHeadWaves = 8;

#ifdef OAC_STAGE_CLOCK   // per-stage wall clock of thread 0 (tools/micro harness)
#define STAGE(i) \
  if (threadIdx.x == 0) a.stage_clock[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = wall_clock64()
#else
#define STAGE(i)
#endif

__global__ void __launch_bounds__(64 * kHeadWaves) policy_head_kernel(const HeadArgs a) {
  // one LDS array (reduction scratch, then the head tile and the actions)
  constexpr int kRed = kHeadWaves * 2 * 16 * 64;
  __shared__ __attribute__((aligned(16))) float lds[kRed];
  const HeadSeg& sg = a.seg[blockIdx.y];
  const int rb = blockIdx.x / a.col_chunks;
  const int chunk = blockIdx.x % a.col_chunks;
  const int m0 = rb * 32;
  const int B = a.B, H = a.H, Da = a.Da, D2 = 2 * Da;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l32 = lane & 31, half = lane >> 5;
  STAGE(0);

  // ---- 0. prefetch what steps 2-3 read from memory (their latency then
  //         overlaps the head GEMM): eps of this thread's rows, the critic
  //         weights and saved projections of this wave's first (net, tile).
  const int cols = (H + a.col_chunks - 1) / a.col_chunks;
  const int n_lo = chunk * cols;
  const int tiles = (cols + 31) / 32;
  const int pairs = sg.n_nets * tiles;
  const int kgroups = (Da + 7) >> 3;          // <= 4 (Da <= 32)
  float eps_pf[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (threadIdx.x >> 5) + i * 2 * kHeadWaves;
    const int m = min(m0 + row, B - 1), j = min((int)(threadIdx.x & 31), Da - 1);
    eps_pf[i] = sg.eps[(long)m * Da + j];
  }
  // head bias of the two columns this thread reduces (tile 0 / tile 1, lane & 31)
  const float bh_pf0 = a.bh[min(l32, D2 - 1)];
  const float bh_pf1 = a.bh[min(32 + l32, D2 - 1)];
  float bw_pf[4][4], pre_pf[16];
  if (wave < pairs) {
    const int net = wave / tiles;
    const int n = n_lo + (wave % tiles) * 32 + l32;
    const bool nv = n < H && n < n_lo + cols;
    const float* wrow = sg.wa[net] + (long)(nv ? n : 0) * a.ld_wa;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        bw_pf[g][c] = wrow[min(8 * g + 4 * half + c, Da - 1)];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = min(m0 + (r & 3) + 8 * (r >> 2) + 4 * half, B - 1);
      pre_pf[r] = sg.pre[net][(long)m * H + (nv ? n : 0)];
    }
  }

  // ---- 1. heads: acc0 = columns 0..31, acc1 = columns 32..63 (2*Da <= 64)
  floatx16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }
  {
    const int m = min(m0 + l32, B - 1);
    const float* arow = sg.h2 + (long)m * H;
    const bool v0 = l32 < D2, v1 = 32 + l32 < D2;
    const float* b0 = a.wh + (long)(v0 ? l32 : 0) * H;
    const float* b1 = a.wh + (long)(v1 ? 32 + l32 : 0) * H;
    const int groups = (H + 7) >> 3;
    constexpr int kG = 4;
#pragma unroll 1
    for (int g0 = wave; g0 < groups; g0 += kG * kHeadWaves) {
      f4u xa[kG], x0[kG], x1[kG];
#pragma unroll
      for (int j = 0; j < kG; ++j)
        if (g0 + j * kHeadWaves < groups) {
          const int kb = 8 * (g0 + j * kHeadWaves) + 4 * half;
          xa[j] = *reinterpret_cast<const f4u*>(arow + kb);
          x0[j] = *reinterpret_cast<const f4u*>(b0 + kb);
          x1[j] = *reinterpret_cast<const f4u*>(b1 + kb);
        }
#pragma unroll
      for (int j = 0; j < kG; ++j)
        if (g0 + j * kHeadWaves < groups) {
          const int kb = 8 * (g0 + j * kHeadWaves) + 4 * half;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const bool kin = kb + c < H;
            const float av = kin ? xa[j][c] : 0.f;
            const float bv0 = (kin && v0) ? x0[j][c] : 0.f;
            const float bv1 = (kin && v1) ? x1[j][c] : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv1, acc1, 0, 0, 0);
          }
        }
    }
  }
  STAGE(1);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    lds[((wave * 2 + 0) * 16 + r) * 64 + lane] = acc0[r];
    lds[((wave * 2 + 1) * 16 + r) * 64 + lane] = acc1[r];
  }
  __syncthreads();
  // fixed-order wave sum; element (tile, reg r, lane l) -> head[row][col]
  float hv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = threadIdx.x + i * 64 * kHeadWaves;   // 0 .. 2047
    const int tile = e >> 10, r = (e >> 6) & 15, l = e & 63;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kHeadWaves; ++w) s += lds[((w * 2 + tile) * 16 + r) * 64 + l];
    hv[i] = s;
  }
  __syncthreads();
  // head tile in LDS: hs[row * 65 + col], cols 0..2*Da-1 ; actions: as[row * 33 + j]
  float* hs = lds;
  float* as = lds + 32 * 65;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = threadIdx.x + i * 64 * kHeadWaves;
    const int tile = e >> 10, r = (e >> 6) & 15, l = e & 63;
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    const int col = tile * 32 + (l & 31);
    if (col < D2) {
      const float h = hv[i] + (tile ? bh_pf1 : bh_pf0);
      hs[row * 65 + col] = h;
      if (chunk == 0 && m0 + row < B) sg.head[(long)(m0 + row) * D2 + col] = h;
    }
  }
  __syncthreads();
  STAGE(2);

  // ---- 2. sample + log-prob: one half-wave per row, lane j = action dim
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int row = (threadIdx.x >> 5) + it * 2 * kHeadWaves;
    const int j = threadIdx.x & 31;
    const int m = m0 + row;
    float l = 0.f, act = 0.f;
    if (m < B && j < Da) {
      const long e = (long)m * Da + j;
      const float mean = hs[row * 65 + j];
      const float ls = fminf(fmaxf(hs[row * 65 + Da + j], -20.f), 2.f);
      const float sd = expf(ls);
      const float z = __fadd_rn(mean, __fmul_rn(sd, eps_pf[it]));
      act = tanhf(z);
      const float u = z - mean;
      const float var = __fmul_rn(sd, sd);
      const float t1 = -(__fmul_rn(u, u)) / (2.f * var);
      l = t1 - logf(sd) - 0.918938533204672742f  // log(sqrt(2*pi))
          - logf(__fadd_rn(1.f - __fmul_rn(act, act), 1e-6f));
      if (chunk == 0) { sg.act[e] = act; sg.stdv[e] = sd; sg.u[e] = u; }
    }
    as[row * 33 + j] = act;   // 0 beyond Da / B
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) l += __shfl_xor(l, o, 32);
    if (j == 0 && m < B && chunk == 0) sg.logp[m] = l;
  }
  __syncthreads();
  STAGE(3);

  // ---- 3. critics' action columns: h1[m, n] = relu(P[m, n] + sum_j a[m, j] W[n, j])
#pragma unroll 1
  for (int pi = wave; pi < pairs; pi += kHeadWaves) {
    const int net = pi / tiles;
    const int n = n_lo + (pi % tiles) * 32 + l32;
    const bool nv = n < H && n < n_lo + cols;
    if (pi != wave) {   // later pairs (only when pairs > waves): load now
      const float* wrow = sg.wa[net] + (long)(nv ? n : 0) * a.ld_wa;
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          bw_pf[g][c] = wrow[min(8 * g + 4 * half + c, Da - 1)];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = min(m0 + (r & 3) + 8 * (r >> 2) + 4 * half, B - 1);
        pre_pf[r] = sg.pre[net][(long)m * H + (nv ? n : 0)];
      }
    }
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (g < kgroups) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int k = 8 * g + 4 * half + c;
          const float av = k < Da ? as[l32 * 33 + k] : 0.f;
          const float bv = (nv && k < Da) ? bw_pf[g][c] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * half;
      if (m < B && nv) sg.h1[net][(long)m * H + n] = fmaxf(acc[r] + pre_pf[r], 0.f);
    }
  }
  STAGE(4);
}

hipError_t launch_policy_head(const HeadArgs& a, int nseg, hipStream_t s) {
  if (a.Da < 1 || 2 * a.Da > 64 || a.col_chunks < 1 || nseg < 1 || nseg > 2)
    return hipErrorInvalidValue;
  for (int i = 0; i < nseg; ++i)
    if (a.seg[i].n_nets < 0 || a.seg[i].n_nets > 2) return hipErrorInvalidValue;
  const int rblocks = (a.B + 31) / 32;
  hipLaunchKernelGGL(policy_head_kernel, dim3(rblocks * a.col_chunks, nseg), dim3(64 * kHeadWaves),
                     0, s, a);
  return hipGetLastError();
}

}  // namespace oac
