// Policy head + tanh-Gaussian sample + the critics' action columns, one launch.
//
// For a 16-row block of one policy batch (obs or next_obs) a workgroup
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
#include "policy_math.h"
#include <algorithm>

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

constexpr int kHeadWaves = 8;

#ifdef OAC_STAGE_CLOCK   // per-stage wall clock of thread 0 (tools/micro harness)
#define STAGE(i) \
  if (threadIdx.x == 0) a.stage_clock[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = wall_clock64()
// drain this wave's outstanding loads first (micro builds only: shows load latency)
#define STAGE_DRAIN(i) do { __builtin_amdgcn_s_waitcnt(0); STAGE(i); } while (0)
#else
#define STAGE(i)
#define STAGE_DRAIN(i)
#endif

// 16 rows per workgroup, v_mfma_f32_16x16x4_f32 (lane l: A[l&15][k=l>>4],
// B[k=l>>4][l&15]; D reg r: row 4*(l>>4)+r, col l&15).  A k-chunk of 16 is one
// 16-byte load per lane and operand: lane group g holds k = 16c + 4g .. +3 and
// MFMA j of the chunk multiplies element j, so the four MFMAs cover the chunk.
constexpr int kRows = 16;

// NT = column tiles of the stacked head (2*act_dim <= 16*NT), a compile-time
// count so the MFMA sequence is branch-free; KP = (net, 16-column tile) pairs
// per wave of step 3 (2: <= 16 pairs per workgroup; 4: a whole 256-column
// hidden layer of both nets in one workgroup, the large-batch form, no
// recomputed heads); KS = k-steps of 4 action dims held per pair (Da <= 4*KS)
template <int NT, int KP, int KS>
__global__ void __launch_bounds__(64 * kHeadWaves) policy_head_kernel(const HeadArgs a) {
  // one LDS array: reduction scratch, then the head tile and the actions
  constexpr int kRed = kHeadWaves * 4 * 4 * 64;   // waves x col tiles x regs x lanes
  __shared__ __attribute__((aligned(16))) float lds[kRed];
  __shared__ float s_lp[kRows];   // per-row logp + te (HeadArgs::logp_part)
  const HeadSeg& sg = a.seg[blockIdx.y];
  const float* wh = sg.wh ? sg.wh : a.wh;
  const float* bh = sg.bh ? sg.bh : a.bh;
  const int rb = blockIdx.x / a.col_chunks;
  const int chunk = blockIdx.x % a.col_chunks;
  const int m0 = rb * kRows;
  const int B = a.B, H = a.H, Da = a.Da, D2 = 2 * Da;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g4 = lane >> 4;
  STAGE(0);

  // ---- 1a. head GEMM operands of the first k-chunks, issued FIRST: vmcnt
  // retires loads in issue order, so with the step-3 prefetch below issued
  // ahead of them the head MFMAs waited for the whole 32-KB prefetch too
  typedef float floatx4 __attribute__((ext_vector_type(4)));
  floatx4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  constexpr int ntile = NT;
  const float* arow = sg.h2 + (long)min(m0 + l16, B - 1) * H;
  const float* brow[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) brow[t] = wh + (long)min(t * 16 + l16, D2 - 1) * H;
  const int chunks = (H + 15) >> 4;
  constexpr int kC = 2;                         // k-chunks in flight per wave
  f4u xa[kC], xb[kC][4];
  // branch-free (clamped k): a branch between these loads and their MFMAs
  // makes the waitcnt pass assume the fewest loads in flight of any path
  auto head_loads = [&](int c0) {
#pragma unroll
    for (int j = 0; j < kC; ++j) {
      const int kb = min(16 * (c0 + j * kHeadWaves) + 4 * g4, H - 4);
      xa[j] = *reinterpret_cast<const f4u*>(arow + kb);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < ntile) xb[j][t] = *reinterpret_cast<const f4u*>(brow[t] + kb);
    }
  };
  auto head_mfma = [&](int c0) {
#pragma unroll
    for (int j = 0; j < kC; ++j)
      if (c0 + j * kHeadWaves < chunks) {
        const int kb = 16 * (c0 + j * kHeadWaves) + 4 * g4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const bool kin = kb + c < H;
          const float av = kin ? xa[j][c] : 0.f;
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (t < ntile) {
              const float bv = (kin && t * 16 + l16 < D2) ? xb[j][t][c] : 0.f;
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t], 0, 0, 0);
            }
        }
      }
  };
  head_loads(wave);   // chunk past the end: clamped, its MFMAs skipped

  // ---- 0. prefetch what steps 2-3 read besides the head GEMM operands
  const int cols = (H + a.col_chunks - 1) / a.col_chunks;
  const int n_lo = chunk * cols;
  const int tiles = (cols + 15) / 16;
  const int pairs = sg.n_nets * tiles;
  const int ksteps = (Da + 3) >> 2;              // <= KS
  const int srow = threadIdx.x >> 5, sj = threadIdx.x & 31;   // step 2: row, action dim
  const float eps_pf = a.det ? 0.f : sg.eps[(long)min(m0 + srow, B - 1) * Da + min(sj, Da - 1)];
  float bh_pf[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + i * 64 * kHeadWaves;          // head element (see step 1)
    bh_pf[i] = bh[min(((e >> 8) << 4) + (e & 15), D2 - 1)];
  }
  constexpr int kPairs = KP;                     // pairs per wave prefetched
  float bw_pf[kPairs][KS], pre_pf[kPairs][4];
#pragma unroll
  for (int q = 0; q < kPairs; ++q) {   // branch-free: a pair past the end reads wh[0]
    const int pi = wave + q * kHeadWaves;
    const bool pv = pi < pairs;
    const int net = pv ? pi / tiles : 0;
    const int n = n_lo + (pi % tiles) * 16 + l16;
    const bool nv = pv && n < H && n < n_lo + cols;
    const float* wrow = pv ? sg.wa[net] + (long)(nv ? n : 0) * a.ld_wa : wh;
    const float* prow = pv ? sg.pre[net] + (nv ? n : 0) : wh;
    const long pld = pv ? (long)H : 0;
#pragma unroll
    for (int st = 0; st < KS; ++st) bw_pf[q][st] = wrow[pv ? min(4 * st + g4, Da - 1) : 0];
#pragma unroll
    for (int r = 0; r < 4; ++r) pre_pf[q][r] = prow[(long)min(m0 + 4 * g4 + r, B - 1) * pld];
  }

  STAGE_DRAIN(5);
  // ---- 1b. heads [mean | ls_raw] for 16 rows: up to 4 column tiles of 16
  STAGE_DRAIN(6);
  head_mfma(wave);
#pragma unroll 1
  for (int c0 = wave + kC * kHeadWaves; c0 < chunks; c0 += kC * kHeadWaves) {
    head_loads(c0);
    head_mfma(c0);
  }
  STAGE(1);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) lds[((wave * 4 + t) * 4 + r) * 64 + lane] = acc[t][r];
  __syncthreads();
  // fixed-order wave sum; element e = (tile, reg r, lane l) -> head[4*(l>>4)+r][16*tile + (l&15)]
  float hv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + i * 64 * kHeadWaves;   // 0 .. 1023
    const int tile = e >> 8, r = (e >> 6) & 3, l = e & 63;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kHeadWaves; ++w) s += lds[((w * 4 + tile) * 4 + r) * 64 + l];
    hv[i] = s;
  }
  __syncthreads();
  float* hs = lds;               // [16][65]
  float* as = lds + kRows * 65;  // [16][33]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + i * 64 * kHeadWaves;
    const int tile = e >> 8, r = (e >> 6) & 3, l = e & 63;
    const int row = 4 * (l >> 4) + r, col = tile * 16 + (l & 15);
    if (col < D2) {
      const float h = hv[i] + bh_pf[i];
      hs[row * 65 + col] = h;
      if (chunk == 0 && m0 + row < B) sg.head[(long)(m0 + row) * D2 + col] = h;
    }
  }
  __syncthreads();
  STAGE(2);

  // ---- 2. sample + log-prob: one half-wave per row, lane j = action dim
  {
    const int row = srow, j = sj, m = m0 + row;
    float l = 0.f, act = 0.f;
    if (m < B && j < Da) {
      const long e = (long)m * Da + j;
      float sd, u;
      if (a.det) {
        act = tanhf(hs[row * 65 + j]);
        if (chunk == 0) sg.act[e] = act;
      } else {
        l = tanh_gauss_sample(hs[row * 65 + j], hs[row * 65 + Da + j], eps_pf, act, sd, u);
        if (chunk == 0) { sg.act[e] = act; sg.stdv[e] = sd; sg.u[e] = u; }
      }
    }
    as[row * 33 + j] = act;   // 0 beyond Da / B
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) l += __shfl_xor(l, o, 32);
    if (j == 0 && m < B && chunk == 0 && !a.det) sg.logp[m] = l;
    if (j == 0) s_lp[row] = m < B ? l + a.target_entropy : 0.f;
  }
  __syncthreads();
  // data-parallel alpha: this row block's sum of (logp + te), rows in order
  if (a.logp_part && blockIdx.y == 0 && chunk == 0 && !a.det && threadIdx.x == 0) {
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < kRows; ++r) sum += s_lp[r];
    a.logp_part[rb] = sum;
  }
  STAGE(3);

  // ---- 3. critics' action columns: h1[m, n] = relu(P[m, n] + sum_j a[m, j] W[n, j])
#pragma unroll
  for (int q = 0; q < kPairs; ++q) {
    const int pi = wave + q * kHeadWaves;
    if (pi >= pairs) break;
    const int net = pi / tiles;
    const int n = n_lo + (pi % tiles) * 16 + l16;
    const bool nv = n < H && n < n_lo + cols;
    floatx4 c = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < KS; ++st)
      if (st < ksteps) {
        const int k = 4 * st + g4;
        const float av = k < Da ? as[l16 * 33 + k] : 0.f;
        const float bv = (nv && k < Da) ? bw_pf[q][st] : 0.f;
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, c, 0, 0, 0);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 4 * g4 + r;
      if (m < B && nv) sg.h1[net][(long)m * H + n] = fmaxf(c[r] + pre_pf[q][r], 0.f);
    }
  }
  STAGE(4);
}

template <int KP, int KS>
static void launch_head_nt(const HeadArgs& a, dim3 grid, dim3 block, hipStream_t s) {
  switch ((2 * a.Da + 15) / 16) {
    case 1: OAC_LAUNCH((policy_head_kernel<1, KP, KS>), grid, block, 0, s, a); break;
    case 2: OAC_LAUNCH((policy_head_kernel<2, KP, KS>), grid, block, 0, s, a); break;
    case 3: OAC_LAUNCH((policy_head_kernel<3, KP, KS>), grid, block, 0, s, a); break;
    default: OAC_LAUNCH((policy_head_kernel<4, KP, KS>), grid, block, 0, s, a); break;
  }
}

hipError_t launch_policy_head(const HeadArgs& a, int nseg, hipStream_t s) {
  if (a.Da < 1 || 2 * a.Da > 64 || a.col_chunks < 1 || nseg < 1 || nseg > 3 ||
      (nseg > 2 && !a.det))
    return hipErrorInvalidValue;
  for (int i = 0; i < nseg; ++i)
    if (a.seg[i].n_nets < 0 || a.seg[i].n_nets > 2) return hipErrorInvalidValue;
  // every (net, 16-column tile) of a workgroup's chunk is prefetched: <= 4 per wave
  const int cols = (a.H + a.col_chunks - 1) / a.col_chunks;
  int pairs = 0;
  for (int i = 0; i < nseg; ++i) pairs = std::max(pairs, a.seg[i].n_nets * ((cols + 15) / 16));
  if (pairs > 4 * kHeadWaves) return hipErrorInvalidValue;
  const int rblocks = (a.B + kRows - 1) / kRows;
  const dim3 grid(rblocks * a.col_chunks, nseg), block(64 * kHeadWaves);
  const bool kp4 = pairs > 2 * kHeadWaves;
  if (a.Da <= 8) {
    if (kp4) launch_head_nt<4, 2>(a, grid, block, s); else launch_head_nt<2, 2>(a, grid, block, s);
  } else if (a.Da <= 20) {
    if (kp4) launch_head_nt<4, 5>(a, grid, block, s); else launch_head_nt<2, 5>(a, grid, block, s);
  } else {
    if (kp4) launch_head_nt<4, 8>(a, grid, block, s); else launch_head_nt<2, 8>(a, grid, block, s);
  }
  return hipGetLastError();
}

}  // namespace oac
