// OAC exploration action as ONE launch: one 1024-thread workgroup per
// observation computes the whole get_optimistic_exploration_action_stochastic
// (/root/reference/optimistic_exploration.py:14-109, two critics, trainer=None)
// for its row, with every intermediate in LDS:
//   policy MLP -> head (mean | log std), std, a = tanh(mean)       (:24-33)
//   Q1, Q2 on [ob | a]; Q_UB = (Q1+Q2)/2 + beta |Q1-Q2|/2           (:35-47)
//   dQ_UB/da by hand: seeds w_i = 1/2 +- beta/2 sign(Q1-Q2) through the
//   last layer, the layer-1 ReLU, W1, the layer-0 ReLU, W0[:, Do:]  (:49-58)
//   grad = dQ_UB/da (1 - a^2), Sigma = std^2,
//   mu_C = sqrt(2 delta) Sigma grad / (sqrt(grad^T Sigma grad) + 1e-5),
//   action = tanh(mu_T + mu_C + std eps)                            (:60-109)
// It replaces a ten-launch GEMM sequence (~70 us per call at one observation,
// each launch a few dependent L2 round trips for ~0.1 MFLOP) at about the same
// device time for one observation: one workgroup streams the row's 2.7 MB of
// weights (Humanoid dims) at ~45-110 GB/s per layer (measured with the stage
// clocks of tools/expl_latency.py; neither 16-byte loads nor an out-of-line
// matvec changed it -- the single CU's memory path is the limit), but one
// launch instead of ten, and N observations are N independent workgroups: a
// row's result does not depend on N (the vectorised-rollout contract) and 64
// observations cost about what one does.
//
// Matrix-vector products: a wave per output row, lanes along the contiguous k
// of the weight row (coalesced), four rows per wave in flight, a fixed-order
// shuffle reduction; the transposed product of the backward (dh1 = dh2 . W1)
// runs a thread per (output column, quarter of the rows), coalesced along k,
// 32 loads in flight per thread, partials added in fixed order.
#include "oac_common.h"
#include "kernels.h"

namespace oac {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// y[n] = act(sum_k W[n, k] x[k] + b[n]), n < N (W row-major, leading dim ldw).
// A wave owns RW rows at a time and issues all of their loads for up to
// 64*U columns before the first FMA, so a layer costs a few L2 round trips
// rather than one per k step (the weight stream is latency-bound from one CU).
__device__ __forceinline__ void matvec(const float* __restrict__ W, long ldw, const float* __restrict__ b,
                                       const float* x, int K, int N, float* y, bool relu) {
  constexpr int RW = 8, U = 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // 16-byte rows (ldw % 4 == 0, aligned base): one dwordx4 per lane and row,
  // four times the bytes per load instruction (a single CU streams the
  // weights, so the load path, not HBM, is the limit)
  const bool vec = (ldw & 3) == 0 && ((reinterpret_cast<unsigned long>(W) & 15) == 0) && (K & 3) == 0;
  for (int n0 = wave * RW; n0 < N; n0 += nw * RW) {
    float acc[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[r] = 0.f;
    if (vec) {
      const int K4 = K >> 2;
      for (int cb = 0; cb < K4; cb += 64 * 2) {
        float4 wv[RW][2], xv[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = cb + u * 64 + lane;
          const int cc = c < K4 ? c : K4 - 1;
          const float4 xx = reinterpret_cast<const float4*>(x)[cc];
          xv[u] = c < K4 ? xx : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int r = 0; r < RW; ++r)
            wv[r][u] = reinterpret_cast<const float4*>(W + (long)min(n0 + r, N - 1) * ldw)[cc];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < RW; ++r) {
            acc[r] = fmaf(wv[r][u].x, xv[u].x, acc[r]);
            acc[r] = fmaf(wv[r][u].y, xv[u].y, acc[r]);
            acc[r] = fmaf(wv[r][u].z, xv[u].z, acc[r]);
            acc[r] = fmaf(wv[r][u].w, xv[u].w, acc[r]);
          }
      }
    } else
    for (int kb = 0; kb < K; kb += 64 * U) {
      float wv[RW][U], xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = kb + u * 64 + lane;
        const int kc = k < K ? k : K - 1;
        xv[u] = k < K ? x[kc] : 0.f;
#pragma unroll
        for (int r = 0; r < RW; ++r) wv[r][u] = W[(long)min(n0 + r, N - 1) * ldw + kc];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RW; ++r) acc[r] = fmaf(wv[r][u], xv[u], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[r] = wave_sum(acc[r]);
    if (lane < RW && n0 + lane < N) {
      float a = acc[0];
#pragma unroll
      for (int r = 1; r < RW; ++r) a = lane == r ? acc[r] : a;
      const float v = a + b[n0 + lane];
      y[n0 + lane] = relu ? fmaxf(v, 0.f) : v;
    }
  }
}

#define XSTAGE(i) \
  if (a.stage_clock && r == 0 && t == 0) a.stage_clock[i] = wall_clock64()

__global__ void __launch_bounds__(1024) oac_expl_fused_kernel(ExplFusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Do = a.Do, Da = a.Da, H = a.H, Dq = Do + Da;
  const int r = blockIdx.x, t = threadIdx.x;
  float* x = sm;                           // [Do + Da]  ob | a
  float* h1 = x + ((Dq + 3) & ~3);         // [H] policy hidden
  float* h2 = h1 + H;
  float* head = h2 + H;                    // [2 Da]
  float* qh1 = head + 128;                 // [2][H]
  float* qh2 = qh1 + 2 * H;                // [2][H]
  float* dh1 = qh2 + 2 * H;                // [2][H]
  float* da = dh1 + 2 * H;                 // [2][64]
  float* misc = da + 128;                  // q1, q2, w1, w2, denom | reduction scratch [64]
  __shared__ long long cnt_s;

  XSTAGE(0);
  if (t == 0) cnt_s = a.state->expl_counter;
  for (int k = t; k < Do; k += blockDim.x) x[k] = a.obs[(long)r * a.ld_obs + k];
  __syncthreads();

  // ---- policy forward (TanhGaussianPolicy.forward, policies.py:272-283)
  matvec(a.pol + a.p_fc0_w, Do, a.pol + a.p_fc0_b, x, Do, H, h1, true);
  __syncthreads();
  XSTAGE(1);
  matvec(a.pol + a.p_fc1_w, H, a.pol + a.p_fc1_b, h1, H, H, h2, true);
  __syncthreads();
  XSTAGE(2);
  matvec(a.pol + a.p_head_w, H, a.pol + a.p_head_b, h2, H, 2 * Da, head, false);
  __syncthreads();
  XSTAGE(9);
  // std = exp(clamp(log_std)); a = tanh(mu_T) appended to the critic input
  if (t < Da) x[Do + t] = tanhf(head[t]);
  __syncthreads();

  // ---- critics on [ob | a]
  XSTAGE(3);
  const int nq = a.nq, KQ = a.K;
  float* qk = da + 64;                     // share_layers: K head values, then their seeds
  float* wk = qk + 16;
  for (int i = 0; i < nq; ++i) {
    const float* q = a.q[i];
    matvec(q + a.q_fc0_w, Dq, q + a.q_fc0_b, x, Dq, H, qh1 + i * H, true);
    if (i == 0) XSTAGE(10);
  }
  __syncthreads();
  XSTAGE(4);
  for (int i = 0; i < nq; ++i) {
    const float* q = a.q[i];
    matvec(q + a.q_fc1_w, H, q + a.q_fc1_b, qh1 + i * H, H, H, qh2 + i * H, true);
  }
  __syncthreads();
  if (nq == 2) {
    const int wave = t >> 6, lane = t & 63;
    if (wave < 2) {
      const float* q = a.q[wave];
      float s = 0.f;
      for (int k = lane; k < H; k += 64) s = fmaf(q[a.q_last_w + k], qh2[wave * H + k], s);
      s = wave_sum(s);
      if (lane == 0) misc[wave] = s + q[a.q_last_b];
    }
  } else {
    matvec(a.q[0] + a.q_last_w, H, a.q[0] + a.q_last_b, qh2, H, KQ, qk, false);
  }
  __syncthreads();
  if (t == 0) {
    if (nq == 2) {   // Q_UB = (Q1+Q2)/2 + beta |Q1-Q2|/2: d|x|/dx = sign(x) (0 at 0)
      const float d = misc[0] - misc[1];
      const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      const float hb = a.beta_UB / 2.f;
      misc[2] = 0.5f + hb * sg;
      misc[3] = 0.5f - hb * sg;
    } else if (a.ub_index >= 0) {   // trainer_UB: Q_UB = sort_k(q)[ub_index] -> seed 1 on
                                    // the head ranked there (ties: lower head index first)
      for (int k = 0; k < KQ; ++k) {
        int rank = 0;
        for (int j = 0; j < KQ; ++j) rank += (qk[j] < qk[k]) || (qk[j] == qk[k] && j < k);
        wk[k] = rank == a.ub_index ? 1.f : 0.f;
      }
    } else {         // Q_UB = mean_k q + beta std_k q (unbiased): dQ_UB/dq_k =
                     // 1/K + beta (q_k - mean) / ((K-1) std)
      float sm = 0.f;
      for (int k = 0; k < KQ; ++k) sm += qk[k];
      const float mu = sm / (float)KQ;
      float ss = 0.f;
      for (int k = 0; k < KQ; ++k) ss += (qk[k] - mu) * (qk[k] - mu);
      const float sd = sqrtf(ss / (float)(KQ - 1));
      for (int k = 0; k < KQ; ++k)
        wk[k] = 1.f / (float)KQ + a.beta_UB * ((qk[k] - mu) / ((float)(KQ - 1) * sd));
    }
  }
  __syncthreads();

  XSTAGE(5);
  // ---- dQ_UB/da: dh2_i[n] = [qh2_i[n] > 0] sum_k w_ik Wl_i[k, n] (kept in qh2),
  //      dh1_i[k] = [qh1_i[k] > 0] sum_n dh2_i[n] W1_i[n, k], da_i = dh1_i . W0_i[:, Do:]
  for (int e = t; e < nq * H; e += blockDim.x) {
    const int i = e / H, n = e - i * H;
    float sv;
    if (nq == 2) {
      sv = misc[2 + i] * a.q[i][a.q_last_w + n];
    } else {
      sv = 0.f;
      for (int k = 0; k < KQ; ++k) sv = fmaf(wk[k], a.q[0][a.q_last_w + (long)k * H + n], sv);
    }
    qh2[e] = qh2[e] > 0.f ? sv : 0.f;
  }
  __syncthreads();
  {
    // dh1 = dh2 . W1: column k of W1 is strided, so the rows n are split into
    // P = blockDim / H parts (thread: column k, part p), each part's loads
    // issued 32 at a time, and the P partial sums added in fixed order
    float* part = misc + 72;                // [P][H] partials
    const int P = blockDim.x / H >= 1 ? (int)blockDim.x / H : 1;
    const int rows = (H + P - 1) / P;
    for (int i = 0; i < nq; ++i) {
      const float* W1 = a.q[i] + a.q_fc1_w;
      const float* g = qh2 + i * H;
      for (int e = t; e < P * H; e += blockDim.x) {
        const int p = e / H, k = e - p * H;
        const int n_lo = p * rows, n_hi = min(H, n_lo + rows);
        float s = 0.f;
        for (int n0 = n_lo; n0 < n_hi; n0 += 32) {
          float w[32];
#pragma unroll
          for (int u = 0; u < 32; ++u) w[u] = W1[(long)min(n0 + u, n_hi - 1) * H + k];
#pragma unroll
          for (int u = 0; u < 32; ++u)
            if (n0 + u < n_hi) s = fmaf(g[n0 + u], w[u], s);
        }
        part[e] = s;
      }
      __syncthreads();
      for (int k = t; k < H; k += blockDim.x) {
        float s = part[k];
        for (int p = 1; p < P; ++p) s += part[p * H + k];
        dh1[i * H + k] = qh1[i * H + k] > 0.f ? s : 0.f;
      }
      __syncthreads();
    }
  }
  XSTAGE(6);
  {
    const int lane = t & 63, wave = t >> 6, nw = blockDim.x >> 6;
    for (int o = wave; o < nq * Da; o += nw) {
      const int i = o / Da, j = o - i * Da;
      const float* W0 = a.q[i] + a.q_fc0_w + Do + j;
      float s = 0.f;
      for (int n = lane; n < H; n += 64) s = fmaf(dh1[i * H + n], W0[(long)n * Dq], s);
      s = wave_sum(s);
      if (lane == 0) da[i * 64 + j] = s;
    }
  }
  __syncthreads();

  XSTAGE(7);
  // ---- shift and sample (optimistic_exploration.py:60-109)
  float g = 0.f, sig = 0.f, sd = 0.f, mean = 0.f;
  float* red = misc + 8;
  if (t < Da) {
    const float act = x[Do + t];
    g = (nq == 2 ? da[t] + da[64 + t] : da[t]) * (1.f - act * act);
    sd = expf(fminf(fmaxf(head[Da + t], -20.f), 2.f));
    sig = sd * sd;
    mean = head[t];
    red[t] = g * g * sig;
  }
  __syncthreads();
  if (t == 0) {
    float s = 0.f;
    for (int i = 0; i < Da; ++i) s += red[i];
    misc[4] = sqrtf(s) + 10e-6f;
  }
  __syncthreads();
  if (t < Da) {
    const long e = (long)r * Da + t;
    const float mu_C = (a.sqrt_2delta * (sig * g)) / misc[4];
    const float mu_E = mean + mu_C;
    const float ev = a.eps ? a.eps[e]
                           : philox_normal(a.seed, (unsigned long long)cnt_s, 3u, (unsigned)(r * Da + t));
    const long nd = (long)a.n * Da;
    a.out[e] = tanhf(__fadd_rn(__fmul_rn(ev, sd), mu_E));   // action
    a.out[nd + e] = mu_E;
    a.out[2 * nd + e] = sd;
    if (a.grad) a.grad[e] = g;
  }
  XSTAGE(8);
  // the Philox counter advances once per call: the last workgroup to finish
  // (every other one has read it) bumps it and re-arms the ticket
  if (!a.eps) {
    __syncthreads();
    if (t == 0) {
      __threadfence();
      const unsigned prev = atomicAdd(a.ticket, 1u);
      if (prev == (unsigned)a.n - 1) {
        a.state->expl_counter = cnt_s + 1;
        atomicExch(a.ticket, 0u);
      }
    }
  }
}

size_t expl_fused_lds_bytes(int Do, int Da, int H) {
  const int Dq = Do + Da;
  const int P = 1024 / H >= 1 ? 1024 / H : 1;
  const size_t parts = (size_t)P * H > (size_t)H ? (size_t)P * H : (size_t)H;
  return sizeof(float) * (((Dq + 3) & ~3) + 2 * (size_t)H + 128 + 6 * (size_t)H + 128 + 72 + parts);
}

hipError_t launch_expl_fused(const ExplFusedArgs& a, hipStream_t s) {
  if (a.n < 1 || a.Da < 1 || a.Da > 63 || a.H < 1) return hipErrorInvalidValue;
  const size_t lds = expl_fused_lds_bytes(a.Do, a.Da, a.H);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  OAC_LAUNCH(oac_expl_fused_kernel, dim3(a.n), dim3(1024), lds, s, a);
  return hipGetLastError();
}

}  // namespace oac
