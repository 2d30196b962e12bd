// Alpha update and twin-min TD target of SACTrainer.train_from_torch
// (/root/reference/trainer/trainer.py:139-196), per row / per block, for
// critic_targets_kernel (rows.hip).
//
// (Measured and rejected at B=256: (1) folding this into the critic-backward
// GEMM launch as a prologue every workgroup runs over all B rows -- the dW
// tiles need every row's dq -- made that launch ~14 us slower than the two
// launches it replaced (~290 workgroups re-reading the same 32 KB of head
// partials); (2) running it as the row-block tail of the layer-1 launch (the
// last arriving tile of each 32-row block, partials handed off write-through
// + an agent-scope arrival counter) removed the launch but not the time: the
// step stayed at 98-99 us, the tail's own dependent round trips costing what
// the launch boundary did.)
#pragma once
#include "adam_common.h"
#include "kernels.h"

namespace oac {

// sum over all B rows of (logp + target_entropy) in a fixed order that does
// not depend on the block size: threads 0..255 accumulate rows i, i+256, ...,
// then a 256-wide tree.  red: 256 floats of LDS.  Every thread gets the sum.
__device__ __forceinline__ float logp_sum256(const float* logp, int B, float te, float* red) {
  if (threadIdx.x < 256) {
    // the same sequential order per thread, its loads issued 16 at a time
    // (a plain loop waited one memory round trip per 256 rows: at B=4096
    // that was most of the critic-targets launch)
    float acc = 0.f;
    int i = threadIdx.x;
    for (; i + 15 * 256 < B; i += 16 * 256) {
      float v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = logp[i + 256 * k];
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += v[k] + te;
    }
    for (; i < B; i += 256) acc += logp[i] + te;
    red[threadIdx.x] = acc;
  }
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float sum = red[0];
  __syncthreads();
  return sum;
}

// alpha update (trainer.py:139-146): L = -mean(log_alpha * (logp + H)), Adam
// on log_alpha with t = n_steps + 1, then alpha = exp(log_alpha).  Returns the
// new alpha; `publish`: also stage next_* / diagnostics (the critic Adam
// commits them), done by exactly one block of a launch.
__device__ __forceinline__ float alpha_update(const CriticTargetArgs& p, float S, bool publish) {
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
  const float alpha = expf(la);
  if (publish) {
    as->next_log_alpha = la; as->next_m = m; as->next_v = v;
    as->alpha = alpha; as->grad = g; as->alpha_loss = -(la_old * S) / n;
  }
  return alpha;
}

// One row's critic values (QV_* order) from the per-tile partial dots of the
// width-1 heads (n_part > 0: bias + fixed-order sum) or the stored q.
struct TargetRowIn {
  float pv[QV_COUNT][16];
  float pb[QV_COUNT];
  float rew, term, logp2;
};

__device__ __forceinline__ void target_row_load(const CriticTargetArgs& p, int rc, TargetRowIn& x) {
  if (p.n_part > 0) {
#pragma unroll
    for (int k = 0; k < QV_COUNT; ++k) {
      const float* pp = p.part[k] + rc;
#pragma unroll
      for (int t = 0; t < 16; ++t)   // unconditional (all in flight), coalesced over rows
        x.pv[k][t] = pp[(long)min(t, p.n_part - 1) * p.B];
    }
  } else {   // (every element assigned on both paths: a partly assigned
             // array kept two of them in scratch across the merge)
#pragma unroll
    for (int k = 0; k < QV_COUNT; ++k) {
      x.pv[k][0] = p.q[k][rc];
#pragma unroll
      for (int t = 1; t < 16; ++t) x.pv[k][t] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < QV_COUNT; ++k) x.pb[k] = p.n_part > 0 ? p.part_bias[k][0] : 0.f;
  x.rew = p.batch[(long)rc * p.ld_batch + p.off_rew];
  x.term = p.batch[(long)rc * p.ld_batch + p.off_term];
  x.logp2 = p.logp2[rc];
}

// y = scale r + (1-d) gamma (min(tq1, tq2) - alpha logp');  dq_i = 2 (q_i - y) / B;
// policy seeds g_i = -1/B on the min critic (torch-1.4 min backward: ties to
// the first).  write: store every per-row output of the step (one block).
__device__ __forceinline__ void target_row(const CriticTargetArgs& p, int r, const TargetRowIn& x,
                                           float alpha, bool write, float& dq1, float& dq2) {
  float qv[QV_COUNT];
#pragma unroll
  for (int k = 0; k < QV_COUNT; ++k) {
    if (p.n_part > 0) {
      float s = x.pb[k];
#pragma unroll
      for (int t = 0; t < 16; ++t)
        if (t < p.n_part) s += x.pv[k][t];
      qv[k] = s;
      if (write) p.q[k][r] = s;
    } else {
      qv[k] = x.pv[k][0];
    }
  }
  const float tq = fminf(qv[QV_TQ1], qv[QV_TQ2]) - __fmul_rn(alpha, x.logp2);
  const float y = __fadd_rn(__fmul_rn(p.reward_scale, x.rew),
                            __fmul_rn(__fmul_rn(1.f - x.term, p.discount), tq));
  const float d1 = qv[QV_Q1] - y, d2 = qv[QV_Q2] - y;
  const float invB = 1.f / (float)p.B;
  dq1 = __fmul_rn(2.f * d1, invB);
  dq2 = __fmul_rn(2.f * d2, invB);
  if (write) {
    p.y[r] = y;
    p.dq1[r] = dq1;
    p.dq2[r] = dq2;
    p.sqe1[r] = d1 * d1;
    p.sqe2[r] = d2 * d2;
    const float a = qv[QV_QN1], b = qv[QV_QN2];
    const bool sel1 = a <= b;
    p.qnew[r] = sel1 ? a : b;
    p.gq1[r] = sel1 ? -invB : 0.f;
    p.gq2[r] = sel1 ? 0.f : -invB;
  }
}

}  // namespace oac
