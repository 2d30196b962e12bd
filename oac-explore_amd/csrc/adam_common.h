// torch-1.4 Adam (optim.Adam.step as constructed at
// /root/reference/trainer/trainer.py:75-91) and Polyak (utils/pytorch_util.py:5-9)
// element updates, shared by the flat Adam kernel (adam.hip) and the GEMM
// epilogues that apply the optimizer to the gradient tile they just produced
// (gemm_small.hip) -- one formula, so both paths are bitwise identical.
#pragma once
#include "oac_common.h"

namespace oac {

struct AdamConsts { float b1, omb1, b2, omb2, step_size, sbc2, eps, tau, omtau; bool polyak; };

// bias corrections of step t (torch-1.4 Adam: bias_correction1/2 in double)
__device__ __forceinline__ void bias_corrections(const StepState* st, long long t, double beta1,
                                                 double beta2, double& bc1, double& sbc2) {
  if (st->bc_t == t) {   // published by the step's first launch (same formula)
    bc1 = st->bc1; sbc2 = st->sbc2;
  } else {
    bc1 = 1.0 - pow(beta1, (double)t);
    sbc2 = sqrt(1.0 - pow(beta2, (double)t));
  }
}

// block 0, thread 0 of a step's first launch (no kernel of that launch reads it)
__device__ __forceinline__ void publish_step_consts(StepState* st, double beta1, double beta2) {
  const long long t = st->n_steps + 1;
  st->bc1 = 1.0 - pow(beta1, (double)t);
  st->bc2 = 1.0 - pow(beta2, (double)t);
  st->sbc2 = sqrt(st->bc2);
  st->bc_t = t;
}

__device__ __forceinline__ AdamConsts adam_consts(const StepState* st, int advance, double lr,
                                                  double beta1, double beta2, double eps,
                                                  const float* target, float tau, int period) {
  const long long nsteps = advance ? st->t_snapshot : st->n_steps;
  double bc1, sbc2;
  bias_corrections(st, nsteps + 1, beta1, beta2, bc1, sbc2);
  AdamConsts c;
  c.b1 = (float)beta1; c.omb1 = (float)(1.0 - beta1);
  c.b2 = (float)beta2; c.omb2 = (float)(1.0 - beta2);
  c.step_size = (float)(lr / bc1);
  c.sbc2 = (float)sbc2;
  c.eps = (float)eps;
  c.tau = tau; c.omtau = (float)(1.0 - (double)tau);
  c.polyak = target && (period <= 1 || (nsteps % period) == 0);
  return c;
}

// m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g g ; p += -(lr/bc1) m / (sqrt(v)/sqrt(bc2) + eps)
// Every operation rounded on its own, as torch's Adam does, in every caller:
// __fmul_rn / __fadd_rn are plain * / + inside the HIP headers, whose own
// contraction setting let the compiler fuse them into (packed) FMAs in the
// flat float4 pass but not in the GEMM epilogue, so the same update differed
// in the last bit between launch layouts -- hence plain operators under the
// pragma here (the pragma does not reach into a called header function)
__device__ __forceinline__ void adam1(const AdamConsts& c, float& p, float g, float& m, float& v) {
#pragma clang fp contract(off)
  m = m * c.b1 + c.omb1 * g;
  v = v * c.b2 + (c.omb2 * g) * g;
  const float denom = __fsqrt_rn(v) / c.sbc2 + c.eps;
  p = p + (-c.step_size * m) / denom;
}

// target = target*(1-tau) + p*tau
__device__ __forceinline__ float polyak1(const AdamConsts& c, float t, float p) {
#pragma clang fp contract(off)
  return t * c.omtau + p * c.tau;
}

// Block 0, thread 0 only.  advance == 0 (critic Adam): snapshot t for the
// final Adam; advance == 1 (final policy Adam): advance the step counters.
// Either may commit the alpha update published earlier in the step (`as`
// non-null: SAC commits in the critic Adam, the particle trainer -- whose
// alpha update comes after the critic step -- in the policy Adam).  No other
// block of the launch reads these fields.
__device__ __forceinline__ void step_bookkeeping_lead(StepState* st, AlphaState* as, int advance) {
  if (advance) {
    st->n_steps = st->t_snapshot + 1;
    st->batch_counter += 1;
  } else {
    st->t_snapshot = st->n_steps;
  }
  if (as) { as->log_alpha = as->next_log_alpha; as->m = as->next_m; as->v = as->next_v; }
}
__device__ __forceinline__ void step_bookkeeping(StepState* st, AlphaState* as, int advance) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  step_bookkeeping_lead(st, as, advance);
}

// one float4 of a flat range: g (already reduced) -> p, m, v (+ target)
__device__ __forceinline__ void adam_float4(const AdamConsts& c, const AdamArgs& a, long i, float4 g) {
  float4 p = reinterpret_cast<float4*>(a.p)[i];
  float4 m = reinterpret_cast<float4*>(a.m)[i];
  float4 v = reinterpret_cast<float4*>(a.v)[i];
  adam1(c, p.x, g.x, m.x, v.x);
  adam1(c, p.y, g.y, m.y, v.y);
  adam1(c, p.z, g.z, m.z, v.z);
  adam1(c, p.w, g.w, m.w, v.w);
  reinterpret_cast<float4*>(a.p)[i] = p;
  reinterpret_cast<float4*>(a.m)[i] = m;
  reinterpret_cast<float4*>(a.v)[i] = v;
  if (c.polyak) {
    float4 t = reinterpret_cast<float4*>(a.target)[i];
    t.x = polyak1(c, t.x, p.x); t.y = polyak1(c, t.y, p.y);
    t.z = polyak1(c, t.z, p.z); t.w = polyak1(c, t.w, p.w);
    reinterpret_cast<float4*>(a.target)[i] = t;
  }
}

// float4 i of a flat range: the split-K slabs summed in fixed order 0 .. S-1
// (written back to g), optionally scaled, then Adam (+ Polyak) -- the body of
// adam_flat_kernel (adam.hip) and of the large-batch GEMMs' side workgroups
__device__ __forceinline__ void adam_flat_elem(const AdamConsts& c, const AdamArgs& a, long i) {
  float4 g;
  if (a.S > 1 || a.gslab != a.g) {
    // the loads of 8 slabs are issued together (a one-slab-per-iteration loop
    // waited out S dependent round trips: B=4096, S=32 -> ~11 us per launch)
    const float4* gs = reinterpret_cast<const float4*>(a.gslab) + i;
    const long st4 = a.slab_stride >> 2;
    g = gs[0];
    int k = 1;
#pragma unroll 1
    for (; k + 8 <= a.S; k += 8) {
      float4 x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = gs[(long)(k + j) * st4];
#pragma unroll
      for (int j = 0; j < 8; ++j) { g.x += x[j].x; g.y += x[j].y; g.z += x[j].z; g.w += x[j].w; }
    }
#pragma unroll 1
    for (; k < a.S; ++k) {
      const float4 x = gs[(long)k * st4];
      g.x += x.x; g.y += x.y; g.z += x.z; g.w += x.w;
    }
    reinterpret_cast<float4*>(a.g)[i] = g;
  } else {
    g = reinterpret_cast<const float4*>(a.g)[i];
  }
  if (a.reduce_only) return;
  if (a.gscale != 1.f) { g.x *= a.gscale; g.y *= a.gscale; g.z *= a.gscale; g.w *= a.gscale; }
  adam_float4(c, a, i, g);
}

// side workgroup `blk` of `nblk` (256 threads each): the flat ranges of
// b.adam listed in b.seg_off / b.seg_n (GemmBatch::side_adam)
__device__ __forceinline__ void adam_side_block(const GemmBatch& b, int blk, int nblk) {
  const AdamArgs& a = b.adam;
  const AdamConsts c = adam_consts(a.state, a.advance, a.lr, a.beta1, a.beta2, a.eps, a.target,
                                   a.tau, a.period);
  const long stride = (long)nblk * 256;
  for (int sgi = 0; sgi < b.nseg; ++sgi) {
    AdamArgs r = a;
    const long off = b.seg_off[sgi];
    r.p += off; r.g += off; r.m += off; r.v += off; r.gslab += off;
    if (r.target) r.target += off;
    const long n4 = b.seg_n[sgi] >> 2;
    for (long i = (long)blk * 256 + threadIdx.x; i < n4; i += stride) adam_flat_elem(c, r, i);
  }
  if (b.side_book && blk == 0 && threadIdx.x == 0) step_bookkeeping_lead(a.state, a.alpha, a.advance);
}

// one element at index i of the group (GEMM epilogue)
__device__ __forceinline__ void adam_elem(const AdamConsts& c, const AdamArgs& a, long i, float g) {
  float p = a.p[i], m = a.m[i], v = a.v[i];
  adam1(c, p, g, m, v);
  a.p[i] = p; a.m[i] = m; a.v[i] = v;
  if (c.polyak) a.target[i] = polyak1(c, a.target[i], p);
}

}  // namespace oac
