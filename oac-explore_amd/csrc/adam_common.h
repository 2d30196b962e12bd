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

// The split-K slabs of float4 i summed in a fixed order that depends on the
// element alone: chunks of kSlabChunk consecutive slabs, each summed in slab
// order, then the chunk sums in chunk order -- so one thread per element (the
// side workgroups, adam_flat_elem) and kSlabLanes lanes per element, one chunk
// each (adam_flat_kernel), give the same bits.
constexpr int kSlabChunk = 8;
constexpr int kSlabLanes = 4;   // lanes per element in adam_flat_kernel (S <= 32)
__device__ __forceinline__ int slab_count(const AdamArgs& a, long i) {
  const long x = 4 * i;
  return (x >= a.s2_lo && x < a.s2_hi) ? min(a.S2, a.S) : a.S;
}
__device__ __forceinline__ float4 slab_chunk(const AdamArgs& a, long i, int c, int S) {
  const float4* gs = reinterpret_cast<const float4*>(a.gslab) + i;
  const long st4 = a.slab_stride >> 2;
  const int k0 = c * kSlabChunk, k1 = min(S, k0 + kSlabChunk);
  float4 x[kSlabChunk];
#pragma unroll
  for (int j = 0; j < kSlabChunk; ++j)   // every load of the chunk in flight together
    if (k0 + j < k1) x[j] = gs[(long)(k0 + j) * st4];
  float4 g = x[0];
#pragma unroll
  for (int j = 1; j < kSlabChunk; ++j)
    if (k0 + j < k1) { g.x += x[j].x; g.y += x[j].y; g.z += x[j].z; g.w += x[j].w; }
  return g;
}
__device__ __forceinline__ void add4(float4& g, const float4& p) {
  g.x += p.x; g.y += p.y; g.z += p.z; g.w += p.w;
}

// the reduced gradient (written back to g), optionally scaled, then Adam (+
// Polyak): the body of adam_flat_kernel and of the large-batch GEMMs' side
// workgroups
__device__ __forceinline__ void adam_flat_finish(const AdamConsts& c, const AdamArgs& a, long i,
                                                 float4 g, bool reduced) {
  if (reduced) reinterpret_cast<float4*>(a.g)[i] = g;
  if (a.reduce_only) return;
  if (a.gscale != 1.f) { g.x *= a.gscale; g.y *= a.gscale; g.z *= a.gscale; g.w *= a.gscale; }
  adam_float4(c, a, i, g);
}

// float4 i of a flat range, one thread (slab order: slab_chunk)
__device__ __forceinline__ void adam_flat_elem(const AdamConsts& c, const AdamArgs& a, long i) {
  if (a.S > 1 || a.gslab != a.g) {
    const int S = slab_count(a, i);
    float4 g = slab_chunk(a, i, 0, S);
    const int nc = (S + kSlabChunk - 1) / kSlabChunk;
#pragma unroll 1
    for (int ch = 1; ch < nc; ++ch) add4(g, slab_chunk(a, i, ch, S));
    adam_flat_finish(c, a, i, g, true);
  } else {
    adam_flat_finish(c, a, i, reinterpret_cast<const float4*>(a.g)[i], false);
  }
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
    r.s2_lo -= off; r.s2_hi -= off;
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
