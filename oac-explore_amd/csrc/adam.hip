// Fused Adam (torch 1.4 optim.Adam.step semantics, as constructed at
// /root/reference/trainer/trainer.py:75-91) + Polyak soft update
// (utils/pytorch_util.py:5-9, called at trainer.py:215-224 with the POST-step
// parameters).  HBM-bound elementwise.
//
// The weight-gradient GEMMs write their results in the parameter-arena
// layout; with split-K they write S partial slabs shaped like the arena, which
// this pass sums in fixed slab order (deterministic) before the update -- one
// float4 pass over g, p, m, v (and target).  Data-parallel: a reduce-only pass
// writes the summed gradient, the caller all-reduces it, then the update pass
// runs with gscale = 1/world.
#include "oac_common.h"
#include "kernels.h"

namespace oac {

struct AdamConsts { float b1, omb1, b2, omb2, step_size, sbc2, eps, tau, omtau; bool polyak; };

__device__ __forceinline__ AdamConsts adam_consts(const StepState* st, int advance, double lr,
                                                  double beta1, double beta2, double eps,
                                                  const float* target, float tau, int period) {
  const long long nsteps = advance ? st->t_snapshot : st->n_steps;
  const double t = (double)(nsteps + 1);
  const double bc1 = 1.0 - pow(beta1, t);
  const double bc2 = 1.0 - pow(beta2, t);
  AdamConsts c;
  c.b1 = (float)beta1; c.omb1 = (float)(1.0 - beta1);
  c.b2 = (float)beta2; c.omb2 = (float)(1.0 - beta2);
  c.step_size = (float)(lr / bc1);
  c.sbc2 = (float)sqrt(bc2);
  c.eps = (float)eps;
  c.tau = tau; c.omtau = (float)(1.0 - (double)tau);
  c.polyak = target && (period <= 1 || (nsteps % period) == 0);
  return c;
}

// m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g g ; p += -(lr/bc1) m / (sqrt(v)/sqrt(bc2) + eps)
__device__ __forceinline__ void adam1(const AdamConsts& c, float& p, float g, float& m, float& v) {
  m = __fadd_rn(__fmul_rn(m, c.b1), __fmul_rn(c.omb1, g));
  v = __fadd_rn(__fmul_rn(v, c.b2), __fmul_rn(__fmul_rn(c.omb2, g), g));
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), c.sbc2), c.eps);
  p = __fadd_rn(p, __fdiv_rn(__fmul_rn(-c.step_size, m), denom));
}

// target = target*(1-tau) + p*tau
__device__ __forceinline__ float polyak1(const AdamConsts& c, float t, float p) {
  return __fadd_rn(__fmul_rn(t, c.omtau), __fmul_rn(p, c.tau));
}

// Block 0, thread 0 only.  advance == 0 (critic Adam): snapshot t for the
// final Adam; advance == 1 (final policy Adam): advance the step counters.
// Either may commit the alpha update published earlier in the step (`as`
// non-null: SAC commits in the critic Adam, the particle trainer -- whose
// alpha update comes after the critic step -- in the policy Adam).  No other
// block of the launch reads these fields.
__device__ __forceinline__ void step_bookkeeping(StepState* st, AlphaState* as, int advance) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  if (advance) {
    st->n_steps = st->t_snapshot + 1;
    st->batch_counter += 1;
  } else {
    st->t_snapshot = st->n_steps;
  }
  if (as) { as->log_alpha = as->next_log_alpha; as->m = as->next_m; as->v = as->next_v; }
}

__global__ void __launch_bounds__(256) adam_flat_kernel(AdamArgs a) {
  const AdamConsts c = adam_consts(a.state, a.advance, a.lr, a.beta1, a.beta2, a.eps, a.target,
                                   a.tau, a.period);
  const long n4 = a.n >> 2;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    float4 g;
    if (a.S > 1 || a.gslab != a.g) {
      g = reinterpret_cast<const float4*>(a.gslab)[i];
#pragma unroll 1
      for (int k = 1; k < a.S; ++k) {
        const float4 x = reinterpret_cast<const float4*>(a.gslab + (long)k * a.slab_stride)[i];
        g.x += x.x; g.y += x.y; g.z += x.z; g.w += x.w;
      }
      reinterpret_cast<float4*>(a.g)[i] = g;
    } else {
      g = reinterpret_cast<const float4*>(a.g)[i];
    }
    if (a.reduce_only) continue;
    if (a.gscale != 1.f) { g.x *= a.gscale; g.y *= a.gscale; g.z *= a.gscale; g.w *= a.gscale; }
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
  if (a.reduce_only) return;
  step_bookkeeping(a.state, a.alpha, a.advance);
}

static int adam_blocks(long n) {
  long b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

hipError_t launch_adam(const AdamArgs& a, hipStream_t s) {
  if (a.n & 3) return hipErrorInvalidValue;   // arena ranges are 16-byte multiples
  hipLaunchKernelGGL(adam_flat_kernel, dim3(adam_blocks((a.n + 3) >> 2)), dim3(256), 0, s, a);
  return hipGetLastError();
}


}  // namespace oac
