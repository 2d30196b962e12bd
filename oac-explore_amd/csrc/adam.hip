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
#include "adam_common.h"

namespace oac {

__global__ void __launch_bounds__(256) adam_flat_kernel(AdamArgs a) {
  const AdamConsts c = adam_consts(a.state, a.advance, a.lr, a.beta1, a.beta2, a.eps, a.target,
                                   a.tau, a.period);
  const long n4 = a.n >> 2;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    float4 g;
    if (a.S > 1 || a.gslab != a.g) {
      // slabs summed in fixed order 0, 1, ..., S-1; the loads of 8 slabs are
      // issued together (a one-slab-per-iteration loop waited out S
      // dependent round trips: B=4096, S=32 -> ~11 us per launch)
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
    if (a.reduce_only) continue;
    if (a.gscale != 1.f) { g.x *= a.gscale; g.y *= a.gscale; g.z *= a.gscale; g.w *= a.gscale; }
    adam_float4(c, a, i, g);
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
  OAC_LAUNCH(adam_flat_kernel, dim3(adam_blocks((a.n + 3) >> 2)), dim3(256), 0, s, a);
  return hipGetLastError();
}


}  // namespace oac
