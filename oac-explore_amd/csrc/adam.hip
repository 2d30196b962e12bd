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

#include <cstdlib>

namespace oac {

__global__ void __launch_bounds__(256) adam_flat_kernel(AdamArgs a) {
  const AdamConsts c = adam_consts(a.state, a.advance, a.lr, a.beta1, a.beta2, a.eps, a.target,
                                   a.tau, a.period);
  const long n4 = a.n >> 2;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) adam_flat_elem(c, a, i);
  if (a.reduce_only || a.no_book) return;
  step_bookkeeping(a.state, a.alpha, a.advance);
}

// The standalone pass with every slab load of a float4 in flight at once
// (SMAX >= S slabs, the index clamped to S - 1 and the surplus terms added as
// +0, so the sum is the same left-to-right slab order as adam_flat_elem's,
// bitwise): the grouped form waited out ceil(S / 8) dependent round trips
// per float4, and a group's launch is a few hundred workgroups at most.
// (adam_flat_elem stays as it is for the GEMM side workgroups, where 4 x SMAX
// extra VGPRs would count against the GEMM kernel's occupancy.)
template <int SMAX>
__global__ void __launch_bounds__(256) adam_flat_wide_kernel(AdamArgs a) {
  const AdamConsts c = adam_consts(a.state, a.advance, a.lr, a.beta1, a.beta2, a.eps, a.target,
                                   a.tau, a.period);
  const long n4 = a.n >> 2;
  const long stride = (long)gridDim.x * 256;
  const long st4 = a.slab_stride >> 2;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    const float4* gs = reinterpret_cast<const float4*>(a.gslab) + i;
    float4 x[SMAX];
#pragma unroll
    for (int j = 0; j < SMAX; ++j) x[j] = gs[(long)min(j, a.S - 1) * st4];
    float4 g = x[0];
#pragma unroll
    for (int j = 1; j < SMAX; ++j) {
      const bool in = j < a.S;   // a select, not a branch: +0 past the last slab
      g.x += in ? x[j].x : 0.f; g.y += in ? x[j].y : 0.f;
      g.z += in ? x[j].z : 0.f; g.w += in ? x[j].w : 0.f;
    }
    reinterpret_cast<float4*>(a.g)[i] = g;
    if (a.reduce_only) continue;
    if (a.gscale != 1.f) { g.x *= a.gscale; g.y *= a.gscale; g.z *= a.gscale; g.w *= a.gscale; }
    adam_float4(c, a, i, g);
  }
  if (a.reduce_only || a.no_book) return;
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
  const dim3 grid(adam_blocks((a.n + 3) >> 2));
  static const bool wide = [] { const char* e = getenv("OAC_ADAM_WIDE"); return !e || atoi(e) != 0; }();
  if (wide && (a.S > 1 || a.gslab != a.g) && a.S <= 32) {
    if (a.S <= 8) OAC_LAUNCH(adam_flat_wide_kernel<8>, grid, dim3(256), 0, s, a);
    else if (a.S <= 16) OAC_LAUNCH(adam_flat_wide_kernel<16>, grid, dim3(256), 0, s, a);
    else OAC_LAUNCH(adam_flat_wide_kernel<32>, grid, dim3(256), 0, s, a);
    return hipGetLastError();
  }
  OAC_LAUNCH(adam_flat_kernel, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}


}  // namespace oac
