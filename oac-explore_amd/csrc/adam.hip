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
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) adam_flat_elem(c, a, i);
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
  OAC_LAUNCH(adam_flat_kernel, dim3(adam_blocks((a.n + 3) >> 2)), dim3(256), 0, s, a);
  return hipGetLastError();
}


}  // namespace oac
