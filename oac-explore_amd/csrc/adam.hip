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

// LANES threads per float4: with split-K slabs (9 <= S <= 32) each lane sums
// one chunk of 8 slabs (slab_chunk), lane 0 adds the chunk sums in chunk
// order -- the same bits as one thread per element (adam_flat_elem), with
// every slab load of the element in flight at once across the lanes and 4x
// the workgroups: configs[4]'s critic / policy Adam (100k parameters, 32
// slabs) ran as 98 workgroups, one float4 and four dependent chunk rounds per
// thread
template <int LANES>
__global__ void __launch_bounds__(256) adam_flat_kernel(AdamArgs a) {
  const AdamConsts c = adam_consts(a.state, a.advance, a.lr, a.beta1, a.beta2, a.eps, a.target,
                                   a.tau, a.period);
  const long n4 = a.n >> 2;
  if (LANES == 1) {
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) adam_flat_elem(c, a, i);
  } else {
    const int q = threadIdx.x % LANES;
    const long stride = (long)gridDim.x * (256 / LANES);
    for (long i0 = (long)blockIdx.x * (256 / LANES); i0 < n4; i0 += stride) {
      const long i = i0 + threadIdx.x / LANES;   // (uniform trip count: every lane shuffles)
      const long ic = i < n4 ? i : n4 - 1;
      const int S = slab_count(a, ic);
      const int nc = (S + kSlabChunk - 1) / kSlabChunk;   // <= LANES (launcher: S2 <= S)
      float4 p = q < nc ? slab_chunk(a, ic, q, S) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 g = p;
#pragma unroll
      for (int j = 1; j < LANES; ++j) {   // chunk sums in chunk order, at lane 0 of the group
        float4 r;
        r.x = __shfl(p.x, (threadIdx.x & 63) - q + j); r.y = __shfl(p.y, (threadIdx.x & 63) - q + j);
        r.z = __shfl(p.z, (threadIdx.x & 63) - q + j); r.w = __shfl(p.w, (threadIdx.x & 63) - q + j);
        if (j < nc) add4(g, r);
      }
      if (q == 0 && i < n4) adam_flat_finish(c, a, i, g, true);
    }
  }
  if (a.reduce_only || a.no_book) return;
  step_bookkeeping(a.state, a.alpha, a.advance);
}

static int adam_blocks(long n, int per_block) {
  long b = (n + per_block - 1) / per_block;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

hipError_t launch_adam(const AdamArgs& a, hipStream_t s) {
  if (a.n & 3) return hipErrorInvalidValue;   // arena ranges are 16-byte multiples
  const long n4 = (a.n + 3) >> 2;
  const bool slabs = a.S > 1 || a.gslab != a.g;
  if (slabs && a.S > kSlabChunk && a.S <= kSlabChunk * kSlabLanes)
    OAC_LAUNCH(adam_flat_kernel<kSlabLanes>, dim3(adam_blocks(n4, 256 / kSlabLanes)), dim3(256), 0, s, a);
  else
    OAC_LAUNCH(adam_flat_kernel<1>, dim3(adam_blocks(n4, 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}


}  // namespace oac
