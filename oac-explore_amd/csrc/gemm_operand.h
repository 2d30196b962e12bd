// Register-direct MFMA operand fetch shared by the small-batch GEMM
// (gemm_small.hip) and the large-batch register-direct GEMM (gemm_big.hip):
// one lane of a 32x32x2 fp32 MFMA holds row/column mn = lane & 31 and, per
// 8-deep k-group, k = 8g + 4*(lane >> 5) + c (c = 0..3), so a k-contiguous
// operand is one 16-byte load per lane per 4 MFMAs.
#pragma once
#include "oac_common.h"

namespace oac {

// Operand kinds (compile-time, so the k loop is straight-line code: every
// load of a wave's k-groups is issued before the first MFMA and fixed up
// -- masking, rank-1 products -- only afterwards).
//   OP_KC     X(mn,k) = p[mn*ld + k]                      (one 16-B load / 4 k)
//   OP_KC_R1  X(mn,k) = s[mn] * v[k] * (mask[mn*ld+k] > 0)
//   OP_MN     X(mn,k) = p[k*ld + mn]                      (dword, coalesced over mn)
//   OP_MN_R1  X(mn,k) = s[k] * v[mn] * (mask[k*ld+mn] > 0)
// k-contiguous loads are dword-aligned dwordx4 (gfx950 global memory takes
// them, so odd row strides such as the critic's 393-wide layer 0 stay
// vectorised) and may read up to 7 floats past a row's last k; those lanes
// are masked.  Every operand buffer is followed by >= 8 readable floats
// (workspace tail pad, arena neighbours, replay row padding).
enum OpKind { OP_KC = 0, OP_KC_R1 = 1, OP_MN = 2, OP_MN_R1 = 3 };

struct Lane {
  const float* p;     // kc: &X(mn, 0) ; mn: &X(0, mn)   (rank-1: of the mask)
  const float* s;     // rank-1 factor indexed by k
  long ld;
  float f;            // rank-1 factor indexed by mn
  bool valid;         // mn in range
  bool ones;          // virtual ones column (dW bias)
};

// rows (k-contiguous kinds only): row mn of the operand is buffer row rows[mn]
template <int KIND>
__device__ __forceinline__ Lane lane_init(int mn, int n_mn, bool ones, const float* p, long ld,
                                          const float* s, const float* v,
                                          const int* rows = nullptr) {
  Lane o;
  o.valid = mn < n_mn;
  o.ones = ones && mn == n_mn;
  const int m = o.valid ? mn : 0;
  o.ld = ld;
  const long mr = rows ? (long)rows[m] : (long)m;
  o.p = (KIND == OP_KC || KIND == OP_KC_R1) ? p + mr * ld : p + m;
  o.s = KIND == OP_KC_R1 ? v : s;
  o.f = KIND == OP_KC_R1 ? s[m] : (KIND == OP_MN_R1 ? v[m] : 1.f);
  return o;
}

typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

// raw loads of X(mn, kb..kb+3); kmax = last valid k (clamp for mn-major rows)
template <int KIND>
__device__ __forceinline__ void load4(const Lane& o, int kb, int kmax, float (&x)[4],
                                      float (&y)[4]) {
  if (KIND == OP_KC || KIND == OP_KC_R1) {
    const f4u a = *reinterpret_cast<const f4u*>(o.p + kb);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
    if (KIND == OP_KC_R1) {
      const f4u b = *reinterpret_cast<const f4u*>(o.s + kb);
      y[0] = b.x; y[1] = b.y; y[2] = b.z; y[3] = b.w;
    }
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = min(kb + c, kmax);
      x[c] = o.p[(long)k * o.ld];
      if (KIND == OP_MN_R1) y[c] = o.s[k];
    }
  }
}

template <int KIND>
__device__ __forceinline__ float fix1(const Lane& o, int k, int k_hi, float x, float y) {
  float val = x;
  if (KIND == OP_KC_R1 || KIND == OP_MN_R1) val = x > 0.f ? o.f * y : 0.f;
  val = o.valid ? val : (o.ones ? 1.f : 0.f);
  return k < k_hi ? val : 0.f;
}

}  // namespace oac
