// Epilogue of the register-direct and LDS-pipelined large-batch GEMMs
// (gemm_big.hip, gemm_fwd.hip): a wave owns a (32 WM) x (32 WN) block of
// v_mfma_f32_32x32x2_f32 accumulators at (mw, nw) and stores it straight from
// the accumulator registers.
//
// The epilogue kind is dispatched once per wave (not per element: a per-element
// switch compiled to a branch tree with exec-mask juggling around every store,
// ~33k cycles per 64x64 wave block -- as long as the whole K loop of a 128x128
// tile), and a block wholly inside M x N stores without bounds checks.  Per
// 32x32 block: every operand an element needs (bias, aux) is loaded before the
// first store, so the block waits one memory round trip, not one per element.
#pragma once
#include "oac_common.h"

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// element (m, n) of an accumulator register: lane l, register r of a 32x32 block
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Per-row sums over the 32 lanes of each half-wave of the 16 registers x[r]
// (register r = one row, lane = one column) as a transposed reduction: each
// xor step halves the registers a lane carries (16 -> 8 -> 4 -> 2 -> 1, then
// one last xor-1 step), 16 lane exchanges instead of 5 per register.  The
// pairs summed are the butterfly's (v_l + v_{l^16}, then + the xor-8 partner's
// partial, ...), so the sums equal a per-register xor butterfly bitwise.
// Returns the sum of register 8 b4 + 4 b3 + 2 b2 + b1 (b = lane bits).
__device__ __forceinline__ float rows_sum16(const float (&x)[16], int lane) {
  float a[8];
  const bool b4 = lane & 16, b3 = lane & 8, b2 = lane & 4, b1 = lane & 2;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float keep = b4 ? x[k + 8] : x[k], give = b4 ? x[k] : x[k + 8];
    a[k] = keep + __shfl_xor(give, 16, 32);
  }
  float b[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float keep = b3 ? a[k + 4] : a[k], give = b3 ? a[k] : a[k + 4];
    b[k] = keep + __shfl_xor(give, 8, 32);
  }
  float c[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float keep = b2 ? b[k + 2] : b[k], give = b2 ? b[k] : b[k + 2];
    c[k] = keep + __shfl_xor(give, 4, 32);
  }
  const float keep = b1 ? c[1] : c[0], give = b1 ? c[0] : c[1];
  const float d = keep + __shfl_xor(give, 2, 32);
  return d + __shfl_xor(d, 1, 32);
}

template <int WM, int WN, int EPI, bool FULL, bool WT = false>
__device__ __forceinline__ void epi_run(const GemmTask& t, int mw, int nw,
                                        const floatx16 (&acc)[WM][WN], bool second) {
  const int lane = threadIdx.x & 63;
  const int M = t.M, N = t.N;
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    // a 32-column block wholly past N stores nothing (its width-1 head
    // partial would land in the next partial column's slot)
    if (!FULL && nw + 32 * j >= N) continue;
    const int n = nw + 32 * j + (lane & 31);
    const bool nin = FULL || n < N;
    float bias = 0.f, w = 0.f;
    if (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_RANK_RELU || EPI == EPI_BIAS_RELU_DOT)
      bias = nin ? t.bias[n] : 0.f;
    if (EPI == EPI_BIAS_RELU_DOT) w = nin ? t.aux[n] : 0.f;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      if (!FULL && mw + 32 * i >= M) continue;
      const int mb = mw + 32 * i + 4 * (lane >> 5);   // row of register 0
      float aux[16];
      if (EPI == EPI_ADD_RELU || EPI == EPI_MASK) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mb + (r & 3) + 8 * (r >> 2);
          aux[r] = (FULL || (nin && m < M)) ? t.aux[(long)m * t.ld_aux + n] : 0.f;
        }
      }
      float dot[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + (r & 3) + 8 * (r >> 2);
        const bool in = FULL || (nin && m < M);
        const float v = acc[i][j][r];
        const long o = (long)m * t.ldc + n;
        if (EPI == EPI_BIAS_RELU_DOT) {
          const float h = fmaxf(v + bias, 0.f);
          if (in) t.C[o] = h;
          dot[r] = in ? h * w : 0.f;
          continue;
        }
        if (!in) continue;
        switch (EPI) {
          case EPI_STORE: t.C[o] = v; break;
          case EPI_GRAD:
            if (t.b_ones && n == N - 1) t.bias_grad[m] = v;
            else if (WT) __hip_atomic_store(t.C + o, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else t.C[o] = v;
            break;
          case EPI_BIAS: t.C[o] = v + bias; break;
          case EPI_BIAS_RELU: t.C[o] = fmaxf(v + bias, 0.f); break;
          case EPI_BIAS_RANK_RELU:   // pass 1: C = X W^T + b ; pass 2 (acc += U V^T): C2 = relu(. + b)
            if (!second) t.C[o] = v + bias;
            else t.C2[(long)m * t.ldc2 + n] = fmaxf(v + bias, 0.f);
            break;
          case EPI_ADD_RELU: t.C[o] = fmaxf(v + aux[r], 0.f); break;
          case EPI_MASK: t.C[o] = aux[r] > 0.f ? v : 0.f; break;
          default: break;
        }
      }
      if (EPI == EPI_BIAS_RELU_DOT) {
        // C = relu(acc + b) and, per row, the partial dot of this 32-column
        // block with aux[n] (the width-1 output layer on the hidden
        // activations), block-major partials C2[(n / 32) * ldc2 + m]
        const float s = rows_sum16(dot, lane);
        const int r = 8 * ((lane >> 4) & 1) + 4 * ((lane >> 3) & 1) + 2 * ((lane >> 2) & 1) +
                      ((lane >> 1) & 1);
        const int m = mb + (r & 3) + 8 * (r >> 2);
        if (!(lane & 1) && m < M) t.C2[(long)((nw + 32 * j) >> 5) * t.ldc2 + m] = s;
      }
    }
  }
}

template <int WM, int WN, int EPI, bool WT = false>
__device__ __forceinline__ void epi_dispatch(const GemmTask& t, int mw, int nw,
                                             const floatx16 (&acc)[WM][WN], bool second) {
  if (mw + 32 * WM <= t.M && nw + 32 * WN <= t.N)
    epi_run<WM, WN, EPI, true, WT>(t, mw, nw, acc, second);
  else
    epi_run<WM, WN, EPI, false, WT>(t, mw, nw, acc, second);
}

// KINDS: bit mask (1 << Epi) of the epilogue kinds a kernel instantiates
constexpr unsigned kEpiAll = 0xffu;
constexpr unsigned kEpiFwd = (1u << EPI_STORE) | (1u << EPI_BIAS) | (1u << EPI_BIAS_RELU) |
                             (1u << EPI_BIAS_RANK_RELU) | (1u << EPI_BIAS_RELU_DOT);

// WT: EPI_GRAD stores write-through (the last-arrival Adam's batches)
template <int WM, int WN, unsigned KINDS = kEpiAll, bool WT = false>
__device__ __forceinline__ void rd_epilogue(const GemmTask& t, int mw, int nw,
                                            const floatx16 (&acc)[WM][WN], bool second) {
#define OAC_EPI_CASE(E) \
  case E: if (KINDS & (1u << E)) epi_dispatch<WM, WN, E, WT>(t, mw, nw, acc, second); break;
  switch (t.epi) {
    OAC_EPI_CASE(EPI_STORE) OAC_EPI_CASE(EPI_GRAD) OAC_EPI_CASE(EPI_BIAS) OAC_EPI_CASE(EPI_BIAS_RELU)
    OAC_EPI_CASE(EPI_BIAS_RANK_RELU) OAC_EPI_CASE(EPI_ADD_RELU) OAC_EPI_CASE(EPI_MASK)
    OAC_EPI_CASE(EPI_BIAS_RELU_DOT)
    default: break;
  }
#undef OAC_EPI_CASE
}

}  // namespace oac
