// LDS-staged grouped fp32 GEMM for the large-batch stages (B >= 1024:
// BASELINE configs 2-4), gemm cfg 4.  One 256-thread workgroup (2 x 2
// waves) per TM x TN output tile; a wave owns a (TM/2) x (TN/2) block of
// 32x32 v_mfma_f32_32x32x2_f32 accumulators.
//
// Why not register-direct (gemm_big.hip): there every wave builds each MFMA
// operand from its own load plus per-element masking / rank-1 / bounds
// selects.  Here each KD-deep stage of a tile is loaded ONCE per workgroup
// with 16-byte loads (bounds, the dW ones column and the rank-1 seeds are
// resolved at load time), written k-major into LDS, and the inner loop is
// ds_read_b32 fragments + MFMAs only.  Double-buffered: the next stage's
// global loads are in flight while the current stage's MFMAs issue; one
// barrier per stage.
//
// Operand kinds (gemm_operand.h): k-contiguous (forward activations /
// weights, dX's dY) and mn-contiguous (batch-major dW operands, dX's W),
// each optionally a rank-1 seed s x v through a ReLU mask.  LDS rows are
// [k][mn] with a pad that keeps both the stores and the fragment reads
// bank-conflict free: +4 floats (16-byte rows, ds_write_b128) for
// mn-contiguous operands, +1 (ds_write_b32 transposes) for k-contiguous ones.
#include <cstdlib>

#include "oac_common.h"
#include "kernels.h"
#include "gemm_operand.h"
#include "adam_common.h"

namespace oac {

typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int KIND> struct LdsPad { static constexpr int v = (KIND == OP_KC || KIND == OP_KC_R1) ? 1 : 4; };

// One operand of a tile: X(mn, k), mn in [mn0, mn0 + T), k in a stage.
struct OpSrc {
  const float* p;      // data (rank-1: the ReLU mask)
  long ld;
  const float* s;      // rank-1: KC -> s[mn], MN -> s[k]
  const float* v;      // rank-1: KC -> v[k],  MN -> v[mn]
  int n_mn;            // valid mn (rows of A / columns of B)
  bool ones;           // column mn == n_mn is a virtual ones column (dW bias)
};

// A stage of one operand is T (mn) x KD (k) floats = P pieces of 8 per thread.
// mn-contiguous piece q: k = (t + 256 q) / (T/8), mn = 8 ((t + 256 q) % (T/8))
// k-contiguous piece q:  mn = (t + 256 q) / (KD/8), k = 8 ((t + 256 q) % (KD/8))
template <int KIND, int T, int KD>
struct Stage {
  static constexpr bool MN = (KIND == OP_MN || KIND == OP_MN_R1);
  static constexpr int P = T * KD / (256 * 8);
  static constexpr int ROW = T + LdsPad<KIND>::v;
  float x[P][8];
  float vpre[P][8];   // MN_R1: v[mn] of the piece's columns (stage-invariant)
  float spre[P];      // KC_R1: s[mn] of the piece's row (stage-invariant)

  __device__ __forceinline__ void init(const OpSrc& o, int mn0) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int e = threadIdx.x + 256 * q;
      if (KIND == OP_MN_R1) {
        const int c = mn0 + 8 * (e % (T / 8));
#pragma unroll
        for (int j = 0; j < 8; ++j) vpre[q][j] = c + j < o.n_mn ? o.v[c + j] : 0.f;
      }
      if (KIND == OP_KC_R1) {
        const int mn = mn0 + e / (KD / 8);
        spre[q] = mn < o.n_mn ? o.s[mn] : 0.f;
      }
    }
  }

  __device__ __forceinline__ void load(const OpSrc& o, int mn0, int k0, int k_hi) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int e = threadIdx.x + 256 * q;
      float* r = x[q];
      if (MN) {
        const int k = k0 + e / (T / 8), c = mn0 + 8 * (e % (T / 8));
        const bool in_k = k < k_hi;
        if (in_k && c + 8 <= o.n_mn) {
          const f4u a = *reinterpret_cast<const f4u*>(o.p + (long)k * o.ld + c);
          const f4u b = *reinterpret_cast<const f4u*>(o.p + (long)k * o.ld + c + 4);
          r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
          r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            r[j] = (in_k && c + j < o.n_mn) ? o.p[(long)k * o.ld + c + j] : 0.f;
        }
        if (KIND == OP_MN_R1) {   // s[k] v[mn] (mask > 0)
          const float sk = in_k ? o.s[k] : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) r[j] = r[j] > 0.f ? sk * vpre[q][j] : 0.f;
        }
        if (o.ones) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (c + j == o.n_mn) r[j] = in_k ? 1.f : 0.f;
        }
      } else {
        const int mn = mn0 + e / (KD / 8), k = k0 + 8 * (e % (KD / 8));
        const bool valid = mn < o.n_mn;
        const float* row = o.p + (long)(valid ? mn : 0) * o.ld;
        if (valid && k + 8 <= k_hi) {
          const f4u a = *reinterpret_cast<const f4u*>(row + k);
          const f4u b = *reinterpret_cast<const f4u*>(row + k + 4);
          r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
          r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) r[j] = (valid && k + j < k_hi) ? row[k + j] : 0.f;
        }
        if (KIND == OP_KC_R1) {   // s[mn] v[k] (mask > 0)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float vk = k + j < k_hi ? o.v[k + j] : 0.f;
            r[j] = r[j] > 0.f ? spre[q] * vk : 0.f;
          }
        }
      }
    }
  }

  __device__ __forceinline__ void store(float* lds) const {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int e = threadIdx.x + 256 * q;
      if (MN) {
        float4* d = reinterpret_cast<float4*>(lds + (e / (T / 8)) * ROW + 8 * (e % (T / 8)));
        d[0] = make_float4(x[q][0], x[q][1], x[q][2], x[q][3]);
        d[1] = make_float4(x[q][4], x[q][5], x[q][6], x[q][7]);
      } else {
        const int mn = e / (KD / 8), k = 8 * (e % (KD / 8));
#pragma unroll
        for (int j = 0; j < 8; ++j) lds[(k + j) * ROW + mn] = x[q][j];
      }
    }
  }
};

template <int TM, int TN, int KD>
struct LdsGeom {
  static constexpr int WM = TM / 64, WN = TN / 64;   // 32x32 accumulators per wave
  static constexpr int floats = 2 * KD * (TM + 4) + 2 * KD * (TN + 4);
};

// acc += A[m0.., k_lo..k_hi) . B[k_lo..k_hi), n0..] for the wave's block
template <int AK, int BK, int TM, int TN, int KD>
__device__ __forceinline__ void lds_loop(const OpSrc& a, const OpSrc& b, int m0, int n0, int k_lo,
                                         int k_hi, float* lds,
                                         floatx16 (&acc)[TM / 64][TN / 64]) {
  constexpr int WM = TM / 64, WN = TN / 64;
  using SA = Stage<AK, TM, KD>;
  using SB = Stage<BK, TN, KD>;
  constexpr int RA = SA::ROW, RB = SB::ROW;
  float* As[2] = {lds, lds + KD * RA};
  float* Bs[2] = {lds + 2 * KD * RA, lds + 2 * KD * RA + KD * RB};
  const int nst = (k_hi - k_lo + KD - 1) / KD;
  if (nst <= 0) return;
  const int lane = threadIdx.x & 63, l32 = lane & 31, half = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  SA sa;
  SB sb;
  sa.init(a, m0);
  sb.init(b, n0);
  sa.load(a, m0, k_lo, k_hi);
  sb.load(b, n0, k_lo, k_hi);
  sa.store(As[0]);
  sb.store(Bs[0]);
  __syncthreads();
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    const bool more = st + 1 < nst;
    if (more) {
      sa.load(a, m0, k_lo + (st + 1) * KD, k_hi);
      sb.load(b, n0, k_lo + (st + 1) * KD, k_hi);
    }
    const float* ap = As[cur] + half * RA + (TM / 2) * wm + l32;
    const float* bp = Bs[cur] + half * RB + (TN / 2) * wn + l32;
#pragma unroll
    for (int kk = 0; kk < KD / 2; ++kk) {
      float af[WM], bf[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i) af[i] = ap[2 * kk * RA + 32 * i];
#pragma unroll
      for (int j = 0; j < WN; ++j) bf[j] = bp[2 * kk * RB + 32 * j];
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      sa.store(As[cur ^ 1]);
      sb.store(Bs[cur ^ 1]);
    }
    __syncthreads();
  }
}

__device__ __forceinline__ int lacc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

__device__ __forceinline__ void lds_epilogue(const GemmTask& t, int mw, int nw, const floatx16& acc,
                                             bool second) {
  const int lane = threadIdx.x & 63;
  const int n = nw + (lane & 31);
  if (n >= t.N) return;
  float bias = 0.f;
  if (t.epi == EPI_BIAS || t.epi == EPI_BIAS_RELU || t.epi == EPI_BIAS_RANK_RELU) bias = t.bias[n];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = mw + lacc_row(r, lane);
    if (m >= t.M) continue;
    const float v = acc[r];
    const long o = (long)m * t.ldc + n;
    switch (t.epi) {
      case EPI_STORE: t.C[o] = v; break;
      case EPI_GRAD:
        if (t.b_ones && n == t.N - 1) t.bias_grad[m] = v;
        else t.C[o] = v;
        break;
      case EPI_BIAS: t.C[o] = v + bias; break;
      case EPI_BIAS_RELU: t.C[o] = fmaxf(v + bias, 0.f); break;
      case EPI_BIAS_RANK_RELU:   // pass 1: C = X W^T + b ; pass 2 (acc += U V^T): C2 = relu(. + b)
        if (!second) t.C[o] = v + bias;
        else t.C2[(long)m * t.ldc2 + n] = fmaxf(v + bias, 0.f);
        break;
      case EPI_ADD_RELU: t.C[o] = fmaxf(v + t.aux[(long)m * t.ld_aux + n], 0.f); break;
      case EPI_MASK: t.C[o] = t.aux[(long)m * t.ld_aux + n] > 0.f ? v : 0.f; break;
      default: break;
    }
  }
}

__device__ __forceinline__ OpSrc op_src(const float* p, long ld, const float* s, const float* v, int n,
                                        bool ones) {
  OpSrc o;
  o.p = p; o.ld = ld; o.s = s; o.v = v; o.n_mn = n; o.ones = ones;
  return o;
}

template <int TM, int TN, int KD>
__global__ void __launch_bounds__(256)
gemm_lds_kernel(int total_tiles, int tb1, int tb2, int tb3, int tb4, int tb5, int tb6, int tb7,
                const GemmBatch batch) {
  constexpr int WM = TM / 64, WN = TN / 64;
  __shared__ __attribute__((aligned(16))) float lds[LdsGeom<TM, TN, KD>::floats];
  const int bid = blockIdx.x;
  if (batch.publish && bid == 0 && threadIdx.x == 0)
    publish_step_consts(batch.publish, batch.pub_beta1, batch.pub_beta2);
  if (bid >= total_tiles) return;
  int ti = 0;   // task from the preloaded tile starts
  ti = bid >= tb1 ? 1 : ti; ti = bid >= tb2 ? 2 : ti; ti = bid >= tb3 ? 3 : ti;
  ti = bid >= tb4 ? 4 : ti; ti = bid >= tb5 ? 5 : ti; ti = bid >= tb6 ? 6 : ti;
  ti = bid >= tb7 ? 7 : ti;
  ti = __builtin_amdgcn_readfirstlane(ti);
  GemmTask t = batch.t[ti];
  int local = bid - t.tile_begin;
  int k_lo = 0, k_hi = t.K;
  if (t.ksplit > 1) {
    const int split = local % t.ksplit;
    local /= t.ksplit;
    k_lo = split * t.kchunk;
    k_hi = min(t.K, k_lo + t.kchunk);
    t.C += (long)split * t.slab_stride;
    t.bias_grad += (long)split * t.slab_stride;
  }
  const int m0 = (local / t.tiles_n) * TM;
  const int n0 = (local % t.tiles_n) * TN;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mw = m0 + (wave >> 1) * (TM / 2), nw = n0 + (wave & 1) * (TN / 2);
  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const bool ones = t.b_ones != 0;
  const int nl = ones ? t.N - 1 : t.N;
  const bool r1 = t.a_mode != A_PLAIN;
  const OpSrc a = op_src(r1 ? t.a_mask : t.A, r1 ? t.ld_mask : t.lda, t.a_s, t.a_v, t.M, false);
  const OpSrc b = op_src(t.B, t.ldb, nullptr, nullptr, nl, ones);
  if (t.a_kc && t.b_kc)   lds_loop<OP_KC, OP_KC, TM, TN, KD>(a, b, m0, n0, k_lo, k_hi, lds, acc);     // forward
  else if (t.a_kc && !r1) lds_loop<OP_KC, OP_MN, TM, TN, KD>(a, b, m0, n0, k_lo, k_hi, lds, acc);     // dX
  else if (t.a_kc)        lds_loop<OP_KC_R1, OP_MN, TM, TN, KD>(a, b, m0, n0, k_lo, k_hi, lds, acc);  // dX, rank-1
  else if (!r1)           lds_loop<OP_MN, OP_MN, TM, TN, KD>(a, b, m0, n0, k_lo, k_hi, lds, acc);     // dW
  else                    lds_loop<OP_MN_R1, OP_MN, TM, TN, KD>(a, b, m0, n0, k_lo, k_hi, lds, acc);  // dW, rank-1
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) lds_epilogue(t, mw + 32 * i, nw + 32 * j, acc[i][j], false);
  if (t.epi == EPI_BIAS_RANK_RELU) {
    // + U V^T on the same accumulators: as a continuation of the row along k
    // (the batch actions follow the observations in a replay row, the action
    // columns follow the observation columns in W0) or from a separate
    // rank-R operand (the policy's a~ against W0's action columns)
    const OpSrc vb = op_src(t.B, t.ldb, nullptr, nullptr, t.N, false);
    if (t.U == t.A + t.K && t.ldu == t.lda && t.V == t.B + t.K && t.ldv == t.ldb)
      lds_loop<OP_KC, OP_KC, TM, TN, KD>(a, vb, m0, n0, t.K, t.K + t.R, lds, acc);
    else
      lds_loop<OP_KC, OP_KC, TM, TN, KD>(op_src(t.U, t.ldu, nullptr, nullptr, t.M, false),
                                         op_src(t.V, t.ldv, nullptr, nullptr, t.N, false), m0, n0,
                                         0, t.R, lds, acc);
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) lds_epilogue(t, mw + 32 * i, nw + 32 * j, acc[i][j], true);
  }
}

// tile variant (OAC_LDS_GEOM: 0 = 64x64 KD 32, 1 = 128x64 KD 32, 2 = 64x64 KD 64,
// 3 = 64x128 KD 32); the plan's tile geometry follows it
static int lds_geom() {
  static const int v = [] { const char* e = getenv("OAC_LDS_GEOM"); return e ? atoi(e) : 0; }();
  return v;
}
int gemm_lds_tile_m() { const int g = lds_geom(); return g == 1 ? 128 : 64; }
int gemm_lds_tile_n() { const int g = lds_geom(); return g == 3 ? 128 : 64; }
static int lds_kd() { return lds_geom() == 2 ? 64 : 32; }

bool gemm_lds_supports(const GemmBatch& b) {
  if (b.fuse_adam) return false;
  for (int i = 0; i < b.ntasks; ++i) {
    const GemmTask& t = b.t[i];
    if (t.K2 > 0 || t.epi == EPI_HEAD_BWD || t.epi == EPI_BIAS_RELU_DOT) return false;
    if (t.b_kc && !t.a_kc) return false;                      // no such product on the step
    if (t.b_kc && t.a_mode != A_PLAIN) return false;
    if (t.ksplit > 1 && t.kchunk % lds_kd()) return false;
    if (t.epi == EPI_BIAS_RANK_RELU && (!t.C2 || t.ksplit > 1)) return false;
  }
  return true;
}

hipError_t gemm_lds_launch(const GemmBatch& b, hipStream_t s) {
  if (b.total_tiles <= 0) return hipSuccess;
  if (!gemm_lds_supports(b)) return hipErrorInvalidValue;
  int tb[8];
  for (int i = 0; i < 8; ++i) tb[i] = i < b.ntasks ? b.t[i].tile_begin : 0x7fffffff;
#define OAC_LDSK(TM_, TN_, KD_)                                                                     \
  OAC_LAUNCH((gemm_lds_kernel<TM_, TN_, KD_>), dim3(b.total_tiles), dim3(256), 0, s, b.total_tiles, \
             tb[1], tb[2], tb[3], tb[4], tb[5], tb[6], tb[7], b)
  switch (lds_geom()) {
    case 1: OAC_LDSK(128, 64, 32); break;
    case 2: OAC_LDSK(64, 64, 64); break;
    case 3: OAC_LDSK(64, 128, 32); break;
    default: OAC_LDSK(64, 64, 32); break;
  }
#undef OAC_LDSK
  return hipGetLastError();
}

}  // namespace oac
