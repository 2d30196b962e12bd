// OAC exploration action with the weight stream of ONE observation spread over
// a group of G workgroups (get_optimistic_exploration_action,
// /root/reference/optimistic_exploration.py:14-109): twin critics, or one K-head critic with mean + beta std or the trainer_UB
// sorted head).
//
// Two kernels: oac_expl_twin_kernel (further down) takes twin critics -- the
// SAC / OAC trainers' exploration -- with one polled hand-off and one
// last-arrival; oac_expl_split_kernel below takes every call (the K-head
// critic of share_layers, dims past the twin kernel's budget) with four.
//
// The round-1 kernel (one workgroup per observation, tools/micro/retired/
// expl_fused.hip) streamed the row's 2.7 MB of weights (Humanoid dims) through
// one CU at 45-110 GB/s per layer: ~59 us of a ~100 us call.  Here the
// matrix-vector products are cut by rows (or, for the transposed product of
// the backward, by columns) over the group, and the group meets at four
// in-launch hand-offs (every spin bounded):
//   S1  policy layer 0 rows + both critics' obs projections P_i = W0_i[:, :Do] ob + b0_i
//   S2  policy layer 1 rows
//   S3  (every workgroup) heads -> mean, std, a = tanh(mean); critic layer 0
//       h1_i = relu(P_i + W0_i[:, Do:] a) for all rows; then its rows of critic layer 1
//   S4  (every workgroup) Q, the Q_UB seeds and dh2 = seed . W_last (x) 1[h2 > 0];
//       then, per fixed column part it owns, those columns of dh1 = (dh2 W1)
//       (x) 1[h1 > 0] and their partial of da = dh1 . W0[:, Do:]
//   S5  (workgroup 0 of the group) da = the parts' partials in order, grad,
//       shift, sample.
// Hand-off forms (MI355X_MICROARCH.md, "Valid forms"):
//   WT    one workgroup per CU (84 KB of static LDS admits no second one):
//         write-through (sc1) stores of the published vectors, every storing
//         wave's vmcnt(0), a barrier, lane 0's agent-scope counter add; the
//         consumer polls with sc1 loads, meets at a barrier and reads the
//         vectors with sc1 loads -- no cache write-back or invalidate (~2 us less
//         per hand-off than the fences);
//   FENCE plain stores, lane-0 agent release before the add, agent acquire after
//         the poll: any number of workgroups per CU (large batches).
// G = 1 (batches of >= 256 observations) needs no hand-off at all.
// Every product's reduction order is a function of the row / column alone (one
// wave per row, lanes along k; dh1 by fixed row parts added in order; da one
// wave per output), never of G or of the observations per launch, so a row of a
// batched call is bitwise the row of a single-observation call.
#include "oac_common.h"
#include "kernels.h"

namespace oac {

#ifdef OAC_EXPL_CLOCK   // tools/micro/expl_micro: stage wall clocks (100 MHz) of the group's first and last workgroup
__device__ long long g_expl_clock[64];
#define EXPL_CLK(i) do { if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == (unsigned)G - 1)) \
    g_expl_clock[(blockIdx.x == 0 ? 0 : 32) + (i)] = wall_clock64(); } while (0)
#else
#define EXPL_CLK(i) do {} while (0)
#endif

// Sum over the 64 lanes of a wave, in every lane: DPP adds within each row of
// 16 lanes (pairs, quads, mirrored halves, mirrored rows), then the four row
// sums read out in lane order -- a fixed order, and no LDS-crossbar round
// trip per step (the xor butterfly's ds_bpermute took ~6 of them).
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wsum64(float v) {
  v = dpp_add<0xB1>(v);    // quad_perm [1,0,3,2]
  v = dpp_add<0x4E>(v);    // quad_perm [2,3,0,1]
  v = dpp_add<0x141>(v);   // row_half_mirror
  v = dpp_add<0x140>(v);   // row_mirror
  const int vi = __float_as_int(v);   // (the builtin is int-typed: move bits, not values)
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(vi, 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(vi, 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(vi, 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(vi, 48));
  return (r0 + r1) + (r2 + r3);
}

// one output of a single-observation call as a tagged granule (ExplFusedArgs::tags)
__device__ __forceinline__ void put_tagged(unsigned long long* g, float v, unsigned tag) {
  const unsigned long long w = (unsigned long long)__float_as_uint(v) | ((unsigned long long)tag << 32);
  __hip_atomic_store(g, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// published-vector traffic of the group (global scratch)
template <bool WT>
__device__ __forceinline__ void st_pub(float* p, float v) {
  if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <bool WT>
__device__ __forceinline__ float ld_pub(const float* p) {
  if constexpr (WT)
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// The first pass of a wave's rows (its first RW rows, k < 64 U) and their
// bias, loaded ahead -- during the hand-off before the stage -- by rows_pre
// and used by rows_matvec in place of those loads (the same values, the same
// order: the result is bitwise the same).
constexpr int kRW = 4, kRU = 4;
struct RowsPre { float wv[kRW][kRU]; float b; };
__device__ __forceinline__ void rows_pre(const float* __restrict__ W, long ldw,
                                         const float* __restrict__ b, int K, int n_lo, int n_hi,
                                         RowsPre& p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = n_lo + wave * kRW;
  if (n0 >= n_hi) return;
#pragma unroll
  for (int u = 0; u < kRU; ++u) {
    const int k = u * 64 + lane, kc = k < K ? k : K - 1;
#pragma unroll
    for (int r = 0; r < kRW; ++r) p.wv[r][u] = W[(long)min(n0 + r, n_hi - 1) * ldw + kc];
  }
  p.b = b ? b[min(n0 + (lane < kRW ? lane : 0), n_hi - 1)] : 0.f;
}

// y[n] = act(W[n, :K] . x + b[n]) for n in [n_lo, n_hi): one wave per row,
// RW rows of loads in flight, lanes along k (fixed-order butterfly sum).
// PUB: y is a published vector (global), else LDS.  pre: the wave's first
// pass, loaded ahead (rows_pre), or null.  wave0: the wave that takes the
// first rows (a second product placed on the waves the first left idle).
template <bool PUB, bool WT>
__device__ __forceinline__ void rows_matvec(const float* __restrict__ W, long ldw,
                                            const float* __restrict__ b, const float* x, int K,
                                            int n_lo, int n_hi, float* y, bool relu,
                                            const RowsPre* pre = nullptr, int wave0 = 0) {
  constexpr int RW = kRW, U = kRU;
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int wave = ((threadIdx.x >> 6) - wave0 % nw + nw) % nw;
  // (read up front: a select between pre's and W's addresses would keep pre in memory)
  float pw[RW][U], pb = 0.f;
  if (pre) {
    pb = pre->b;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RW; ++r) pw[r][u] = pre->wv[r][u];
  }
  for (int n0 = n_lo + wave * RW; n0 < n_hi; n0 += nw * RW) {
    const bool first = pre && n0 == n_lo + wave * RW;
    float acc[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[r] = 0.f;
    for (int kb = 0; kb < K; kb += 64 * U) {
      float wv[RW][U], xv[U];
      if (first && kb == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < RW; ++r) wv[r][u] = pw[r][u];
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int kc = min(kb + u * 64 + lane, K - 1);
#pragma unroll
          for (int r = 0; r < RW; ++r) wv[r][u] = W[(long)min(n0 + r, n_hi - 1) * ldw + kc];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = kb + u * 64 + lane;
        xv[u] = k < K ? x[k < K ? k : K - 1] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RW; ++r) acc[r] = fmaf(wv[r][u], xv[u], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[r] = wsum64(acc[r]);
    if (lane < RW && n0 + lane < n_hi) {
      float v = acc[0];
#pragma unroll
      for (int r = 1; r < RW; ++r) v = lane == r ? acc[r] : v;
      v += first ? pb : (b ? b[n0 + lane] : 0.f);
      v = relu ? fmaxf(v, 0.f) : v;
      if constexpr (PUB) st_pub<WT>(y + n0 + lane, v);
      else y[n0 + lane] = v;
    }
  }
}

// The group's hand-off, in two halves so that the next stage's weight loads
// can be issued between them (their round trips then overlap the group's
// arrival skew and the poll).  group_arrive: every storing wave drains its
// stores, the workgroup meets, the last wave's lane 0 arrives on the stage
// counter (FENCE: behind an agent release).  group_wait: that lane polls the
// counter (relaxed, bounded) until all G workgroups arrived (FENCE: then
// acquires), and the workgroup meets again.  G = 1: the workgroup's own
// barriers order its scratch.  The last wave issues no loads ahead.
template <bool WT>
__device__ __forceinline__ void group_arrive(unsigned* ctr, unsigned target) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // (the polling wave arrives too: a wave with the add in flight waits for it
  // before its next loads)
  if (target > 1 && threadIdx.x == blockDim.x - 64) {
    if constexpr (!WT) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
template <bool WT>
__device__ __forceinline__ bool group_wait(unsigned* ctr, unsigned target) {
  __shared__ int ok_s;
  if (target <= 1) {
    __syncthreads();
    return true;
  }
  if (threadIdx.x == blockDim.x - 64) {   // (vmcnt is in order: a poll behind loads
    int ok = 1;                            // ahead would wait for them)
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 25)) { ok = 0; break; }   // ~0.3 s: a stuck group gives up
    }
    if constexpr (!WT) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    ok_s = ok;
  }
  __syncthreads();
  return ok_s != 0;
}
template <bool WT>
__device__ __forceinline__ bool group_sync(unsigned* ctr, unsigned target) {
  group_arrive<WT>(ctr, target);
  return group_wait<WT>(ctr, target);
}

// the dh1 columns are cut into kExplParts fixed parts (never by the group
// size): part p's partial of da is published, and S5 adds the parts in order
constexpr int kExplParts = 32;
// the twin-critic kernel's fixed parts (oac_expl_twin_kernel below)
constexpr int kTwinParts = 32;
// per-observation scratch (floats) in the workspace, the larger of the two
// kernels' layouts: here vectors [8H] | da partials [kExplParts][64] | 4
// counters; the twin kernel's [2][kTwinParts][H] partials | [2H] | [64] | counters
__host__ __device__ inline long expl_split_scratch(int H) {
  const long split = 8L * H + kExplParts * 64L + 64;
  const long twin = 2L * kTwinParts * H + 2L * H + 128;
  return split > twin ? split : twin;
}
// LDS floats: x | v1 [2H] | v2 [2H] | head [64] | misc [128] | partials [threads] |
// a part's dh1 columns | their da products
__host__ __device__ inline long expl_split_lds(int Do, int Da, int H, int threads) {
  // the dh1 columns of one workgroup (G = 1: all 2H) and a part's da products
  const long w = (2L * H + kExplParts - 1) / kExplParts;
  return ((Do + Da + 3) & ~3L) + 4L * H + 64 + 128 + threads + (2L * H + 32) + w * 64;
}
constexpr int kWtLdsFloats = 21 * 1024;   // 84 KB: one workgroup per CU
// OBS: the (single) observation is the argument `oa` (launch_expl_split_obs)
template <bool WT, bool OBS>
__global__ void __launch_bounds__(1024) oac_expl_split_kernel(ExplFusedArgs a, int row0, int G,
                                                              float* scratch, ExplObsArg oa) {
  float* sm;
  if constexpr (WT) {
    __shared__ __attribute__((aligned(16))) float sm_wt[kWtLdsFloats];
    sm = sm_wt;
  } else {
    extern __shared__ __attribute__((aligned(16))) float sm_dyn[];
    sm = sm_dyn;
  }
  const int Do = a.Do, Da = a.Da, H = a.H, Dq = Do + Da;
  const int gi = blockIdx.x / G, wg = blockIdx.x - gi * G;
  const int r = row0 + gi, t = threadIdx.x, nt = blockDim.x;
  const int nq = a.nq, KQ = a.K;
  // the critics' parameter blocks in registers: a.q[i] with i per lane would be
  // a vector load from the argument segment (and a wait) per use
  const float* const q0p = a.q[0];
  const float* const q1p = a.q[1];
  auto Qp = [&](int i) { return i == 0 ? q0p : q1p; };
  float* Gv = scratch + (long)gi * expl_split_scratch(H);   // group's published vectors
  float* g_h1p = Gv;            // [H]   policy layer 0
  float* g_P = Gv + H;          // [2H]  critics' obs projections (+ b0)
  float* g_h2p = Gv + 3 * H;    // [H]   policy layer 1
  float* g_qh2 = Gv + 4 * H;    // [2H]  critic layer 1
  float* g_dap = Gv + 6 * H + 2 * H;   // [kExplParts][64] da partials
  unsigned* ctr = reinterpret_cast<unsigned*>(g_dap + kExplParts * 64);   // [4] stage counters
  float* x = sm;                           // [Do + Da] ob | a
  float* v1 = x + ((Dq + 3) & ~3);         // [2H] scratch vectors
  float* v2 = v1 + 2 * H;                  // [2H]
  float* head = v2 + 2 * H;                // [64] mean | raw log std
  float* misc = head + 64;                 // [128] q, seeds, norm, K heads, reductions
  float* qk = misc + 16;                   // [16] K head values
  float* wk = qk + 16;                     // [16] K head seeds
  float* red = misc + 64;                  // [64]
  float* prt = misc + 128;                 // [threads] dh1 partials
  __shared__ long long cnt_s;
  if (t == 0) cnt_s = a.state->expl_counter;
  // rows of a length-L product owned by this workgroup
  auto part = [&](int L, int& lo, int& hi) {
    const int per = (L + G - 1) / G;
    lo = min(L, wg * per);
    hi = min(L, lo + per);
  };
  // the part [l, h) of rows [b0, b0 + L) within the range [lo, hi)
  auto clip = [](int lo, int hi, int b0, int L, int& l, int& h) {
    l = max(lo, b0) - b0;
    h = min(hi, b0 + L) - b0;
  };
  int lo1, hi1, lo2, hi2, lo3, hi3;
  part((1 + nq) * H, lo1, hi1);
  part(H, lo2, hi2);
  part(nq * H, lo3, hi3);
  const int e01 = min(hi1, H);   // S1 policy rows [lo1, e01)
  // S2's and S4's first weight loads are issued ahead, during the hand-off
  // before the stage (the group's arrival skew and the poll), into registers:
  // the stage then starts on its published inputs' round trip alone.  (S3's
  // -- heads, W0_i[:, Do:], its layer-1 rows, ~47 loads per wave -- made
  // hand-off 1 longer by more than they saved.)
  RowsPre pre;
  EXPL_CLK(0);
  if constexpr (OBS) {
    for (int k = t; k < Do; k += nt) x[k] = oa.v[k];
  } else {
    for (int k = t; k < Do; k += nt) x[k] = a.obs[(long)r * a.ld_obs + k];
  }
  __syncthreads();
  EXPL_CLK(1);
  // ---- S1: policy layer 0 | critic obs projections (3H or 2H rows)
  if (lo1 < e01)
    rows_matvec<true, WT>(a.pol + a.p_fc0_w, Do, a.pol + a.p_fc0_b, x, Do, lo1, e01, g_h1p, true);
  for (int i = 0; i < nq; ++i) {
    int l, h;
    clip(lo1, hi1, (1 + i) * H, H, l, h);
    if (l < h) {
      const float* q = Qp(i);
      rows_matvec<true, WT>(q + a.q_fc0_w, Dq, q + a.q_fc0_b, x, Do, l, h, g_P + i * H, false);
    }
  }
  EXPL_CLK(2);
  group_arrive<WT>(ctr + 0, G);
  if (lo2 < hi2) rows_pre(a.pol + a.p_fc1_w, H, a.pol + a.p_fc1_b, H, lo2, hi2, pre);
  bool ok = group_wait<WT>(ctr + 0, G);
  EXPL_CLK(3);
  // ---- S2: policy layer 1 rows
  for (int k = t; k < H; k += nt) v1[k] = ld_pub<WT>(g_h1p + k);
  __syncthreads();
  if (lo2 < hi2)
    rows_matvec<true, WT>(a.pol + a.p_fc1_w, H, a.pol + a.p_fc1_b, v1, H, lo2, hi2, g_h2p, true, &pre);
  EXPL_CLK(4);
  ok = group_sync<WT>(ctr + 1, G) && ok;
  EXPL_CLK(5);
  // ---- S3: heads (every workgroup), a = tanh(mean), critic layer 0, its layer-1 rows
  // (the published h2 and P_i: one round of loads)
  for (int k = t; k < H; k += nt) v1[k] = ld_pub<WT>(g_h2p + k);
  for (int e = t; e < nq * H; e += nt) v2[e] = ld_pub<WT>(g_P + e);
  __syncthreads();
  rows_matvec<false, WT>(a.pol + a.p_head_w, H, a.pol + a.p_head_b, v1, H, 0, 2 * Da, head, false);
  __syncthreads();
  if (t < Da) x[Do + t] = tanhf(head[t]);
  __syncthreads();
  EXPL_CLK(6);
  for (int e = t; e < nq * H; e += nt) {   // h1_i = relu(P_i + W0_i[:, Do:] a)
    const int i = e / H, n = e - i * H;
    const float* w = Qp(i) + a.q_fc0_w + (long)n * Dq + Do;
    float s = v2[e];
    for (int j = 0; j < Da; ++j) s = fmaf(w[j], x[Do + j], s);
    v2[e] = fmaxf(s, 0.f);
  }
  __syncthreads();
  for (int i = 0; i < nq; ++i) {
    int l, h;
    clip(lo3, hi3, i * H, H, l, h);
    if (l < h) {
      const float* q = Qp(i);
      rows_matvec<true, WT>(q + a.q_fc1_w, H, q + a.q_fc1_b, v2 + i * H, H, l, h, g_qh2 + i * H, true);
    }
  }
  EXPL_CLK(7);
  // S4 ahead: the last layers (Q dot: waves 0 and 1; dh2: this thread's
  // element), the first column block's rows of W1 and the first part's
  // (column, j) elements of W0_i[:, Do:]
  const int R4 = nq * H, c4 = t & 31, pp4 = t >> 5, np4 = nt >> 5;
  const int rows4 = (H + np4 - 1) / np4;
  // this workgroup's parts are contiguous, p0 .. p1 - 1 (a function of G,
  // but each part's partial is not)
  const int p0 = wg * kExplParts / G, p1 = (wg + 1) * kExplParts / G;
  const int lo4 = p0 * R4 / kExplParts, hi4 = p1 * R4 / kExplParts;
  const bool pre_q = nq == 2 && H <= 64 * kRU && R4 <= nt;
  const bool pre_c = rows4 <= 16 && t < nt - 64;   // (per thread: not the polling wave)
  float wq[kRU], qb = 0.f, wd = 0.f, w1[16], wda = 0.f;
  group_arrive<WT>(ctr + 2, G);
  if (pre_q) {
    const int wave = t >> 6, lane = t & 63;
    if (wave < 2) {
      const float* q = Qp(wave);
#pragma unroll
      for (int u = 0; u < kRU; ++u) wq[u] = q[a.q_last_w + min(lane + 64 * u, H - 1)];
      qb = q[a.q_last_b];
    }
    if (t < R4) {
      const int i = t / H;
      wd = Qp(i)[a.q_last_w + (t - i * H)];
    }
  }
  const int e = lo4 + c4;
  if (pre_c && e < hi4) {
    const int i = e / H, k = e - i * H;
    const float* W1 = Qp(i) + a.q_fc1_w + k;
    const int n_lo = min(H, pp4 * rows4), n_hi = min(H, n_lo + rows4);
#pragma unroll
    for (int u = 0; u < 16; ++u) w1[u] = W1[(long)max(0, min(n_lo + u, n_hi - 1)) * H];
  }
  const int plo = p0 * R4 / kExplParts, phi = (p0 + 1) * R4 / kExplParts;
  if (p0 < p1 && t < (phi - plo) * Da) {
    const int cl = t / Da, j = t - cl * Da, col = plo + cl;
    const int i = col / H, k = col - i * H;
    wda = Qp(i)[a.q_fc0_w + (long)k * Dq + Do + j];
  }
  ok = group_wait<WT>(ctr + 2, G) && ok;
  EXPL_CLK(8);
  // ---- S4: Q, seeds, dh2 (every workgroup), then its columns of dh1
  for (int e = t; e < nq * H; e += nt) v1[e] = ld_pub<WT>(g_qh2 + e);
  __syncthreads();
  if (nq == 2) {
    const int wave = t >> 6, lane = t & 63;
    if (wave < 2) {
      const float* q = Qp(wave);
      float s = 0.f;
      if (pre_q) {
#pragma unroll
        for (int u = 0; u < kRU; ++u)
          if (lane + 64 * u < H) s = fmaf(wq[u], v1[wave * H + lane + 64 * u], s);
      } else {
        for (int k = lane; k < H; k += 64) s = fmaf(q[a.q_last_w + k], v1[wave * H + k], s);
      }
      s = wsum64(s);
      if (lane == 0) misc[wave] = s + (pre_q ? qb : q[a.q_last_b]);
    }
  } else {
    rows_matvec<false, WT>(Qp(0) + a.q_last_w, H, Qp(0) + a.q_last_b, v1, H, 0, KQ, qk, false);
  }
  __syncthreads();
  if (t == 0) {
    if (nq == 2) {   // Q_UB = (Q1+Q2)/2 + beta |Q1-Q2|/2: d|x|/dx = sign(x) (0 at 0)
      const float d = misc[0] - misc[1];
      const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      const float hb = a.beta_UB / 2.f;
      misc[2] = 0.5f + hb * sg;
      misc[3] = 0.5f - hb * sg;
    } else if (a.ub_index >= 0) {   // trainer_UB: the head ranked ub_index (ties: lower index)
      for (int k = 0; k < KQ; ++k) {
        int rank = 0;
        for (int j = 0; j < KQ; ++j) rank += (qk[j] < qk[k]) || (qk[j] == qk[k] && j < k);
        wk[k] = rank == a.ub_index ? 1.f : 0.f;
      }
    } else {         // mean_k + beta std_k (unbiased)
      float s = 0.f;
      for (int k = 0; k < KQ; ++k) s += qk[k];
      const float mu = s / (float)KQ;
      float ss = 0.f;
      for (int k = 0; k < KQ; ++k) ss += (qk[k] - mu) * (qk[k] - mu);
      const float sd = sqrtf(ss / (float)(KQ - 1));
      for (int k = 0; k < KQ; ++k)
        wk[k] = 1.f / (float)KQ + a.beta_UB * ((qk[k] - mu) / ((float)(KQ - 1) * sd));
    }
  }
  __syncthreads();
  if (pre_q) {   // dh2 (in v1)
    const int i = t / H;
    if (t < R4) v1[t] = v1[t] > 0.f ? misc[2 + i] * wd : 0.f;
  } else {
    for (int e = t; e < R4; e += nt) {
      const int i = e / H, n = e - i * H;
      float sv;
      if (nq == 2) {
        sv = misc[2 + i] * Qp(i)[a.q_last_w + n];
      } else {
        sv = 0.f;
        for (int k = 0; k < KQ; ++k) sv = fmaf(wk[k], Qp(0)[a.q_last_w + (long)k * H + n], sv);
      }
      v1[e] = v1[e] > 0.f ? sv : 0.f;
    }
  }
  __syncthreads();
  {   // dh1_i[k] = 1[h1_i[k] > 0] sum_n dh2_i[n] W1_i[n, k] over the columns of the
      // fixed parts this workgroup owns, 32 columns at a time, the rows cut into
      // threads/32 parts (thread: column c, part pp; coalesced along the columns),
      // the parts added in order; then the part's partial of da = dh1 . W0[:, Do:]
      // (its columns in order), published for S5
    float* dcol = prt + nt;   // [R / G + 32] dh1 of this workgroup's columns
    float* prod = dcol + (2 * H + G - 1) / G + 32;   // [part width][Da]
    for (int cb = lo4; cb < hi4; cb += 32) {
      const int e = cb + c4;
      float s = 0.f;
      if (e < hi4) {
        const int i = e / H, k = e - i * H;
        const float* W1 = Qp(i) + a.q_fc1_w + k;
        const float* g = v1 + i * H;
        const int n_lo = min(H, pp4 * rows4), n_hi = min(H, n_lo + rows4);
        for (int n0 = n_lo; n0 < n_hi; n0 += 16) {
          float w[16];
          if (pre_c && cb == lo4) {
#pragma unroll
            for (int u = 0; u < 16; ++u) w[u] = w1[u];
          } else {
#pragma unroll
            for (int u = 0; u < 16; ++u) w[u] = W1[(long)min(n0 + u, n_hi - 1) * H];
          }
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (n0 + u < n_hi) s = fmaf(g[n0 + u], w[u], s);
        }
      }
      prt[pp4 * 32 + c4] = s;
      __syncthreads();
      if (t < 32 && cb + t < hi4) {
        float v = prt[t];
        for (int q = 1; q < np4; ++q) v += prt[q * 32 + t];
        dcol[cb - lo4 + t] = v2[cb + t] > 0.f ? v : 0.f;
      }
      __syncthreads();
    }
    for (int pq = p0; pq < p1; ++pq) {
      // the part's da partial: every (column, j) product in one round of loads
      // (thread e = column * Da + j), then its columns in order
      const int plo = pq * R4 / kExplParts, phi = (pq + 1) * R4 / kExplParts;
      for (int e = t; e < (phi - plo) * Da; e += nt) {
        const int cl = e / Da, j = e - cl * Da, col = plo + cl;
        const int i = col / H, k = col - i * H;
        const float w = pq == p0 && e == t ? wda : Qp(i)[a.q_fc0_w + (long)k * Dq + Do + j];
        prod[e] = dcol[col - lo4] * w;
      }
      __syncthreads();
      if (t < Da) {
        float s = 0.f;
        for (int cl = 0; cl < phi - plo; ++cl) s += prod[cl * Da + t];
        st_pub<WT>(g_dap + pq * 64 + t, s);
      }
      __syncthreads();
    }
  }
  EXPL_CLK(9);
  if (wg != 0) {   // the group's other workgroups only publish (their arrival is the signal)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      if constexpr (!WT) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_fetch_add(ctr + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  ok = group_sync<WT>(ctr + 3, G) && ok;
  EXPL_CLK(10);
  // ---- S5 (workgroup 0): da = the parts' partials in order, grad, shift, sample
  float da = 0.f;
  if (t < Da) {
    float dp[kExplParts];   // every part's load in flight before the first add
#pragma unroll
    for (int q = 0; q < kExplParts; ++q) dp[q] = ld_pub<WT>(g_dap + q * 64 + t);
#pragma unroll
    for (int q = 0; q < kExplParts; ++q) da += dp[q];
  }
  EXPL_CLK(11);
  float g = 0.f, sig = 0.f, sd = 0.f, mean = 0.f;
  if (t < Da) {
    const float act = x[Do + t];
    g = da * (1.f - act * act);
    sd = expf(fminf(fmaxf(head[Da + t], -20.f), 2.f));
    sig = sd * sd;
    mean = head[t];
    red[t] = g * g * sig;
  }
  __syncthreads();
  if (t == 0) {
    float s = 0.f;
    for (int i = 0; i < Da; ++i) s += red[i];
    misc[4] = sqrtf(s) + 10e-6f;
    if (G > 1)   // every member is past its last hand-off
      for (int c = 0; c < 4; ++c) __hip_atomic_store(ctr + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (a.n == 1 && a.tags) {   // tagged granules (ExplFusedArgs::tags): no drain, no word
    unsigned tag = a.done_seq | (ok ? 0u : 0x80000000u);
    if (t < Da) {
      const float mu_C = (a.sqrt_2delta * (sig * g)) / misc[4];
      const float mu_E = mean + mu_C;
      const float ev = a.eps ? a.eps[t] : philox_normal(a.seed, (unsigned long long)cnt_s, 3u, (unsigned)t);
      const float nan = __int_as_float(0x7fc00000);
      put_tagged(a.tags + t, ok ? tanhf(__fadd_rn(__fmul_rn(ev, sd), mu_E)) : nan, tag);
      put_tagged(a.tags + Da + t, ok ? mu_E : nan, tag);
      put_tagged(a.tags + 2 * Da + t, sd, tag);
      if (a.grad) a.grad[t] = g;
    }
    if (t == 0) {
      if (!a.eps) a.state->expl_counter = cnt_s + 1;
      if (!ok && a.fail) __hip_atomic_store(a.fail, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (t < Da) {
    const long e = (long)r * Da + t;
    const float mu_C = (a.sqrt_2delta * (sig * g)) / misc[4];
    const float mu_E = mean + mu_C;
    const float ev = a.eps ? a.eps[e]
                           : philox_normal(a.seed, (unsigned long long)cnt_s, 3u, (unsigned)(r * Da + t));
    const long nd = (long)a.n * Da;
    // a stuck hand-off (ok == false) leaves NaNs, never silently wrong values
    const float nan = __int_as_float(0x7fc00000);
    a.out[e] = ok ? tanhf(__fadd_rn(__fmul_rn(ev, sd), mu_E)) : nan;
    a.out[nd + e] = ok ? mu_E : nan;
    a.out[2 * nd + e] = sd;
    if (a.grad) a.grad[e] = g;
  }
  EXPL_CLK(12);
  // a timed-out hand-off of this group is reported through the call's fail
  // word (and so through the completion word below)
  if (t == 0 && !ok && a.fail)
    __hip_atomic_fetch_or(a.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the Philox counter advances once per call and the completion word (host
  // polling, oac_expl_action_now) is written once per call: the last group to
  // finish does both
  if (!a.eps || a.done || a.fail) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system: the outputs may be host memory
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned prev =
          __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == (unsigned)a.n - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (!a.eps) a.state->expl_counter = cnt_s + 1;
        __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned failed = 0;
        if (a.fail) {   // every group's report precedes its ticket (release / acquire above)
          failed = __hip_atomic_load(a.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.fail, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (a.done) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(a.done, a.done_seq | (failed ? 0x80000000u : 0u), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Twin critics (nq = 2, K = 1; the SAC / OAC trainers): the same action with
// one polled hand-off and one arrival instead of four hand-offs.  Two
// rewrites make that possible, both exact in real arithmetic:
//  * policy layer 1 from partial sums: the group's fixed parts of the policy's
//    hidden layer 0 (part p = rows [pH/32, (p+1)H/32), owned whole by one
//    workgroup) publish z_p = W1[:, part] h1[part] for all H outputs, so the
//    consumers of layer 1 add 32 partials instead of waiting for a hand-off
//    of h1 and another of h2;
//  * the Q_UB gradient through critic layer 1 with the seed factored out:
//    dh1_i = seed_i (sum_n W_last_i[n] [h2_i[n] > 0] W1_i[n, :]) (x) [h1_i > 0]
//    and seed_i = 1/2 +- beta |.|' depends only on sign(Q1 - Q2); so the
//    parts of critic layer 1's rows (16 per critic) publish their Q partial
//    W_last . h2 and their seed-free share of da, v_p = (u_p (x) [h1_i > 0])
//    W0_i[:, Do:] with u_p = sum_{n in part} ... W1_i[n, :] (Da floats, not
//    the H of u_p: round 4), and the workgroup whose arrival comes last reads
//    the partials and finishes alone in one wave (seeds, da = seed-weighted
//    sums of the parts, shift, sample).
//   S1  policy layer 0 rows of the workgroup's parts, their z_p; the critic
//       obs projections P_i of its parts      -> hand-off A (polled)
//   S2  (every workgroup) h2 = relu(b1 + sum_p z_p), heads, a = tanh(mean),
//       critic layer 0 h1_i = relu(P_i + W0_i[:, Do:] a); its parts of
//       critic layer 1: Q partials and v_p   -> arrival B (the last one goes on)
//   S3  (the last arrival, wave 0) Q_i, seeds, da, grad, shift, sample.
// Every sum runs over fixed parts or fixed lanes in a fixed order, so a row of
// a batched call is bitwise the same row of a single-observation call.
constexpr int kTwinZW = 8;   // policy rows per part held in registers (H <= 8 * kTwinParts)
constexpr int kTwinW0 = 9;   // W0_i[:, Do:] elements per thread in flight (2 H Da <= 9 x 1024)
__host__ __device__ inline long expl_twin_lds(int Do, int Da, int H, int threads) {
  return ((Do + Da + 3) & ~3L) + 4L * H + 64 + 128 + 2L * H * Da + (long)(threads / 64) * H;
}
// the twin kernel takes the call: twin critics, dims within its register and LDS budget
static bool expl_twin_ok(const ExplFusedArgs& a, int threads, bool wt) {
  if (a.nq != 2 || a.K != 1 || a.H < 1 || a.H > 64 * kRU || a.H > kTwinZW * kTwinParts ||
      (a.H + kTwinParts / 2 - 1) / (kTwinParts / 2) > threads / 64 || 2 * a.Da > 64 || 2 * a.H > threads || a.Do > 512 ||
      2L * a.H * a.Da > (long)kTwinW0 * threads)
    return false;
  const long lds = expl_twin_lds(a.Do, a.Da, a.H, threads);
  return wt ? lds <= kWtLdsFloats : lds * (long)sizeof(float) <= 64 * 1024;
}

#ifdef OAC_EXPL_CLOCK   // S3 runs on the last arrival, whichever workgroup that is
#define EXPL_CLK3(i) do { if (threadIdx.x == 0) g_expl_clock[i] = wall_clock64(); } while (0)
#else
#define EXPL_CLK3(i) do {} while (0)
#endif

template <bool WT, bool OBS>
__global__ void __launch_bounds__(1024) oac_expl_twin_kernel(ExplFusedArgs a, int row0, int G,
                                                             float* scratch, ExplObsArg oa) {
  float* sm;
  if constexpr (WT) {
    __shared__ __attribute__((aligned(16))) float sm_wt[kWtLdsFloats];
    sm = sm_wt;
  } else {
    extern __shared__ __attribute__((aligned(16))) float sm_dyn[];
    sm = sm_dyn;
  }
  constexpr int NP = kTwinParts, NPQ = kTwinParts / 2;
  const int Do = a.Do, Da = a.Da, H = a.H, Dq = Do + Da;
  const int gi = blockIdx.x / G, wg = blockIdx.x - gi * G;
  const int r = row0 + gi, t = threadIdx.x, nt = blockDim.x;
  const int lane = t & 63, wave = t >> 6, nw = nt >> 6;
  const float* const q0p = a.q[0];
  const float* const q1p = a.q[1];
  auto Qp = [&](int i) { return i == 0 ? q0p : q1p; };
  const float* pol = a.pol;
  float* Gv = scratch + (long)gi * expl_split_scratch(H);
  float* g_z = Gv;                         // [NP][H] policy layer-1 partials
  float* g_v = g_z + (long)NP * H;         // [NP][Da] seed-free da partials of the parts
  float* g_P = g_v + (long)NP * H;         // [2H]    critic obs projections (+ b0) (g_v keeps [NP][H] room)
  float* g_q = g_P + 2 * H;                // [NP]    Q partials
  unsigned* ctr = reinterpret_cast<unsigned*>(g_q + 64);   // [2] hand-off A, arrival B
  float* x = sm;                           // [Dq] ob | a
  float* h1p = x + ((Dq + 3) & ~3);        // [H]  policy layer 0 (this workgroup's rows)
  float* h2p = h1p + H;                    // [H]  policy layer 1
  float* h1q = h2p + H;                    // [2H] P_i, then critic layer 0
  float* head = h1q + 2 * H;               // [64] mean | raw log std
  float* misc = head + 64;                 // [128] Q, seeds, norm, row Q terms, da
  float* qrow = misc + 16;                 // [<= 48] per-row Q terms of a part
  float* w0a = misc + 128;                 // [2H][Da] W0_i[:, Do:]
  float* ctb = w0a + 2L * H * Da;          // [nw][H] per-row u terms, row 0 then u_p
  __shared__ long long cnt_s;
  if (t == 0) cnt_s = a.state->expl_counter;
  const int p0 = wg * NP / G, p1 = (wg + 1) * NP / G;   // this workgroup's parts
  // ---- ahead of everything: the weights of S1's first rows and of z.  The
  // S1 rows of this workgroup form one list -- its policy layer-0 rows
  // [rp0, rp1), then its obs-projection rows [rq0, rq1) over both critics;
  // wave w takes list rows 2w, 2w + 1 (+ 2 nw ...), lanes along k, every k of
  // a row in flight at once (Do <= 512).  The sum order is rows_matvec's
  // (k ascending per lane, then the butterfly), so the values are the same.
  const int rp0 = p0 * H / NP, rp1 = p1 * H / NP;
  const int rq0 = p0 * 2 * H / NP, rq1 = p1 * 2 * H / NP;
  const int npol = rp1 - rp0, n_s1 = npol + (rq1 - rq0);
  auto s1_src = [&](int l, const float*& w, const float*& bias) {
    if (l < npol) {
      w = pol + a.p_fc0_w + (long)(rp0 + l) * Do;
      bias = pol + a.p_fc0_b + rp0 + l;
    } else {
      const int rr = rq0 + l - npol, i = rr >= H ? 1 : 0, n = rr - i * H;
      w = Qp(i) + a.q_fc0_w + (long)n * Dq;
      bias = Qp(i) + a.q_fc0_b + n;
    }
  };
  constexpr int U1 = 8;
  float s1w[2][U1], s1b[2];
  if (n_s1 > 0) {   // (clamped rows: unconditional loads keep the wait counts exact)
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const float *w, *bias;
      s1_src(min(2 * wave + rr, n_s1 - 1), w, bias);
#pragma unroll
      for (int u = 0; u < U1; ++u) s1w[rr][u] = w[min(lane + 64 * u, Do - 1)];
      s1b[rr] = *bias;
    }
  }
  const int zs = nt / H, zm = t % H, zslot = t / H;
  const float* W1p = pol + a.p_fc1_w;
  float zw[kTwinZW];
  {
    const int p = p0 + zslot;
    const int n0 = p * H / NP, n1 = (p + 1) * H / NP;
    if (zslot < zs && p < p1 && n1 > n0) {
#pragma unroll
      for (int u = 0; u < kTwinZW; ++u) zw[u] = W1p[(long)zm * H + min(n0 + u, n1 - 1)];
    }
  }
  EXPL_CLK(0);
  if constexpr (OBS) {
    for (int k = t; k < Do; k += nt) x[k] = oa.v[k];
  } else {
    for (int k = t; k < Do; k += nt) x[k] = a.obs[(long)r * a.ld_obs + k];
  }
  __syncthreads();
  EXPL_CLK(1);
  // ---- S1: policy layer 0 rows (LDS) and the obs-projection rows (published)
  for (int l0 = 2 * wave; l0 < n_s1; l0 += 2 * nw) {
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int l = l0 + rr;
      if (l >= n_s1) break;
      const float *w, *bias;
      s1_src(l, w, bias);
      float acc = 0.f;
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        const int k = lane + 64 * u;
        const float wv = l0 == 2 * wave ? s1w[rr][u] : w[min(k, Do - 1)];
        acc = fmaf(wv, k < Do ? x[k] : 0.f, acc);
      }
      acc = wsum64(acc) + (l0 == 2 * wave ? s1b[rr] : *bias);
      if (lane == 0) {
        if (l < npol) h1p[rp0 + l] = fmaxf(acc, 0.f);
        else st_pub<WT>(g_P + rq0 + l - npol, acc);
      }
    }
  }
  __syncthreads();
  // z_p[m] = sum_{n in part p} W1[m, n] h1[n], n ascending, for every output m
  for (int pb = p0; pb < p1; pb += zs) {
    const int p = pb + zslot;
    if (zslot < zs && p < p1) {
      const int n0 = p * H / NP, n1 = (p + 1) * H / NP;
      float s = 0.f;
#pragma unroll
      for (int u = 0; u < kTwinZW; ++u)
        if (n0 + u < n1) s = fmaf(pb == p0 ? zw[u] : W1p[(long)zm * H + n0 + u], h1p[n0 + u], s);
      st_pub<WT>(g_z + (long)p * H + zm, s);
    }
  }
  EXPL_CLK(2);
  group_arrive<WT>(ctr + 0, G);
  // ahead, during the hand-off: the heads' rows, W0_i[:, Do:] into LDS, the
  // layer-1 bias, and the first critic part's W1 row of each wave
  RowsPre preh;
  // (every wave: the polling wave is past the heads' rows and loads nothing;
  // a pointer chosen per wave would keep preh in scratch)
  rows_pre(pol + a.p_head_w, H, pol + a.p_head_b, H, 0, 2 * Da, preh);
  const float b1v = t < H ? pol[a.p_fc1_b + t] : 0.f;
  int ci = 0, ra = 0, rb = 0;   // the first critic part: critic ci, rows [ra, rb)
  float w1r[kRU], b1q = 0.f, wlq = 0.f;
  if (p0 < p1) {
    ci = p0 / NPQ;
    ra = (p0 % NPQ) * H / NPQ;
    rb = (p0 % NPQ + 1) * H / NPQ;
    if (wave < rb - ra) {   // (the polling wave too: its first poll waits these out, inside the hand-off)
      const float* q = Qp(ci);
      const int n = ra + wave;
#pragma unroll
      for (int u = 0; u < kRU; ++u) w1r[u] = q[a.q_fc1_w + (long)n * H + min(lane + 64 * u, H - 1)];
      b1q = q[a.q_fc1_b + n];
      wlq = q[a.q_last_w + n];
    }
  }
  // W0_i[:, Do:] element e = t + u * threads (u < kTwinW0) of the [2H][Da]
  // image: its source, stepped without a division per element
  const int n0a = 2 * H * Da;
  const float* wsrc[kTwinW0];
  {
    const int ers = t / Da, ej = t - ers * Da;           // row (over both critics), column
    const int drow = nt / Da, dj = nt - drow * Da;
    int rw = ers, jj = ej;
#pragma unroll
    for (int u = 0; u < kTwinW0; ++u) {
      const int rr = min(rw, 2 * H - 1), i = rr >= H ? 1 : 0;
      wsrc[u] = Qp(i) + a.q_fc0_w + (long)(rr - i * H) * Dq + Do + (rw < 2 * H ? jj : 0);
      rw += drow; jj += dj;
      if (jj >= Da) { jj -= Da; ++rw; }
    }
  }
  bool ok = group_wait<WT>(ctr + 0, G);
  EXPL_CLK(3);
  // ---- S2 (every workgroup): policy layer 1 from the parts' partials (H <=
  // threads: one output per thread) and P; W0_i[:, Do:] requested behind them
  // (into LDS after the heads; every load in flight before the first store;
  // expl_twin_ok: at most kTwinW0 per thread)
  // (loads unconditional, clamped: a branch between a load and its use makes
  // the wait count assume no load in flight)
  float zz[NP];
  const int tz = min(t, H - 1);
#pragma unroll
  for (int p = 0; p < NP; ++p) zz[p] = ld_pub<WT>(g_z + (long)p * H + tz);
  const float pv = ld_pub<WT>(g_P + min(t, 2 * H - 1));
  float wt[kTwinW0];
#pragma unroll
  for (int u = 0; u < kTwinW0; ++u) wt[u] = *wsrc[u];
  if (t < H) {
    float s = zz[0];
#pragma unroll
    for (int p = 1; p < NP; ++p) s += zz[p];
    h2p[t] = fmaxf(s + b1v, 0.f);
  }
  if (t < 2 * H) h1q[t] = pv;
  __syncthreads();
  EXPL_CLK(4);
  rows_matvec<false, WT>(pol + a.p_head_w, H, pol + a.p_head_b, h2p, H, 0, 2 * Da, head, false,
                         &preh);
  __syncthreads();
  if (t < Da) x[Do + t] = tanhf(head[t]);
#pragma unroll
  for (int u = 0; u < kTwinW0; ++u)
    if (t + u * nt < n0a) w0a[t + u * nt] = wt[u];
  __syncthreads();
  EXPL_CLK(5);
  for (int e = t; e < 2 * H; e += nt) {   // h1_i = relu(P_i + W0_i[:, Do:] a)
    float s = h1q[e];
    for (int j = 0; j < Da; ++j) s = fmaf(w0a[(long)e * Da + j], x[Do + j], s);
    h1q[e] = fmaxf(s, 0.f);
  }
  __syncthreads();
  EXPL_CLK(6);
  // critic layer 1 rows of the parts: one wave per row (lanes along k), the
  // row's Q term W_last[n] h2[n] and its u term c_n W1[n, :] (c_n = W_last[n]
  // [h2[n] > 0]); per part the terms are summed in row order
  for (int p = p0; p < p1; ++p) {
    const int i = p / NPQ, na = (p % NPQ) * H / NPQ, nb = (p % NPQ + 1) * H / NPQ;
    const float* q = Qp(i);
    if (wave < nb - na) {
      const int n = na + wave;
      float wv[kRU];
      float bq, wl;
      if (p == p0) {
#pragma unroll
        for (int u = 0; u < kRU; ++u) wv[u] = w1r[u];
        bq = b1q; wl = wlq;
      } else {
#pragma unroll
        for (int u = 0; u < kRU; ++u) wv[u] = q[a.q_fc1_w + (long)n * H + min(lane + 64 * u, H - 1)];
        bq = q[a.q_fc1_b + n]; wl = q[a.q_last_w + n];
      }
      float s = 0.f;
#pragma unroll
      for (int u = 0; u < kRU; ++u)
        if (lane + 64 * u < H) s = fmaf(wv[u], h1q[i * H + lane + 64 * u], s);
      s = wsum64(s);
      const float h2 = fmaxf(s + bq, 0.f);
      const float c = h2 > 0.f ? wl : 0.f;
#pragma unroll
      for (int u = 0; u < kRU; ++u)
        if (lane + 64 * u < H) ctb[(long)wave * H + lane + 64 * u] = c * wv[u];
      if (lane == 0) qrow[wave] = wl * h2;
    }
    __syncthreads();
    // (rows of a part <= 16: every LDS read before the first add; an empty
    // part publishes zeros).  u_p[k] goes to row 0 of ctb: thread k is the
    // only reader and writer of column k (H <= nt, expl_twin_ok)
    for (int k = t; k < H; k += nt) {
      float cc[16];
#pragma unroll
      for (int w = 0; w < 16; ++w) cc[w] = w < nb - na ? ctb[(long)w * H + k] : 0.f;
      float s = cc[0];
#pragma unroll
      for (int w = 1; w < 16; ++w)
        if (w < nb - na) s += cc[w];
      ctb[k] = s;
    }
    if (t == nt - 64) {   // (a wave without u columns when H <= nt - 64)
      float cc[16];
#pragma unroll
      for (int w = 0; w < 16; ++w) cc[w] = w < nb - na ? qrow[w] : 0.f;
      float s = cc[0];
#pragma unroll
      for (int w = 1; w < 16; ++w)
        if (w < nb - na) s += cc[w];
      st_pub<WT>(g_q + p, s);
    }
    __syncthreads();
    // the part's seed-free share of da: v_p[j] = sum_k [h1_i[k] > 0] u_p[k]
    // W0_i[k, Do + j] (one half-wave per j, lanes along k in a fixed order),
    // Da floats published instead of the H of u_p -- the last arrival then
    // only weighs the parts by the seeds (S3)
    {
      const int hw = t >> 5, l32 = t & 31;
      if (hw < Da) {
        float cv[16], wv[16];   // (H <= 512: every LDS read before the first FMA)
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int k = l32 + 32 * u;
          const bool in = k < H;
          cv[u] = in && h1q[i * H + k] > 0.f ? ctb[k] : 0.f;
          wv[u] = in ? w0a[(long)(i * H + k) * Da + hw] : 0.f;
        }
        float sj = 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u) sj = fmaf(cv[u], wv[u], sj);
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) sj += __shfl_xor(sj, o, 32);
        if (l32 == 0) st_pub<WT>(g_v + (long)p * Da + hw, sj);
      }
    }
    __syncthreads();
  }
  EXPL_CLK(7);
  // S3's per-lane terms that need no other workgroup's parts -- the action,
  // std, mean and the exploration draw -- ahead of the arrival in every
  // workgroup's wave 0 (whichever arrives last goes on with them in registers)
  float p_act = 0.f, p_sd = 0.f, p_mean = 0.f, p_ev = 0.f;
  if (wave == 0 && lane < Da) {
    p_act = x[Do + lane];
    p_sd = expf(fminf(fmaxf(head[Da + lane], -20.f), 2.f));
    p_mean = head[lane];
    p_ev = a.eps ? a.eps[(long)r * Da + lane]
                 : philox_normal(a.seed, (unsigned long long)cnt_s, 3u, (unsigned)(r * Da + lane));
  }
  // ---- arrival B: the last workgroup of the group goes on to S3.  The add
  // carries this workgroup's hand-off failure in bit 16, so the last arrival
  // learns every member's from the value its add returns.
  if (t == 0 && !ok && a.fail)   // a timed-out hand-off of this workgroup: reported
    __hip_atomic_fetch_or(a.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ unsigned arr_s;
  if (t == 0) {
    unsigned prev = 0;
    if (G > 1) {
      if constexpr (!WT) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      prev = __hip_atomic_fetch_add(ctr + 1, ok ? 1u : 0x10001u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (!WT) {
        if ((prev & 0xffffu) == (unsigned)G - 1) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
    }
    arr_s = prev;
  }
  __syncthreads();
  const unsigned arrived = arr_s;
  if ((arrived & 0xffffu) != (unsigned)G - 1) return;
  const bool others_failed = (arrived >> 16) != 0;
  EXPL_CLK3(8);
  // ---- S3 (the last arrival): Q_i, seeds, da
  if (t == 0 && G > 1) {   // every member is past both hand-offs: re-arm
    __hip_atomic_store(ctr + 0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // wave 0 alone: lane p < 32 reads part p's Q partial (critic p / 16), lane
  // j < Da the 32 parts' da partials v_p[j]
  if (wave != 0) return;
  const float qv = ld_pub<WT>(g_q + (lane & (NP - 1)));
  const float blast = Qp(lane & NPQ ? 1 : 0)[a.q_last_b];
  float vv[NP];
  {
    const int j = min(lane, Da - 1);
#pragma unroll
    for (int p = 0; p < NP; ++p) vv[p] = ld_pub<WT>(g_v + (long)p * Da + j);
  }
  // Q_i: a fixed butterfly over the critic's 16 parts, then the bias
  float q = qv;
#pragma unroll
  for (int o = NPQ / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  q += blast;
  const float q0 = __shfl(q, 0, 64), q1 = __shfl(q, NPQ, 64);
  // Q_UB = (Q1+Q2)/2 + beta |Q1-Q2|/2: d|x|/dx = sign(x) (0 at 0)
  const float dq = q0 - q1;
  const float sg = dq > 0.f ? 1.f : (dq < 0.f ? -1.f : 0.f);
  const float hb = a.beta_UB / 2.f;
  const float seed0 = 0.5f + hb * sg, seed1 = 0.5f - hb * sg;
  EXPL_CLK3(9);
  // da[j] = seed_1 sum_{p < 16} v_p[j] + seed_2 sum_{p >= 16} v_p[j], parts in order
  float v0 = vv[0], v1 = vv[NPQ];
#pragma unroll
  for (int p = 1; p < NPQ; ++p) { v0 += vv[p]; v1 += vv[NPQ + p]; }
  const float da = seed0 * v0 + seed1 * v1;
  EXPL_CLK3(10);
  // grad, shift, sample (Da <= 32), the norm as a wave sum
  const float sd = p_sd, sig = p_sd * p_sd, mean = p_mean, ev = p_ev;
  const float g = lane < Da ? da * (1.f - p_act * p_act) : 0.f;
  const float nrm = sqrtf(wsum64(lane < Da ? g * g * sig : 0.f)) + 10e-6f;
  // the call's only group with a host-polled completion word: the outputs
  // (host memory) as system-scope stores, drained, then the word -- no ticket
  const bool solo = a.n == 1 && a.done;
  if (a.n == 1 && a.tags) {   // tagged granules: no store drain, no completion word
    const unsigned tag = a.done_seq | ((!ok || others_failed) ? 0x80000000u : 0u);
    if (lane < Da) {
      const float mu_C = (a.sqrt_2delta * (sig * g)) / nrm;
      const float mu_E = mean + mu_C;
      const float nan = __int_as_float(0x7fc00000);
      put_tagged(a.tags + lane, ok ? tanhf(__fadd_rn(__fmul_rn(ev, sd), mu_E)) : nan, tag);
      put_tagged(a.tags + Da + lane, ok ? mu_E : nan, tag);
      put_tagged(a.tags + 2 * Da + lane, sd, tag);
      if (a.grad) a.grad[lane] = g;
    }
    if (lane == 0) {
      if (!a.eps) a.state->expl_counter = cnt_s + 1;
      if ((!ok || others_failed) && a.fail)
        __hip_atomic_store(a.fail, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    EXPL_CLK3(11);
    return;
  }
  if (lane < Da) {
    const long e = (long)r * Da + lane;
    const float mu_C = (a.sqrt_2delta * (sig * g)) / nrm;
    const float mu_E = mean + mu_C;
    const long nd = (long)a.n * Da;
    const float nan = __int_as_float(0x7fc00000);
    const float o0 = ok ? tanhf(__fadd_rn(__fmul_rn(ev, sd), mu_E)) : nan, o1 = ok ? mu_E : nan;
    if (solo) {
      __hip_atomic_store(a.out + e, o0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.out + nd + e, o1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.out + 2 * nd + e, sd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      a.out[e] = o0;
      a.out[nd + e] = o1;
      a.out[2 * nd + e] = sd;
    }
    if (a.grad) a.grad[e] = g;
  }
  if (solo) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      if (!a.eps) a.state->expl_counter = cnt_s + 1;
      const unsigned failed = (!ok || others_failed) ? 1u : 0u;   // (the arrival told)
      if (failed && a.fail) __hip_atomic_store(a.fail, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.done, a.done_seq | (failed ? 0x80000000u : 0u), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
    EXPL_CLK3(11);
    return;
  }
  EXPL_CLK3(11);
  if (t == 0 && !ok && a.fail)
    __hip_atomic_fetch_or(a.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the Philox counter and the completion word: the last group to finish
  if (!a.eps || a.done || a.fail) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (wave 0 alone from here)
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system: the outputs may be host memory
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned prev =
          __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == (unsigned)a.n - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (!a.eps) a.state->expl_counter = cnt_s + 1;
        __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned failed = 0;
        if (a.fail) {
          failed = __hip_atomic_load(a.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.fail, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (a.done) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(a.done, a.done_seq | (failed ? 0x80000000u : 0u), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
}

long expl_split_scratch_floats(int H) { return expl_split_scratch(H); }

// threads per workgroup: 1024.  Humanoid, one observation, host wall per call
// (round 2, tools/gpu_expl_ab.sh): 256 / 512 / 1024 threads 54.6 / 46.5 / 45.2
// us at 16 workgroups per row; 1024 threads 49.4 / 45.2 / 44.4 us at 8 / 16 /
// 32 workgroups per row
int expl_split_threads() { return 1024; }

size_t expl_split_lds_bytes(int Do, int Da, int H) {
  return sizeof(float) * expl_split_lds(Do, Da, H, 1024);
}

// compute units of the current device (read once per process: one device per
// process, as the trainer is built)
int expl_device_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      return 1;   // unknown: one workgroup per observation, no hand-offs
    return n;
  }();
  return v;
}

// group size for a launch of n_rows observations: the device's CUs shared
// out, at most kExplGroup
// (tools/micro/expl_micro's group-size sweep lowers it)
int g_expl_group_cap = kExplGroup;
int expl_split_group(int n_rows) {
  const int g = expl_device_cus() / (n_rows < 1 ? 1 : n_rows);
  const int cap = g_expl_group_cap;
  return g < 1 ? 1 : (g > cap ? cap : g);
}

// the twin-critic kernel off (tools/micro/expl_micro's A/B against the split kernel)
bool g_expl_twin_off = false;

// rows [row0, row0 + n_rows) of the call, one group of G workgroups each
hipError_t launch_expl_split(const ExplFusedArgs& a, int row0, int n_rows, float* scratch,
                             hipStream_t s) {
  if (n_rows < 1 || n_rows > kExplRows || a.Da < 1 || a.Da > 63 || a.H < 1 || a.K > 16)
    return hipErrorInvalidValue;
  const int nt = expl_split_threads();
  const int G = expl_split_group(n_rows);
  static const ExplObsArg none{};   // (unread)
  // write-through hand-offs need every workgroup of the launch on a CU of its own
  const bool own_cu = G > 1 && (long)n_rows * G <= expl_device_cus();
  if (!g_expl_twin_off && expl_twin_ok(a, nt, own_cu)) {
    if (own_cu) {
      OAC_LAUNCH((oac_expl_twin_kernel<true, false>), dim3(n_rows * G), dim3(nt), 0, s, a, row0, G,
                 scratch, none);
    } else {
      OAC_LAUNCH((oac_expl_twin_kernel<false, false>), dim3(n_rows * G), dim3(nt),
                 expl_twin_lds(a.Do, a.Da, a.H, nt) * sizeof(float), s, a, row0, G, scratch, none);
    }
    return hipGetLastError();
  }
  const long lds = expl_split_lds(a.Do, a.Da, a.H, nt);
  const bool wt = own_cu && lds <= kWtLdsFloats;
  if (wt) {
    OAC_LAUNCH((oac_expl_split_kernel<true, false>), dim3(n_rows * G), dim3(nt), 0, s, a, row0, G,
               scratch, none);
  } else {
    if (lds * sizeof(float) > 64 * 1024) return hipErrorInvalidValue;
    OAC_LAUNCH((oac_expl_split_kernel<false, false>), dim3(n_rows * G), dim3(nt), lds * sizeof(float),
               s, a, row0, G, scratch, none);
  }
  return hipGetLastError();
}

hipError_t launch_expl_split_obs(const ExplFusedArgs& a, const ExplObsArg& obs, float* scratch,
                                 hipStream_t s) {
  if (a.n != 1 || a.Do > kExplObsArg || a.Da < 1 || a.Da > 63 || a.H < 1 || a.K > 16)
    return hipErrorInvalidValue;
  const int nt = expl_split_threads();
  const int G = expl_split_group(1);
  const bool own_cu = G > 1 && G <= expl_device_cus();
  if (own_cu && !g_expl_twin_off && expl_twin_ok(a, nt, true)) {
    OAC_LAUNCH((oac_expl_twin_kernel<true, true>), dim3(G), dim3(nt), 0, s, a, 0, G, scratch, obs);
    return hipGetLastError();
  }
  const long lds = expl_split_lds(a.Do, a.Da, a.H, nt);
  if (!(own_cu && lds <= kWtLdsFloats)) return launch_expl_split(a, 0, 1, scratch, s);
  OAC_LAUNCH((oac_expl_split_kernel<true, true>), dim3(G), dim3(nt), 0, s, a, 0, G, scratch, obs);
  return hipGetLastError();
}

}  // namespace oac
