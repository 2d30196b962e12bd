// OAC exploration action with the weight stream of ONE observation spread over
// a group of G workgroups (get_optimistic_exploration_action,
// /root/reference/optimistic_exploration.py:14-109; same outputs and modes as
// expl_fused.hip: twin critics, or one K-head critic with mean + beta std or
// the trainer_UB sorted head).
//
// Every layer is cut into P = kExplParts row parts (part p: rows [pH/P,
// (p+1)H/P)); workgroup w of the group owns parts w, w + G, ...  A part turns
// the product that CONSUMES its rows into a partial sum over them, so the
// group meets only twice (two in-launch hand-offs) instead of once per layer:
//   A  (parts)  policy layer 0 rows -> h1p;  the critics' obs projections
//               P_i = W0_i[:, :Do] ob + b0_i of the part's rows (published);
//               the policy layer-1 partial t_p = W1p[:, rows] h1p[rows] (published)
//   -- hand-off 1 --
//   B  (every workgroup) h2p = relu(b1p + sum_p t_p), the heads -> mean, std,
//               a = tanh(mean), critic layer 0 h1_i = relu(P_i + W0_i[:, Do:] a);
//      (parts)  critic layer-1 rows h2_i[rows]; the Q partial over the part's
//               rows (q = w_last . h2 + b) and the backward partial to the action
//                 v_o = W0a^T (1[h1 > 0] (W1[rows]^T (1[h2[rows] > 0] w_last_o[rows])))
//               for each seed output o (two critics, or K heads): dQ_o/da is
//               linear in the rows' contributions, so it is a sum over parts
//   -- hand-off 2 --
//   C  (workgroup 0) Q_o = b_last_o + sum_p q_p, the Q_UB seeds s_o, da =
//               sum_o s_o sum_p v_o,p, grad, shift, sample.
// Hand-off forms (MI355X_MICROARCH.md, "Valid forms"):
//   WT    one workgroup per CU (84 KB of static LDS admits no second one):
//         write-through (sc1) stores of the published vectors, every storing
//         wave's vmcnt(0), a barrier, lane 0's agent-scope counter add; the
//         consumer polls with sc1 loads, meets at a barrier and reads the
//         vectors with sc1 loads -- no cache write-back or invalidate;
//   FENCE plain stores, lane-0 agent release before the add, agent acquire after
//         the poll: any number of workgroups per CU (large batches).
// G = 1 (batches of >= 256 observations) needs no hand-off at all.
// Every sum's order is fixed by the parts (p = 0 .. P-1) and the lanes, never
// by G or by the observations per launch, so a row of a batched call is
// bitwise the row of a single-observation call.
#include "oac_common.h"
#include "kernels.h"

namespace oac {

constexpr int kExplParts = 32;   // row parts of every layer (>= the largest group)
constexpr int kExplKq = 16;      // seed outputs: 2 critics or up to 16 heads

__device__ __forceinline__ float wsum64(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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

// out(e, row(e) . x(e)[0:K]) for the items e < n: RW items per wave at once,
// lanes along k (U loads per lane in flight per round), a fixed-order
// butterfly over the lanes
template <int RW, int U, class RowFn, class XFn, class OutFn>
__device__ __forceinline__ void dot_items(int n, int K, RowFn row, XFn xv, OutFn out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int e0 = wave * RW; e0 < n; e0 += nw * RW) {
    float acc[RW];
    const float* rp[RW];
    const float* xp[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int e = min(e0 + r, n - 1);
      acc[r] = 0.f;
      rp[r] = row(e);
      xp[r] = xv(e);
    }
    for (int kb = 0; kb < K; kb += 64 * U) {
      float w[RW][U], xx[RW][U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = kb + u * 64 + lane;
        const int kc = k < K ? k : K - 1;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          w[r][u] = rp[r][kc];
          xx[r][u] = k < K ? xp[r][kc] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RW; ++r) acc[r] = fmaf(w[r][u], xx[r][u], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const float v = wsum64(acc[r]);
      if (lane == 0 && e0 + r < n) out(e0 + r, v);
    }
  }
}

// The group's hand-off: every storing wave drains its stores, the workgroup
// meets, lane 0 arrives on the stage counter (FENCE: behind an agent release)
// and polls it (relaxed, bounded) until all G workgroups arrived (FENCE: then
// acquires); the workgroup meets again.  wait = false: arrive only.
template <bool WT>
__device__ __forceinline__ bool group_sync(unsigned* ctr, unsigned target, bool wait = true) {
  __shared__ int ok_s;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (target <= 1) return true;   // G = 1: the workgroup's own barrier orders its scratch
  if (threadIdx.x == 0) {
    if constexpr (!WT) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    if (wait) {
      unsigned spins = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 25)) { ok = 0; break; }   // ~0.3 s: a stuck group gives up
      }
      if constexpr (!WT) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    ok_s = ok;
  }
  __syncthreads();
  return ok_s != 0;
}

// per-observation scratch (floats): t partials [P][H] | obs projections [2][H]
// | Q partials [P][Kq] | action partials [P][Kq][Da] | 4 counters
__host__ __device__ inline long expl_split_scratch(int H, int Da) {
  return (long)kExplParts * H + 2L * H + (long)kExplParts * kExplKq * (1 + Da) + 64;
}
// LDS floats: x = ob | a [Do + Da] | h1p part [H] | h2p [H] | head [128] |
// critic h1 [2H] | critic h2 part [2H] | u [Kq][H] | misc [128]
__host__ __device__ inline long expl_split_lds(int Do, int Da, int H, int threads) {
  (void)threads;
  return ((Do + Da + 3) & ~3L) + 6L * H + (long)kExplKq * H + 256;
}
constexpr int kWtLdsFloats = 21 * 1024;   // 84 KB: one workgroup per CU

template <bool WT>
__global__ void __launch_bounds__(1024) oac_expl_split_kernel(ExplFusedArgs a, int row0, int G,
                                                              float* scratch) {
  float* sm;
  if constexpr (WT) {
    __shared__ __attribute__((aligned(16))) float sm_wt[kWtLdsFloats];
    sm = sm_wt;
  } else {
    extern __shared__ __attribute__((aligned(16))) float sm_dyn[];
    sm = sm_dyn;
  }
  constexpr int P = kExplParts;
  const int Do = a.Do, Da = a.Da, H = a.H, Dq = Do + Da;
  const int gi = blockIdx.x / G, wg = blockIdx.x - gi * G;
  const int r = row0 + gi, t = threadIdx.x, nt = blockDim.x;
  const int nq = a.nq, KQ = a.K;
  const int Kq = nq == 2 ? 2 : KQ;   // seed outputs: the two critics, or the K heads
  float* Gv = scratch + (long)gi * expl_split_scratch(H, Da);   // group's published vectors
  float* g_t = Gv;                         // [P][H]   policy layer-1 partials
  float* g_P = g_t + (long)P * H;          // [2][H]   critics' obs projections (+ b0)
  float* g_q = g_P + 2L * H;               // [P][Kq]  Q partials
  float* g_v = g_q + P * kExplKq;          // [P][Kq][Da] action-gradient partials
  unsigned* ctr = reinterpret_cast<unsigned*>(g_v + (long)P * kExplKq * Da);   // [2]
  float* x = sm;                           // [Do + Da] ob | a
  float* h1p = x + ((Dq + 3) & ~3);        // [H] policy layer 0 of the current part's rows
  float* h2p = h1p + H;                    // [H] policy layer 1
  float* head = h2p + H;                   // [128] mean | raw log std
  float* qh1 = head + 128;                 // [2][H] critic layer 0
  float* qh2 = qh1 + 2 * H;                // [2][H] critic layer 1, the current part's rows
  float* u = qh2 + 2 * H;                  // [Kq][H] W1[rows]^T c_o
  float* misc = u + kExplKq * H;           // [128]
  const float* W0p = a.pol + a.p_fc0_w;
  const float* W1p = a.pol + a.p_fc1_w;
  auto qw = [&](int i) { return a.q[i]; };
  // seed output o: its critic and its last-layer row
  auto crit = [&](int o) { return nq == 2 ? o : 0; };
  auto lastw = [&](int o) { return nq == 2 ? a.q[o] + a.q_last_w : a.q[0] + a.q_last_w + (long)o * H; };
  auto lastb = [&](int o) { return nq == 2 ? a.q[o][a.q_last_b] : a.q[0][a.q_last_b + o]; };
  __shared__ long long cnt_s;
  if (t == 0) cnt_s = a.state->expl_counter;
  for (int k = t; k < Do; k += nt) x[k] = a.obs[(long)r * a.ld_obs + k];
  __syncthreads();

  // ---- A: per part, policy layer 0 rows, critic obs projections, layer-1 partial
  for (int p = wg; p < P; p += G) {
    const int lo = p * H / P, hi = (p + 1) * H / P, nr = hi - lo;
    if (nr > 0) {
      dot_items<2, 8>((1 + nq) * nr, Do,
          [&](int e) {
            const int which = e / nr, n = lo + e - which * nr;
            return which == 0 ? W0p + (long)n * Do : qw(which - 1) + a.q_fc0_w + (long)n * Dq;
          },
          [&](int) { return (const float*)x; },
          [&](int e, float v) {
            const int which = e / nr, n = lo + e - which * nr;
            if (which == 0) h1p[n - lo] = fmaxf(v + a.pol[a.p_fc0_b + n], 0.f);
            else st_pub<WT>(g_P + (which - 1) * H + n, v + qw(which - 1)[a.q_fc0_b + n]);
          });
      __syncthreads();
      for (int m = t; m < H; m += nt) {   // t_p[m] = sum_{n in part} W1p[m, n] h1p[n]
        const float* w = W1p + (long)m * H + lo;
        float s = 0.f;
        for (int j = 0; j < nr; ++j) s = fmaf(w[j], h1p[j], s);
        st_pub<WT>(g_t + (long)p * H + m, s);
      }
      __syncthreads();
    }
  }
  bool ok = group_sync<WT>(ctr + 0, G);

  // ---- B: the whole policy forward's tail and critic layer 0 (every workgroup)
  for (int m = t; m < H; m += nt) {
    float tp[P];
#pragma unroll
    for (int p = 0; p < P; ++p) tp[p] = ld_pub<WT>(g_t + (long)p * H + m);
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < P; ++p) s += tp[p];
    h2p[m] = fmaxf(s + a.pol[a.p_fc1_b + m], 0.f);
  }
  __syncthreads();
  dot_items<3, 4>(2 * Da, H, [&](int e) { return a.pol + a.p_head_w + (long)e * H; },
                  [&](int) { return (const float*)h2p; },
                  [&](int e, float v) { head[e] = v + a.pol[a.p_head_b + e]; });
  __syncthreads();
  if (t < Da) x[Do + t] = tanhf(head[t]);
  __syncthreads();
  for (int e = t; e < nq * H; e += nt) {   // h1_i = relu(P_i + W0_i[:, Do:] a)
    const int i = e / H, n = e - i * H;
    const float* w = qw(i) + a.q_fc0_w + (long)n * Dq + Do;
    float s = ld_pub<WT>(g_P + e);
    for (int j = 0; j < Da; ++j) s = fmaf(w[j], x[Do + j], s);
    qh1[e] = fmaxf(s, 0.f);
  }
  __syncthreads();
  // ---- B (parts): critic layer-1 rows, Q partials, action-gradient partials
  for (int p = wg; p < P; p += G) {
    const int lo = p * H / P, hi = (p + 1) * H / P, nr = hi - lo;
    if (nr > 0) {
      dot_items<1, 4>(nq * nr, H,
          [&](int e) {
            const int i = e / nr, n = lo + e - i * nr;
            return qw(i) + a.q_fc1_w + (long)n * H;
          },
          [&](int e) { return (const float*)(qh1 + (e / nr) * H); },
          [&](int e, float v) {
            const int i = e / nr, n = lo + e - i * nr;
            qh2[i * H + n - lo] = fmaxf(v + qw(i)[a.q_fc1_b + n], 0.f);
          });
      __syncthreads();
      if (t < Kq) {   // q partial of seed output o over the part's rows
        const float* w = lastw(t);
        const float* h = qh2 + crit(t) * H;
        float s = 0.f;
        for (int j = 0; j < nr; ++j) s = fmaf(w[lo + j], h[j], s);
        st_pub<WT>(g_q + p * kExplKq + t, s);
      }
      for (int e = t; e < Kq * H; e += nt) {   // u_o[k] = sum_{n in part} c_o[n] W1[n, k]
        const int o = e / H, k = e - o * H, i = crit(o);
        const float* w = lastw(o);
        const float* h = qh2 + i * H;
        const float* W1 = qw(i) + a.q_fc1_w + k;
        float s = 0.f;
        for (int j = 0; j < nr; ++j) {
          const float c = h[j] > 0.f ? w[lo + j] : 0.f;
          s = fmaf(c, W1[(long)(lo + j) * H], s);
        }
        u[e] = s;
      }
      __syncthreads();
      // v_o[j] = sum_k u_o[k] 1[h1_i[k] > 0] W0_i[k, Do + j]: one wave per (o, j)
      {
        const int lane = t & 63, wave = t >> 6, nw = nt >> 6;
        for (int e = wave; e < Kq * Da; e += nw) {
          const int o = e / Da, j = e - o * Da, i = crit(o);
          const float* W0 = qw(i) + a.q_fc0_w + Do + j;
          const float* uo = u + o * H;
          const float* h = qh1 + i * H;
          float s = 0.f;
          for (int k = lane; k < H; k += 64)
            s = fmaf(h[k] > 0.f ? uo[k] : 0.f, W0[(long)k * Dq], s);
          s = wsum64(s);
          if (lane == 0) st_pub<WT>(g_v + ((long)p * kExplKq + o) * Da + j, s);
        }
      }
      __syncthreads();
    }
  }
  if (wg != 0) {   // the group's other workgroups only publish (their arrival is the signal)
    group_sync<WT>(ctr + 1, G, false);
    return;
  }
  ok = group_sync<WT>(ctr + 1, G) && ok;

  // ---- C (workgroup 0): Q, the Q_UB seeds, da, grad, shift, sample
  float* qv = misc;        // [16] Q_o
  float* sd_o = misc + 16; // [16] seeds
  float* red = misc + 32;  // [64]
  if (t < Kq) {
    float s = 0.f;
    for (int p = 0; p < P; ++p) s += ld_pub<WT>(g_q + p * kExplKq + t);
    qv[t] = s + lastb(t);
  }
  __syncthreads();
  if (t == 0) {
    if (nq == 2) {   // Q_UB = (Q1+Q2)/2 + beta |Q1-Q2|/2: d|x|/dx = sign(x) (0 at 0)
      const float d = qv[0] - qv[1];
      const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      const float hb = a.beta_UB / 2.f;
      sd_o[0] = 0.5f + hb * sg;
      sd_o[1] = 0.5f - hb * sg;
    } else if (a.ub_index >= 0) {   // trainer_UB: the head ranked ub_index (ties: lower index)
      for (int k = 0; k < KQ; ++k) {
        int rank = 0;
        for (int j = 0; j < KQ; ++j) rank += (qv[j] < qv[k]) || (qv[j] == qv[k] && j < k);
        sd_o[k] = rank == a.ub_index ? 1.f : 0.f;
      }
    } else {         // mean_k + beta std_k (unbiased)
      float s = 0.f;
      for (int k = 0; k < KQ; ++k) s += qv[k];
      const float mu = s / (float)KQ;
      float ss = 0.f;
      for (int k = 0; k < KQ; ++k) ss += (qv[k] - mu) * (qv[k] - mu);
      const float sdv = sqrtf(ss / (float)(KQ - 1));
      for (int k = 0; k < KQ; ++k)
        sd_o[k] = 1.f / (float)KQ + a.beta_UB * ((qv[k] - mu) / ((float)(KQ - 1) * sdv));
    }
  }
  __syncthreads();
  float g = 0.f, sig = 0.f, sd = 0.f, mean = 0.f;
  if (t < Da) {
    float da = 0.f;
    for (int o = 0; o < Kq; ++o) {
      float vs = 0.f;
      for (int p = 0; p < P; ++p) vs += ld_pub<WT>(g_v + ((long)p * kExplKq + o) * Da + t);
      da = fmaf(sd_o[o], vs, da);
    }
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
    misc[64 + 48] = sqrtf(s) + 10e-6f;
    if (G > 1)   // every member is past its last hand-off
      for (int c = 0; c < 2; ++c) __hip_atomic_store(ctr + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (t < Da) {
    const long e = (long)r * Da + t;
    const float mu_C = (a.sqrt_2delta * (sig * g)) / misc[64 + 48];
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

long expl_split_scratch_floats(int H, int Da) { return expl_split_scratch(H, Da); }

// threads per workgroup (OAC_EXPL_THREADS: 256 / 512 / 1024)
int expl_split_threads() {
  static const int v = [] {
    const char* e = getenv("OAC_EXPL_THREADS");
    const int n = e ? atoi(e) : 1024;
    return (n == 256 || n == 512 || n == 1024) ? n : 1024;
  }();
  return v;
}

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
// out, at most kExplGroup (OAC_EXPL_GROUP overrides the cap: tuning runs;
// never more than the row parts)
int expl_split_group(int n_rows) {
  static const int cap = [] {
    const char* e = getenv("OAC_EXPL_GROUP");
    const int v = e ? atoi(e) : kExplGroup;
    return v < 1 ? 1 : (v > kExplParts ? kExplParts : v);
  }();
  const int g = expl_device_cus() / (n_rows < 1 ? 1 : n_rows);
  return g < 1 ? 1 : (g > cap ? cap : g);
}

// rows [row0, row0 + n_rows) of the call, one group of G workgroups each
hipError_t launch_expl_split(const ExplFusedArgs& a, int row0, int n_rows, float* scratch,
                             hipStream_t s) {
  if (n_rows < 1 || n_rows > kExplRows || a.Da < 1 || a.Da > 63 || a.H < 1 || a.K > kExplKq ||
      2 * a.Da > 128)
    return hipErrorInvalidValue;
  const int nt = expl_split_threads();
  const int G = expl_split_group(n_rows);
  const long lds = expl_split_lds(a.Do, a.Da, a.H, nt);
  // write-through hand-offs need every workgroup of the launch on a CU of its own
  const bool wt = G > 1 && (long)n_rows * G <= expl_device_cus() && lds <= kWtLdsFloats;
  if (wt) {
    OAC_LAUNCH(oac_expl_split_kernel<true>, dim3(n_rows * G), dim3(nt), 0, s, a, row0, G, scratch);
  } else {
    if (lds * sizeof(float) > 64 * 1024) return hipErrorInvalidValue;
    OAC_LAUNCH(oac_expl_split_kernel<false>, dim3(n_rows * G), dim3(nt), lds * sizeof(float), s, a,
               row0, G, scratch);
  }
  return hipGetLastError();
}

}  // namespace oac
