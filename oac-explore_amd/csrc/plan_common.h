// Shared machinery of the launch plans (SAC / particle trainers): workspace
// bookkeeping, split-K sizing, GEMM task constructors, HIP-event timing.
#pragma once
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "kernels.h"
#include "oac_common.h"

namespace oac {

static inline int64_t al4(int64_t x) { return (x + 3) & ~int64_t(3); }
static inline int64_t al64(int64_t x) { return (x + 63) & ~int64_t(63); }

enum Kind { K_GEMM = 0, K_ROW = 1, K_ADAM = 2, K_GATHER = 3, OAC_NUM_KINDS = 4 };

struct WsBuf { int64_t off, rows, cols; };
struct Split { int S, kchunk; };

struct PlanBase {
  int cfg = 0;  // gemm tile config
  BatchCache bcache;   // the launches' GemmBatch records in device memory (kernels.h)
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipStream_t graph_stream = nullptr;
  int graph_flags = -1;
  int graph_n = 0;          // steps captured in the graph
  hipStream_t cap_stream = nullptr;   // capture stream (graphs launch on the caller's stream)
  // the caller's captured data-parallel step (oac_sac_set_step_graph; not owned)
  hipGraphExec_t ext_exec = nullptr;
  int ext_flags = 0;   // the step flags ext_exec was captured with
  int launches = 0;
  // drop-in host-index staging (oac_sac_set_host_ring): pinned [slots][B] int32,
  // one completion event per 16-slot chunk, recorded when staging leaves the
  // chunk (behind every step enqueued so far, so behind all of the chunk's
  // readers) and waited on when staging enters it again; last_bc is the
  // batch counter of the previous staging call (-1: none since the ring was set)
  int32_t* host_ring = nullptr;
  std::vector<hipEvent_t> ring_ev;
  std::vector<char> ring_ev_set;
  int64_t last_bc = -1;
  // direct mode (oac_sac_set_host_ring(NULL)): the ring is the plan's own
  // host-coherent allocation and the small-batch layer-0 launch reads the
  // indices from it (no H2D copy, no gather launch); the chunk's completion
  // event is recorded at the next staging call, behind the step that read it
  bool rows_direct = false;
  // host-read mode (the plan's own ring, not rows_direct: the large-batch SAC
  // step and the particle / det trainers): an oac_sac_step_host_idx step's
  // gather (and counts) launch reads the slot straight from the host ring
  // (kStepHostIdx), so no H2D copy precedes the step's graph
  bool idx_host = false;
  bool owns_host_ring = false;
  // HIP-event kernel timing (bench instrumentation; never inside a graph)
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, int>> ev_pending;   // (kind, index of the start event)
  int ev_next = 0;
  double kind_ms[OAC_NUM_KINDS] = {0};
  long long kind_count[OAC_NUM_KINDS] = {0};
};

static inline Split choose_split(int K, int tiles, int cfg) {
  const int bk = cfg == 0 ? 64 : 32;
  int S = 1;
  if (K >= 512) {
    int want = (512 + tiles - 1) / tiles;
    int maxS = K / (cfg == 0 ? 256 : 128);
    S = want < maxS ? want : maxS;
    if (S < 1) S = 1;
  }
  int kchunk = (K + S - 1) / S;
  kchunk = ((kchunk + bk - 1) / bk) * bk;
  S = (K + kchunk - 1) / kchunk;
  return {S, kchunk};
}

// split-K of a dW on gemm_bwdp.hip (64x64 tiles over the N - 1 real columns):
// about 768 workgroups per gradient kind, chunks of >= 256 batch rows.  B=4096
// SAC step (OAC_SPLITS sweep): critic layer 0 13, the rest 16 splits -- 3,225
// steps/s against 3,108 with the register-direct kernel's splits (19 / 16 /
// 32).  (Sizing each dW for the slots its launch's dX tiles and side blocks
// leave -- critic layer 1 12 splits, one round of 992 workgroups instead of
// 1,152; layer 0 15; policy layer 0 32 -- measured slower on every one of
// those launches, round 3: 33.9 -> 34.7, 26.0 -> 29.8, 15.2 -> 16.0 us; the
// per-workgroup prologue / epilogue and slab traffic outweigh the tail.)
static inline Split choose_split_pipe(int K, int tiles) {
  tiles = std::max(1, tiles);
  int S = std::max(1, std::min(K / 256, 768 / tiles));
  // a power of two (equal chunks of a power-of-two batch): B=4096 SAC critic
  // layer 0 dW 13 -> 8 splits, 26.0 -> 24.4 us, 3,884 -> 3,918 steps/s (same
  // box after the round-robin XCD mapping; 10 and 6 splits: 30-31 us); the
  // other launches of the measured configs already were
  while (S & (S - 1)) S &= S - 1;
  // a small dW (configs[4]'s 256 x 119 critic layer 0: 8 tiles) would leave
  // CUs idle: chunks down to 128 rows until one workgroup per CU
  if (S * tiles < 256) S = std::max(S, std::min(K / 128, (256 + tiles - 1) / tiles));
  int kchunk = (K + S - 1) / S;
  kchunk = ((kchunk + 31) / 32) * 32;
  S = (K + kchunk - 1) / kchunk;
  return {S, kchunk};
}

// ------------------------------------------------------------ task makers
static inline GemmTask task0() {
  GemmTask t;
  std::memset(&t, 0, sizeof(t));
  t.ksplit = 1;
  return t;
}

// Y[M,N] = X[M,K] . W[N,K]^T   (W row-major [N, ldw])
static inline GemmTask t_fwd(const float* X, long ldx, int M, int K, const float* W, long ldw, int N,
                      float* C, long ldc, int epi, const float* bias) {
  GemmTask t = task0();
  t.A = X; t.lda = ldx; t.a_kc = 1;
  t.B = W; t.ldb = ldw; t.b_kc = 1;
  t.C = C; t.ldc = ldc; t.M = M; t.N = N; t.K = K;
  t.epi = epi; t.bias = bias;
  return t;
}

// dX[M,N] = dY[M,K] . W[K,N]  (W row-major [K, ldw]); epilogue mask from aux.
static inline GemmTask t_dx(const float* dY, long lddy, int M, int K, const float* W, long ldw, int N,
                     float* C, long ldc, const float* mask_src, long ld_mask_src) {
  GemmTask t = task0();
  t.A = dY; t.lda = lddy; t.a_kc = 1;
  t.B = W; t.ldb = ldw; t.b_kc = 0;
  t.C = C; t.ldc = ldc; t.M = M; t.N = N; t.K = K;
  if (mask_src) { t.epi = EPI_MASK; t.aux = mask_src; t.ld_aux = ld_mask_src; }
  else t.epi = EPI_STORE;
  return t;
}

// dY rows given as s[b] * v[n] * (mask[b,n] > 0)  (rank-1 seed through a ReLU)
static inline void set_rank1(GemmTask& t, const float* s, const float* v, const float* mask, long ldm) {
  t.a_mode = A_RANK1_MASK; t.a_s = s; t.a_v = v; t.a_mask = mask; t.ld_mask = ldm;
}

// dW[M, Kin] and db[M] = dY^T[M,B] . [X | 1][B, Kin+1], written in the
// parameter-arena layout (gw / gb point into the gradient arena, or into
// split-K slab `split` at +split*slab_stride).  dY row-major [B, lddy].
static inline GemmTask t_dw(const float* dY, long lddy, int M, int Bn, const float* X, long ldx,
                            int Kin, float* gw, float* gb, long slab_stride, Split sp) {
  GemmTask t = task0();
  t.A = dY; t.lda = lddy; t.a_kc = 0;
  t.B = X; t.ldb = ldx; t.b_kc = 0; t.b_ones = 1;
  t.M = M; t.N = Kin + 1; t.K = Bn;
  t.C = gw; t.ldc = Kin; t.bias_grad = gb; t.epi = EPI_GRAD;
  t.ksplit = sp.S; t.kchunk = sp.kchunk; t.slab_stride = slab_stride;
  return t;
}

static inline int tick(PlanBase& p, hipStream_t s) {
  if (!p.timing) return -1;
  if (p.ev_next + 2 > (int)p.ev_pool.size()) {
    for (int i = 0; i < 64; ++i) {
      hipEvent_t e;
      OAC_HIP_CHECK(hipEventCreate(&e));
      p.ev_pool.push_back(e);
    }
  }
  const int i = p.ev_next;
  p.ev_next += 2;
  // the launch records the pair on its dispatch (OAC_LAUNCH, hipExtLaunchKernel)
  g_ext_timing.start = p.ev_pool[i];
  g_ext_timing.stop = p.ev_pool[i + 1];
  g_ext_timing.consumed = false;
  return i;
}
static inline int tock(PlanBase& p, int kind, int i, hipStream_t s) {
  (void)s;
  if (i < 0) return 0;
  if (g_ext_timing.consumed) p.ev_pending.push_back({kind, i});
  g_ext_timing.start = g_ext_timing.stop = nullptr;
  g_ext_timing.consumed = false;
  return 0;
}
#define TIMED(p, kind, s, call)          \
  do {                                   \
    const int _t = tick(p, s);           \
    call;                                \
    if (tock(p, kind, _t, s)) return 1;  \
  } while (0)


// Plan-level tile configuration (PlanBase::cfg): 0 = the small-batch kernel
// for every product, 1 = the LDS-tiled kernel (gemm.hip) for every product the
// small kernel does not take, 2 = the large-batch per-launch choice below
// (the default at batch >= 1024).  The round-1 register-direct kernel
// (gemm_big.hip, launch cfg 2 / 3) that cfg 2 once fell back on took no
// launch of any measured workload after round 3 and was removed in round 5.
constexpr int kCfgLargeBatch = 2;
// split-K sizing tile of the products sized before the per-launch choice
// (the head dW's sp_ph at large batch: 128 x 64, as the kernel the sizing was
// tuned on)
static inline int split_tile_m(int cfg) { return cfg == 0 ? 32 : cfg == kCfgLargeBatch ? 128 : 64; }
static inline int split_tile_n(int cfg) { return cfg == 0 ? 32 : 64; }

bool gemm_fwd_supports(const GemmBatch& b);

// Forward batches at large batch go to gemm_fwd.hip (LDS-DMA pipelined
// 128x128 / 128x64 / 64x64 tiles, cfg 6 / 7 / 8).  Measured per launch at B=4096
// against the register-direct kernel of rounds 1-3 (tools/micro/fwd_micro,
// bitwise equal to it): SAC layer 0 (6 tasks) 77.5 -> 66.4 us on 128x64 (74.6 on 128x128: 384 tiles = 1.5 rounds), critic
// layer 1 + head partials (4 tasks) 35.6 -> 27.7 us on 128x128, policy layer 1
// (2 tasks) 21.9 -> 15.4 us on 128x64.
// 128x64 tiles (three workgroups per CU on the 2-stage ring) when they give
// every CU at least one, 64x64 otherwise (a single 4096 x 256 product: 128
// tiles of 128x64 would leave half the chip idle).  128x128 measured equal to
// 128x64 at 256 tiles and worse elsewhere (tools/micro/fwd_micro).
static inline int fwd2_cfg(const GemmBatch& gb) {
  // rounds of tiles per CU x tile area, 64x64 tiles charged ~18 % more per
  // unit of work (fewer MFMAs per LDS read): 384 tiles of 128x64 (configs[4]
  // policy layer 1) leave half the CUs with one tile and half with two, where
  // 768 tiles of 64x64 are three everywhere
  int t7 = 0, t8 = 0;
  for (int i = 0; i < gb.ntasks; ++i) {
    t7 += ((gb.t[i].M + 127) / 128) * ((gb.t[i].N + 63) / 64);
    t8 += ((gb.t[i].M + 63) / 64) * ((gb.t[i].N + 63) / 64);
  }
  const double c7 = 2.0 * ((t7 + 255) / 256), c8 = 1.18 * ((t8 + 255) / 256);
  return c8 < c7 ? 8 : 7;
}

// Backward batches at large batch go to gemm_bwdp.hip (LDS-DMA pipelined,
// cfg 9 = 128x64 tiles, 10 = 64x64, 11 = 128x128, 12 = 64x64 on a 2-stage ring).
bool gemm_bwdp_supports(const GemmBatch& b);
static inline int bwdp_cfg(const GemmBatch& gb) {
  // 64x64 tiles beat 128x64 on every backward launch of the B=4096 SAC step
  // (tools/micro/bwd_micro: critic layer 1 48.8 -> 38.6 us, layer 0 dW 37.9
  // -> 33.0, -min Q dX 20.7 -> 19.0), and on a 2-stage ring (cfg 12: 36 KB of
  // LDS, four workgroups per CU instead of three, bitwise the same) critic
  // layer 0 dW 33.6 -> 30.2, layer 1 38.7 -> 37.8, the rest equal (round 3)
  const int forced = tuning(OAC_TUNE_BWDP_CFG);
  (void)gb;
  return (forced >= 9 && forced <= 17 && forced != 16) ? forced : 12;
}

static inline int launch_cfg(int cfg, const GemmBatch& gb) {
  if (cfg == 0) return 0;
  for (int i = 0; i < gb.ntasks; ++i)   // the fused head backward exists on the small kernel only
    if (gb.t[i].epi == EPI_HEAD_BWD) return 0;
  // narrow products at large batch (width-1 critic heads, dL/da with N = act
  // dim): a 64-wide LDS tile computes 1-17 useful columns over 8 barriered K
  // blocks; the small-batch kernel's 32x32 tiles with K split over waves
  // finish them in a fraction of the time
  bool narrow = !gb.fuse_adam;
  for (int i = 0; i < gb.ntasks && narrow; ++i)
    narrow = gb.t[i].N <= 32 && gb.t[i].ksplit <= 1 && gb.t[i].K2 == 0;
  if (narrow) return 0;
  if (cfg != kCfgLargeBatch) return cfg;
  bool all_fwd = true, all_bwd = true, dot = false;
  for (int i = 0; i < gb.ntasks; ++i) {
    all_fwd = all_fwd && gb.t[i].a_kc && gb.t[i].b_kc && gb.t[i].N >= 64;
    all_bwd = all_bwd && !gb.t[i].b_kc;
    dot = dot || gb.t[i].epi == EPI_BIAS_RELU_DOT;
  }
  // (narrow-row dW batches on the small kernel measured -1 % at B=4096 and were dropped)
  if (all_fwd && gemm_fwd_supports(gb)) return fwd2_cfg(gb);
  // a dX with a short K (the head's 2 Da, a K-output critic's K) rides
  // along with its batch's dW (same-box A/B, B=4096: SAC 3,276 -> 3,310,
  // configs[4] 4,106 -> 4,200 steps/s against keeping those batches on the
  // register-direct kernel of the time)
  if (all_bwd && gemm_bwdp_supports(gb)) return bwdp_cfg(gb);
  // the rest (hidden < 64, ragged dims, mixed batches): the LDS-tiled kernel,
  // or the small kernel for a batch carrying the width-1 head dot (an
  // epilogue the LDS-tiled kernel does not have)
  return dot ? 0 : 1;
}

static inline int run_gemm(PlanBase& p, GemmBatch& gb, hipStream_t s) {
  const int cfg = launch_cfg(p.cfg, gb);
  gemm_batch_finalize(gb, cfg);
  if (tuning(OAC_TUNE_DEBUG_CFG)) {
    fprintf(stderr, "launch %d cfg %d tiles %d:", p.launches, cfg, gb.total_tiles);
    for (int i = 0; i < gb.ntasks; ++i)
      fprintf(stderr, " [M%d N%d K%d akc%d bkc%d r1%d epi%d S%d]", gb.t[i].M, gb.t[i].N, gb.t[i].K,
              gb.t[i].a_kc, gb.t[i].b_kc, gb.t[i].a_mode, gb.t[i].epi, gb.t[i].ksplit);
    fprintf(stderr, "\n");
  }
  TIMED(p, K_GEMM, s, OAC_HIP_CHECK(gemm_batch_launch(gb, cfg, s, &p.bcache, p.launches)));
  p.launches++;
  return 0;
}

static inline void add(GemmBatch& gb, const GemmTask& t) { gb.t[gb.ntasks++] = t; }

}  // namespace oac
