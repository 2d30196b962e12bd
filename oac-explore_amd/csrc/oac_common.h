// Shared host/device definitions for liboac_amd (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/oac_amd.h"

namespace oac {

// ---------------------------------------------------------------------------
// Grouped fp32 GEMM task:  C(m,n) = sum_k A(m,k) * B(k,n)  (+ fused epilogue)
//
// Operand storage is described by (row, col) of the underlying row-major
// buffer, so one task type covers the three products of an MLP step:
//   forward  Y  = X  . W^T   A k-contig (row=m,col=k)  B k-contig (row=n,col=k)
//   dX       dX = dY . W     A k-contig                B n-contig (row=k,col=n)
//   dW       dW = dY^T . X   A m-contig (row=k,col=m)  B n-contig
// ---------------------------------------------------------------------------
enum AMode : int {
  A_PLAIN = 0,        // A[row*lda + col]
  A_RANK1_MASK = 1,   // s[row] * v[col] * (mask[row*ld_mask + col] > 0)
};

enum Epi : int {
  EPI_STORE = 0,          // C = acc
  EPI_BIAS = 1,           // C = acc + bias[n]
  EPI_BIAS_RELU = 2,      // C = relu(acc + bias[n])
  EPI_BIAS_RANK_RELU = 3, // C = acc + bias[n];  C2 = relu(C + sum_j U[m,j] V[n,j])
  EPI_ADD_RELU = 4,       // C = relu(acc + aux[m,n])
  EPI_MASK = 5,           // C = aux[m,n] > 0 ? acc : 0
  EPI_GRAD = 6,           // weight gradient in the parameter-arena layout:
                          // C[m*ldc + n] (n < N-1), bias_grad[m] (n == N-1, the
                          // ones column); both offset by split*slab_stride
  EPI_HEAD_BWD = 8,       // acc = dL/da (N = act_dim): tanh-Gaussian head backward
                          // (policy_math.h) -> C[m*ldc + n] = dmean, C[m*ldc + N + n]
                          // = dls_raw; ex[] = act, std, u, eps, head, &alpha (small kernel).
                          // C2 set: the head's dX follows in the same workgroup,
                          // C2[m*ldc2 + c] = [aux[m*ld_aux + c] > 0] sum_k dhead[m, k] U[k*ldu + c]
                          // for the R columns c at C2 / aux / U (one column chunk of
                          // the hidden layer; dup: the dhead stores are another task's)
  EPI_BIAS_RELU_DOT = 7,  // C = relu(acc + bias[n]) and, per row, the partial
                          // dot of this 32-column tile with aux[n] (a width-1
                          // output layer): C2[(n0/32)*ldc2 + m]  (small kernel)
};

struct GemmTask {
  const float* A;
  const float* a_s;
  const float* a_v;
  const float* a_mask;
  const float* B;
  float* C;
  float* C2;
  const float* bias;
  const float* aux;
  const float* U;
  const float* V;
  float* bias_grad;
  long lda, ldb, ldc, ldc2, ld_aux, ldu, ldv, ld_mask;
  int M, N, K;
  int a_kc;      // 1: A(m,k) at row=m,col=k ; 0: row=k,col=m
  int b_kc;      // 1: B(k,n) at row=n,col=k ; 0: row=k,col=n
  int a_mode;
  int b_ones;    // 1: column n == N-1 of B is virtual ones (dW bias column)
  int epi;
  int R;         // rank of the EPI_BIAS_RANK_RELU update
  int ksplit;    // K chunks (EPI_GRAD only); chunk = kchunk (multiple of 64)
  int kchunk;
  // small kernel, rank-1-seeded dW (A = s[k] v[m] [x(k, m) > 0]) unsplit:
  // the tiles of the first column block also reduce, per output row m, the
  // bias column sum_k A(m, k) into bias_grad[m] (b_ones off: no ones-column
  // tiles) and the seed's width-1 layer gradient sum_k s[k] x(k, m) into
  // C2[m], and the m0 = 0 tile sum_k s[k] into C2[ldc2] (that layer's bias)
  int fold;
  long slab_stride;
  int tile_begin;
  int tiles_n;
  // optional second product accumulated into the same tile (same layouts and
  // leading dimensions, K2 > 0, unsplit): acc = A.B + A2.B2
  const float* A2;
  const float* B2;
  int K2;
  int dup;              // EPI_HEAD_BWD with C2: the tiles recompute another task's dhead for
                        // their column chunk of the head's dX and store only that (here: the
                        // padding after K2, the record keeps its 304 bytes)
  const float* ex[6];   // extra epilogue operands (EPI_HEAD_BWD)
  int a_rows;           // small kernel: A (and U) row m is row batch.rg rows[m] of the buffer
  int no_adam;          // EPI_GRAD in a fused-Adam batch: store the gradient only (another group's)
};

struct StepState;
struct AlphaState;

struct AdamArgs {
  float* p; float* g; float* m; float* v; long n;
  // split-K gradient slabs shaped like the arena range: g = sum_s gslab[s*stride + i]
  // (written back to g); gslab == g with S == 1 reads g directly
  const float* gslab; int S; int S2; long slab_stride;
  // elements [s2_lo, s2_hi) of the range (16-byte aligned) hold only S2 < S
  // slabs (a layer split fewer ways than the group's widest; S2 = 0: none)
  long s2_lo, s2_hi;
  float* target; float tau; int period;   // target != null -> Polyak after the step
  double lr, beta1, beta2, eps;
  StepState* state;
  int advance;       // 0: critic Adam (t = n_steps; block 0 snapshots t, commits alpha)
                     // 1: final policy Adam (t = t_snapshot; block 0 advances the step)
  AlphaState* alpha; // commit next_* (critic Adam only); may be null
  float gscale;      // gradient scale (1/world_size after an all-reduce SUM)
  int reduce_only;   // data-parallel: only reduce the slabs into g (all-reduce next)
  int no_book;       // skip the state / alpha bookkeeping (a partial range of the group)
  float* p_out;      // small-kernel epilogue Adam: the updated p goes here (same index), not to p
  const float* copy_src;   // small-kernel side blocks: copy this (same index) into p, no Adam
  int preview;       // small-kernel epilogue Adam: write only p (to p_out), leave m, v, target
};

constexpr int kMaxTasks = 8;
constexpr int kLaTickets = 4096;   // GemmBatch::la_ticket entries

// The layer-0 launch of a direct drop-in step (small kernel, sac_plan phase0):
// the batch's rows are read straight from the replay through the host-written
// index slot rows = ring + (batch_counter % slots) * B, and `blocks` extra
// workgroups copy those rows to `out` (the step's batch for the later launches)
// and draw the step's Philox eps -- the gather launch's work, off the chain.
// inl (host pointer, B <= kInlineRows): the step's indices themselves, which
// the launcher copies into the kernel arguments (no host-memory read in the
// kernel; never under stream capture, whose kernel arguments are frozen).
constexpr int kInlineRows = 256;
struct RowGather {
  const int* ring; int slots, B;
  const int* inl;
  const StepState* state;
  int blocks;
  const float* replay; long row_stride; float* out;
  float* eps1; float* eps2; int n_eps; unsigned long long seed;
};

struct GemmBatch {
  GemmTask t[kMaxTasks];
  int ntasks;
  int total_tiles;
  // Fused optimizer (small-batch kernel, unsplit K): every EPI_GRAD element is
  // also Adam(+Polyak)-updated in the epilogue (its index in the group is its
  // gradient pointer minus adam.g), and blocks [total_tiles, +adam_blocks) run
  // the flat Adam over the group's other ranges (gradients finished by earlier
  // launches of the step).  adam.state / adam.alpha bookkeeping: block 0.
  int fuse_adam;
  int nseg;
  StepState* publish;        // non-null: block 0 publishes the step's Adam constants
  double pub_beta1, pub_beta2;
  int adam_blocks;           // set by the launcher
  int force_nw, force_gpw;   // small kernel: waves per workgroup / k-groups in flight (0 = auto)
  long seg_off[2], seg_n[2]; // flat ranges (floats, multiples of 4) from the group base
  AdamArgs adam;
  // Side optimizer (large-batch kernels, gemm_bwdp.hip): side_adam > 0 extra
  // workgroups (blockIdx >= total_tiles) run the flat Adam -- split-K slabs
  // summed in fixed order, as adam_flat_kernel -- over the ranges
  // seg_off/seg_n[0 .. nseg) of `adam`, whose gradients earlier launches of
  // the step finished and whose parameters no tile of this launch reads;
  // side_book: the first side workgroup also does adam.state / adam.alpha
  // bookkeeping.  Independent of fuse_adam (small kernel only).
  // side_first: the side workgroups are blockIdx [0, side_adam) (a multiple
  // of 8, so every tile keeps its XCD), dispatched ahead of the tiles.
  int side_adam, side_book, side_first;
  // Last-arrival optimizer (gemm_bwdp.hip, la_adam != 0): the batch's
  // split-K dW tasks store their slabs write-through, and the workgroup that
  // finishes a dW tile last (an agent-scope ticket per (m, n) tile in
  // la_ticket[tile_begin + tile], re-armed by that workgroup) sums the
  // tile's t.ksplit slabs in adam_flat_kernel's fixed order and applies
  // `adam` (+ Polyak) to the tile's elements -- the group's Adam launch for
  // those elements, without the launch; la_book: the (0, 0) tile's last
  // arrival also does the adam.state / adam.alpha bookkeeping
  unsigned* la_ticket;        // kLaTickets of them (a launch's tiles: at most that many)
  int la_adam, la_book;
  RowGather rg;              // rg.ring != null: direct row gather (small kernel only)
};

// A launch's GemmBatch read from device memory (kernels.h BatchCache) through a
// pointer declared global: through a generic one the compiler cannot tell that
// the operand pointers loaded from the record are global, and every operand
// access becomes a flat load
typedef __attribute__((address_space(1))) GemmBatch GemmBatchG;

// ---------------------------------------------------------------------------
// Device-resident step state (read by every kernel of a step; advanced by the
// last block of the step's final kernel, so the launch sequence is static and
// can be replayed as one hipGraph).
// ---------------------------------------------------------------------------
//
// No kernel writes a field another block of the same launch reads, so no
// fences or tickets are needed: the critic Adam copies n_steps to t_snapshot
// (block 0), and the policy Adam -- which reads t_snapshot -- advances
// n_steps and batch_counter (block 0).
struct StepState {
  long long n_steps;        // SACTrainer._n_train_steps_total
  long long batch_counter;  // replay ring cursor / Philox counter
  long long expl_counter;   // Philox counter for exploration draws
  long long t_snapshot;     // n_steps as seen by this step (for the last Adam)
  // Adam bias corrections for t = bc_t (= n_steps + 1: all three optimisers of
  // a step share t), published by the step's first launch so no later kernel
  // evaluates pow() per thread
  double bc1, bc2, sbc2;    // 1 - beta1^t, 1 - beta2^t, sqrt(bc2)
  long long bc_t;
};

// alpha (auto entropy tuning) state, 16 floats.  critic_targets computes the
// update (every block, identically) and block 0 publishes next_*; the critic
// Adam commits next_* -> current (trainer.py:139-146).
struct AlphaState {
  float log_alpha, m, v;       // current (log_alpha is the snapshot's 'log_alpha')
  float alpha, alpha_loss, grad;
  float sum;                   // data-parallel: all-reduced sum(logp + target_entropy)
  float pad0;
  float next_log_alpha, next_m, next_v;
  float pad1[5];
};

}  // namespace oac

#define OAC_HIP_CHECK(expr)                                                     \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      oac::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,              \
                     hipGetErrorString(_e));                                    \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

namespace oac {
void set_error(const char* fmt, ...);

// the process's non-default kernel / schedule choices (oac_tuning_set; all 0
// = the defaults)
extern int g_tuning[OAC_TUNE_COUNT];
inline int tuning(int key) { return g_tuning[key]; }

// Kernel-exact timing (bench instrumentation, never inside a graph): when
// g_ext_timing.start is set, the next OAC_LAUNCH records the pair on the
// dispatch itself (hipExtLaunchKernel start/stop events = the kernel's begin
// and end timestamps, the same interval rocprofv3's kernel trace reports) and
// marks the pair consumed.
struct ExtTiming {
  hipEvent_t start = nullptr, stop = nullptr;
  bool consumed = false;
};
extern thread_local ExtTiming g_ext_timing;
}

#include <hip/hip_ext.h>
#define OAC_LAUNCH(kernel, grid, block, shmem, stream, ...)                                  \
  do {                                                                                      \
    if (oac::g_ext_timing.start && !oac::g_ext_timing.consumed) {                           \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, oac::g_ext_timing.start,    \
                            oac::g_ext_timing.stop, 0, __VA_ARGS__);                        \
      oac::g_ext_timing.consumed = true;                                                    \
    } else {                                                                                \
      hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                  \
    }                                                                                       \
  } while (0)
