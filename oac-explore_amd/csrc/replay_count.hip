// Device side of the replay buffer's insert path and of ReplayBufferCount
// (/root/reference/replay_buffer.py:50-104, 151-197):
//
// * insert: n transitions, given in the reference's host dtypes (float64
//   fields, uint8 terminals), packed into the fp32 ring rows at
//   (top + i) % capacity -- the f64 -> f32 rounding the reference does at
//   sample time (ptu.from_numpy(...).float()), done once at insert, so the
//   stored rows are bit-identical to a host-packed insert.
// * counts: counts_out[i] = counts[idx[i]] (before the update), then
//   counts[j] += 1 once per DISTINCT j of the batch -- numpy's buffered fancy
//   indexing, `self._counts[indices] += 1` (replay_buffer.py:196), increments
//   a duplicated index once.  Distinctness by an atomic tag exchange with a
//   per-call epoch, so no tag array is ever cleared.
// * priority sampling: np.random.choice(arange(size), B, p=1/(c+1) / sum)
//   (replay_buffer.py:180-184) is cdf = cumsum(p), cdf /= cdf[-1],
//   idx = searchsorted(cdf, random_sample(B), 'right').  The uniforms are
//   numpy's own random_sample draws (the caller's host stream, so the global
//   RNG advances exactly as in the reference); the cdf is an fp64 device scan
//   of w_j = 1 / (c_j + 1) and idx = #{j : W_j <= u * W_total}.  Only the
//   scan's association differs from numpy's sequential cumsum, so an index can
//   differ only where u lands within fp64 rounding of a cdf step.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "oac_common.h"

namespace oac {

// ------------------------------------------------------------------ insert
__global__ void __launch_bounds__(256) replay_insert_kernel(ReplayInsertArgs a) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)a.n * a.row_stride;
  if (e >= total) return;
  const int i = (int)(e / a.row_stride);
  const int c = (int)(e - (long)i * a.row_stride);
  float v = 0.f;   // row padding stays zero
  if (c >= a.off_obs && c < a.off_obs + a.obs_dim) v = (float)a.obs[(long)i * a.obs_dim + c - a.off_obs];
  else if (c >= a.off_act && c < a.off_act + a.act_dim) v = (float)a.act[(long)i * a.act_dim + c - a.off_act];
  else if (c == a.off_rew) v = (float)a.rew[i];
  else if (c == a.off_term) v = a.term[i] ? 1.f : 0.f;
  else if (c >= a.off_next_obs && c < a.off_next_obs + a.obs_dim)
    v = (float)a.next_obs[(long)i * a.obs_dim + c - a.off_next_obs];
  const long row = (a.top + i) % a.capacity;
  a.storage[row * a.row_stride + c] = v;
}

hipError_t launch_replay_insert(const ReplayInsertArgs& a, hipStream_t s) {
  const long total = (long)a.n * a.row_stride;
  if (total <= 0) return hipSuccess;
  OAC_LAUNCH(replay_insert_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------ counts
__global__ void __launch_bounds__(256) counts_read_kernel(const int* counts, const int* idx, int B,
                                                          float* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < B) out[i] = (float)counts[idx[i]];
}

__global__ void __launch_bounds__(256) counts_bump_kernel(int* counts, int* tags, const int* idx,
                                                          int B, int epoch) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B) return;
  const int j = idx[i];
  if (atomicExch(tags + j, epoch) != epoch) counts[j] += 1;   // first occurrence only
}

hipError_t launch_counts_update(int* counts, int* tags, const int* idx, int B, int epoch,
                                float* counts_out, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const dim3 g((B + 255) / 256);
  if (counts_out) OAC_LAUNCH(counts_read_kernel, g, dim3(256), 0, s, (const int*)counts, idx, B, counts_out);
  OAC_LAUNCH(counts_bump_kernel, g, dim3(256), 0, s, counts, tags, idx, B, epoch);
  return hipGetLastError();
}

// Ring path of the counts=True trainers: one workgroup per step reads the
// batch counts (before the draw's update) and then bumps every distinct drawn
// row, so every read precedes every bump without a launch boundary; the tag
// epoch is a device counter advanced by the same workgroup (the step's graph
// carries no host value).  The step's indices are ring slot batch_counter %
// ring_slots, as in gather_kernel.
__global__ void __launch_bounds__(1024) counts_step_kernel(CountsStepArgs a) {
  const long long bc = a.state ? a.state->batch_counter : 0;
  const int* idx = a.ring_slots > 0 ? a.idx + (bc % a.ring_slots) * (long long)a.B : a.idx;
  const int e = *a.epoch;
  for (int i = threadIdx.x; i < a.B; i += blockDim.x) a.out[i] = (float)a.counts[idx[i]];
  __syncthreads();
  for (int i = threadIdx.x; i < a.B; i += blockDim.x) {
    const int j = idx[i];
    if (atomicExch(a.tags + j, e) != e) a.counts[j] += 1;   // first occurrence only
  }
  __syncthreads();
  if (threadIdx.x == 0) *a.epoch = e + 1;
}

hipError_t launch_counts_step(const CountsStepArgs& a, hipStream_t s) {
  if (a.B <= 0) return hipSuccess;
  OAC_LAUNCH(counts_step_kernel, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------- priority sampling
// Two-level inclusive scan of w_j = 1/(c_j + 1) in fp64: 1024 threads x 4
// elements per block (kScanBlock), block totals scanned by one block (up to
// 1024 blocks: size <= 4M), then per-sample binary search.
constexpr int kScanBlock = 4096;

__global__ void __launch_bounds__(1024) prio_scan_blocks(const int* counts, long size, double* W,
                                                         double* block_tot) {
  __shared__ double sh[1024];
  const long base = (long)blockIdx.x * kScanBlock + threadIdx.x * 4;
  double v[4], run = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long j = base + k;
    const double w = j < size ? 1.0 / ((double)counts[j] + 1.0) : 0.0;
    run += w;
    v[k] = run;
  }
  sh[threadIdx.x] = run;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {   // Hillis-Steele over the thread totals
    const double add = threadIdx.x >= off ? sh[threadIdx.x - off] : 0.0;
    __syncthreads();
    sh[threadIdx.x] += add;
    __syncthreads();
  }
  const double pre = threadIdx.x > 0 ? sh[threadIdx.x - 1] : 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + k < size) W[base + k] = pre + v[k];
  if (threadIdx.x == 1023) block_tot[blockIdx.x] = sh[1023];
}

__global__ void __launch_bounds__(1024) prio_scan_tops(double* block_tot, int nblk) {
  __shared__ double sh[1024];
  sh[threadIdx.x] = threadIdx.x < nblk ? block_tot[threadIdx.x] : 0.0;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const double add = threadIdx.x >= off ? sh[threadIdx.x - off] : 0.0;
    __syncthreads();
    sh[threadIdx.x] += add;
    __syncthreads();
  }
  if (threadIdx.x < nblk) block_tot[threadIdx.x] = sh[threadIdx.x];   // inclusive block prefix
}

// idx = #{j : W_j <= t}, t = u * W_total, W_j = block prefix + in-block scan
__global__ void __launch_bounds__(256) prio_search(const double* W, const double* block_pre, long size,
                                                   int nblk, const double* u, int B, int* idx_out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B) return;
  const double total = block_pre[nblk - 1];
  const double t = u[i] * total;
  // block: first b with block_pre[b] > t
  int lo = 0, hi = nblk;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (block_pre[mid] <= t) lo = mid + 1; else hi = mid;
  }
  const int b = lo < nblk ? lo : nblk - 1;
  const double pre = b > 0 ? block_pre[b - 1] : 0.0;
  long l = (long)b * kScanBlock, h = l + kScanBlock < size ? l + kScanBlock : size;
  while (l < h) {
    const long mid = (l + h) >> 1;
    if (pre + W[mid] <= t) l = mid + 1; else h = mid;
  }
  idx_out[i] = (int)(l < size ? l : size - 1);
}

long prio_scratch_doubles(long size) {
  return size + (size + kScanBlock - 1) / kScanBlock + 1;
}

hipError_t launch_priority_sample(const int* counts, long size, const double* u, int B,
                                  double* scratch, int* idx_out, hipStream_t s) {
  const int nblk = (int)((size + kScanBlock - 1) / kScanBlock);
  if (size <= 0 || nblk > 1024) return hipErrorInvalidValue;
  double* W = scratch;
  double* tops = scratch + size;
  OAC_LAUNCH(prio_scan_blocks, dim3(nblk), dim3(1024), 0, s, counts, size, W, tops);
  OAC_LAUNCH(prio_scan_tops, dim3(1), dim3(1024), 0, s, tops, nblk);
  OAC_LAUNCH(prio_search, dim3((B + 255) / 256), dim3(256), 0, s, (const double*)W, (const double*)tops,
             size, nblk, u, B, idx_out);
  return hipGetLastError();
}

}  // namespace oac
