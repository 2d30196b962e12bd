// Row-wise evaluation of the trainer's networks off the gradient step: the
// forward of the arena modules (FlattenMlp, networks.py:154-161 -> Mlp.forward
// 62-79; TanhGaussianPolicy.forward, trainer/policies.py:260-316) and
// SACTrainer.predict / ParticleTrainer.predict (trainer/trainer.py:105-123,
// trainer/particle_trainer_oac.py:147-167), whose Q_UB the reference
// differentiates w.r.t. the action (optimistic_exploration.py:39, 64).
//
// One 256-thread workgroup per (row, network): the row's input and hidden
// activations stay in LDS; a layer is one wave per output unit (lanes stride
// the inputs, coalesced, fixed-order butterfly sum).  With `jac` the same
// workgroup backpropagates each output to the input:
//   d q_k / d x = W0^T (1[h0 > 0] . W1^T (1[h1 > 0] . W_last[k]))
// (thread i of a reduction owns input i, so the weight reads are coalesced).
#include <cstring>

#include "oac_common.h"
#include "kernels.h"
#include "policy_math.h"

namespace oac {

__device__ __forceinline__ float wave_sum(float s) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  return s;
}

// out[j] = act(b[j] + sum_k W[j, k] in[k]) for j < n_out; W row-major [n_out, n_in]
__device__ __forceinline__ void dense_rows(const float* W, const float* b, const float* in,
                                           int n_in, int n_out, float* out, bool relu) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int j = wave; j < n_out; j += nw) {
    const float* w = W + (long)j * n_in;
    float s = 0.f;
    for (int k = lane; k < n_in; k += 64) s = fmaf(w[k], in[k], s);
    s = wave_sum(s) + b[j];
    if (lane == 0) out[j] = relu ? fmaxf(s, 0.f) : s;
  }
}

// the shared trunk: x (LDS, n_in) -> h0, h1 (LDS, H each)
__device__ __forceinline__ void trunk(const float* net, const MlpEvalArgs& a, const float* x,
                                      int n_in, float* h0, float* h1) {
  dense_rows(net + a.w0, net + a.b0, x, n_in, a.H, h0, true);
  __syncthreads();
  dense_rows(net + a.w1, net + a.b1, h0, a.H, a.H, h1, true);
  __syncthreads();
}

__device__ __forceinline__ void load_input(const MlpEvalArgs& a, int row, float* x) {
  for (int k = threadIdx.x; k < a.d0 + a.d1; k += blockDim.x)
    x[k] = k < a.d0 ? a.x0[(long)row * a.ld_x0 + k] : a.x1[(long)row * a.ld_x1 + (k - a.d0)];
  __syncthreads();
}

// grid (N, n_nets): FlattenMlp outputs (+ input Jacobian)
__global__ void __launch_bounds__(256) critic_eval_kernel(MlpEvalArgs a) {
  extern __shared__ float lds[];
  const int row = blockIdx.x, ni = blockIdx.y;
  const int din = a.d0 + a.d1, H = a.H;
  float* x = lds;
  float* h0 = x + din;
  float* h1 = h0 + H;
  float* g1 = h1 + H;
  float* g2 = g1 + H;
  float* q = g2 + H;
  const float* net = a.net[ni];
  load_input(a, row, x);
  trunk(net, a, x, din, h0, h1);
  dense_rows(net + a.wl, net + a.bl, h1, H, a.Q, q, false);
  __syncthreads();
  for (int k = threadIdx.x; k < a.Q; k += blockDim.x)
    a.out[(long)row * a.ld_out + ni * a.Q + k] = q[k];
  if (!a.jac) return;
  const float* W1 = net + a.w1;
  const float* W0 = net + a.w0;
  for (int k = 0; k < a.Q; ++k) {
    for (int j = threadIdx.x; j < H; j += blockDim.x)
      g2[j] = h1[j] > 0.f ? net[a.wl + (long)k * H + j] : 0.f;
    __syncthreads();
    for (int i = threadIdx.x; i < H; i += blockDim.x) {
      float s = 0.f;
      for (int j = 0; j < H; ++j) s = fmaf(g2[j], W1[(long)j * H + i], s);
      g1[i] = h0[i] > 0.f ? s : 0.f;
    }
    __syncthreads();
    float* out = a.jac + ((long)row * a.n_nets * a.Q + (long)ni * a.Q + k) * din;
    for (int c = threadIdx.x; c < din; c += blockDim.x) {
      float s = 0.f;
      for (int i = 0; i < H; ++i) s = fmaf(g1[i], W0[(long)i * din + c], s);
      out[c] = s;
    }
    __syncthreads();
  }
}

// grid (N): TanhGaussianPolicy.forward; the heads are stored stacked [2 Da, H]
// (mean rows, then log-std rows).  outs: action | mean | log_std | std |
// pre_tanh [N, Da] and log_prob [N] (return_log_prob, stochastic only).
__global__ void __launch_bounds__(256) policy_eval_kernel(MlpEvalArgs a) {
  extern __shared__ float lds[];
  const int row = blockIdx.x;
  const int din = a.d0, H = a.H, Da = a.Q / 2;
  float* x = lds;
  float* h0 = x + din;
  float* h1 = h0 + H;
  float* hd = h1 + H;        // [2 Da] head outputs
  float* lp = hd + 2 * Da;   // [Da] per-dim log-prob terms
  const float* net = a.net[0];
  load_input(a, row, x);
  trunk(net, a, x, din, h0, h1);
  dense_rows(net + a.wl, net + a.bl, h1, H, 2 * Da, hd, false);
  __syncthreads();
  for (int i = threadIdx.x; i < Da; i += blockDim.x) {
    const long o = (long)row * Da + i;
    const float mean = hd[i];
    const float ls = fminf(fmaxf(hd[Da + i], -20.f), 2.f);   // policies.py:279
    a.p_mean[o] = mean;
    a.p_log_std[o] = ls;
    if (a.p_eps) {
      float act, sd, u;
      lp[i] = tanh_gauss_sample(mean, hd[Da + i], a.p_eps[o], act, sd, u);
      a.p_action[o] = act;
      a.p_std[o] = sd;
      a.p_pre_tanh[o] = __fadd_rn(mean, u);   // z = mean + std eps
    } else {                                   // deterministic: tanh(mean), policies.py:286-288
      a.p_action[o] = tanhf(mean);
      a.p_std[o] = expf(ls);
      a.p_pre_tanh[o] = mean;
      lp[i] = 0.f;
    }
  }
  __syncthreads();
  if (a.p_log_prob && threadIdx.x == 0) {   // sum over the action dims (keepdim), in order
    float s = 0.f;
    for (int i = 0; i < Da; ++i) s += lp[i];
    a.p_log_prob[row] = s;
  }
}

size_t mlp_eval_lds_bytes(const MlpEvalArgs& a, bool policy) {
  const int din = a.d0 + a.d1;
  return sizeof(float) * (size_t)(policy ? din + 2 * a.H + a.Q + a.Q / 2 + 4
                                         : din + 4 * a.H + a.Q + 4);
}

hipError_t launch_critic_eval(const MlpEvalArgs& a, hipStream_t s) {
  if (a.N <= 0) return hipSuccess;
  OAC_LAUNCH(critic_eval_kernel, dim3(a.N, a.n_nets), dim3(256), mlp_eval_lds_bytes(a, false), s, a);
  return hipGetLastError();
}

hipError_t launch_policy_eval(const MlpEvalArgs& a, hipStream_t s) {
  if (a.N <= 0) return hipSuccess;
  OAC_LAUNCH(policy_eval_kernel, dim3(a.N), dim3(256), mlp_eval_lds_bytes(a, true), s, a);
  return hipGetLastError();
}

}  // namespace oac

using namespace oac;

extern "C" int oac_critic_eval(const float* const* nets, int n_nets, const int64_t* offsets, int obs_dim,
                               int act_dim, int hidden, int q_out, const float* obs, int64_t ld_obs,
                               const float* act, int64_t ld_act, int n, float* q_out_buf,
                               float* jac, void* stream) {
  if (!nets || n_nets < 1 || n_nets > 2 || !offsets || obs_dim < 1 || act_dim < 0 || hidden < 1 ||
      q_out < 1 || n < 0 || !obs || (act_dim > 0 && !act) || !q_out_buf) {
    set_error("critic eval: bad arguments");
    return 1;
  }
  if ((size_t)(obs_dim + act_dim + 4 * hidden + q_out) * 4 > 160 * 1024) {
    set_error("critic eval: dims exceed the workgroup's LDS");
    return 1;
  }
  MlpEvalArgs a;
  memset(&a, 0, sizeof(a));
  for (int i = 0; i < n_nets; ++i) a.net[i] = nets[i];
  a.n_nets = n_nets;
  a.w0 = offsets[0]; a.b0 = offsets[1]; a.w1 = offsets[2]; a.b1 = offsets[3];
  a.wl = offsets[4]; a.bl = offsets[5];
  a.x0 = obs; a.ld_x0 = ld_obs; a.d0 = obs_dim;
  a.x1 = act; a.ld_x1 = ld_act; a.d1 = act_dim;
  a.H = hidden; a.Q = q_out; a.N = n;
  a.out = q_out_buf; a.ld_out = (long)n_nets * q_out; a.jac = jac;
  OAC_HIP_CHECK(launch_critic_eval(a, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int oac_policy_eval(const float* net, const int64_t* offsets, int obs_dim, int act_dim,
                               int hidden, const float* obs, int64_t ld_obs, int n, const float* eps,
                               float* action, float* mean, float* log_std, float* log_prob,
                               float* std_out, float* pre_tanh, void* stream) {
  if (!net || !offsets || obs_dim < 1 || act_dim < 1 || hidden < 1 || n < 0 || !obs || !action ||
      !mean || !log_std || !std_out || !pre_tanh) {
    set_error("policy eval: bad arguments");
    return 1;
  }
  if ((size_t)(obs_dim + 2 * hidden + 3 * act_dim + 4) * 4 > 160 * 1024) {
    set_error("policy eval: dims exceed the workgroup's LDS");
    return 1;
  }
  MlpEvalArgs a;
  memset(&a, 0, sizeof(a));
  a.net[0] = net; a.n_nets = 1;
  a.w0 = offsets[0]; a.b0 = offsets[1]; a.w1 = offsets[2]; a.b1 = offsets[3];
  a.wl = offsets[4]; a.bl = offsets[5];
  a.x0 = obs; a.ld_x0 = ld_obs; a.d0 = obs_dim;
  a.H = hidden; a.Q = 2 * act_dim; a.N = n;
  a.p_eps = eps; a.p_action = action; a.p_mean = mean; a.p_log_std = log_std;
  a.p_log_prob = log_prob; a.p_std = std_out; a.p_pre_tanh = pre_tanh;
  OAC_HIP_CHECK(launch_policy_eval(a, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}
