// Per-element math of TanhGaussianPolicy / TanhNormal shared by every kernel
// that evaluates it (rows.hip, head.hip, the GEMM head-backward epilogue), so
// all paths round identically.
#pragma once
#include <hip/hip_runtime.h>

namespace oac {

// TanhGaussianPolicy.forward tail (/root/reference/trainer/policies.py:275-304)
// for one action dim: log_std = clamp(ls_raw, -20, 2); std = exp(log_std);
// z = mean + std*eps; a = tanh(z); returns the log-prob term
//   -(z-mean)^2/(2 std^2) - log std - log sqrt(2 pi) - log(1 - a^2 + 1e-6)
// (TanhNormal.log_prob, policies.py:147-160; log std is std.log()).
__device__ __forceinline__ float tanh_gauss_sample(float mean, float ls_raw, float eps, float& act,
                                                   float& sd, float& u) {
  const float ls = fminf(fmaxf(ls_raw, -20.f), 2.f);
  sd = expf(ls);
  const float z = __fadd_rn(mean, __fmul_rn(sd, eps));
  act = tanhf(z);
  u = z - mean;
  const float var = __fmul_rn(sd, sd);
  const float t1 = -(__fmul_rn(u, u)) / (2.f * var);
  return t1 - logf(sd) - 0.918938533204672742f  // log(sqrt(2*pi))
         - logf(__fadd_rn(1.f - __fmul_rn(act, act), 1e-6f));
}

// Its backward for the policy loss mean(alpha*logp - minQ): ga = dL/da from
// the critics, G = alpha/B = dL/dlogp; through log_prob, tanh, z = mean +
// std*eps and std = exp(clamp(ls_raw)) (clamp passes the gradient on
// -20 <= ls_raw <= 2).
__device__ __forceinline__ void tanh_gauss_backward(float ga, float a, float sd, float u, float eps,
                                                    float ls_raw, float G, float& dmean,
                                                    float& dls) {
  const float var = sd * sd;
  const float one_m_a2 = 1.f - a * a;
  const float da = ga + G * (2.f * a / (one_m_a2 + 1e-6f));
  const float uv = u / var;
  const float dz = da * one_m_a2 - G * uv;
  dmean = dz + G * uv;
  const float dstd = dz * eps + G * (u * u * sd / (var * var) - 1.f / sd);
  dls = (ls_raw >= -20.f && ls_raw <= 2.f) ? dstd * sd : 0.f;
}

}  // namespace oac
