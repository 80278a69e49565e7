// GELU and its derivative for the epilogues (vv_gemm.hip) and the fused tower MLP (vv_tower.hip):
// nn.GELU() (exact, erf form; networks_old/utils/swinblock.py:13-29 Mlp act_layer) at fp32 level, branch-free.
//
//   h(x)    = Phi(-|x|) = 0.5 erfc(|x| / sqrt 2) = 2^(u S(u) - 1),  u = min(|x|, 5.75)
//   Phi(x)  = x >= 0 ? 1 - h : h
//   GELU(x) = x Phi(x)  = x >= 0 ? x - x h : x h
//   GELU'(x) = Phi(x) + x phi(x),  phi(x) = 2^(x^2 (-0.5 log2 e) + log2(1 / sqrt(2 pi)))
//
// S: degree-8 polynomial fitted to log2(2 h(u)) / u (tools/fit_erf.py, weights towards minimax on the GELU error
// relative to |x|). In float32 (Horner fma chain, v_exp_f32): GELU within 8.7e-8 |x|, Phi and GELU' within 8.2e-8
// absolute of float64 over [-9, 9] -- the rounding of the result itself; the libm erff path costs ~40 VALU
// instructions per element with its two divergent ranges, this one 15 (GELU) / 19 (GELU').
// Infinities: GELU(+inf) = +inf (x - x h would be inf - inf), GELU(-inf) ~ 0 and GELU'(+-inf) = 1 / ~0
// (x phi(x) would be inf * 0): the x that multiplies h and phi is clamped to +-30 by one v_med3_f32. For |x| <= 30
// that is x itself; beyond it x h < 2^-25 x for x > 0, and the true x h and x phi(x) are below 1.4e-7 for x < -30.
// A NaN stays NaN (GELU: the x - x h side of the select; GELU': phi from the unclamped x * x).
// Checked on the device over a dense grid against float64 erf (tests/test_gpu_kernels.py::test_gelu_device_*).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

namespace vv {

__device__ __forceinline__ float gelu_h(float x) {
  const float u = fminf(fabsf(x), 5.75f);
  float s = 5.128587759e-07f;
  s = fmaf(s, u, -9.560183571e-06f);
  s = fmaf(s, u, 7.497351908e-05f);
  s = fmaf(s, u, -2.843466355e-04f);
  s = fmaf(s, u, 1.498893471e-05f);
  s = fmaf(s, u, 6.931121461e-03f);
  s = fmaf(s, u, -5.243476480e-02f);
  s = fmaf(s, u, -4.592214525e-01f);
  s = fmaf(s, u, -1.151104212e+00f);
  return __builtin_amdgcn_exp2f(fmaf(u, s, -1.0f));
}

// four at a time, each Horner step over the four before the next, so the four dependent chains interleave
__device__ __forceinline__ void gelu_h4(const float (&x)[4], float (&h)[4]) {
  float u[4], s[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u[i] = fminf(fabsf(x[i]), 5.75f);
    s[i] = fmaf(5.128587759e-07f, u[i], -9.560183571e-06f);
  }
  constexpr float c[7] = {7.497351908e-05f, -2.843466355e-04f, 1.498893471e-05f, 6.931121461e-03f,
                          -5.243476480e-02f, -4.592214525e-01f, -1.151104212e+00f};
#pragma unroll
  for (int k = 0; k < 7; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = fmaf(s[i], u[i], c[k]);
#pragma unroll
  for (int i = 0; i < 4; ++i) h[i] = __builtin_amdgcn_exp2f(fmaf(u[i], s[i], -1.0f));
}

__device__ __forceinline__ float gelu_clamp(float x) { return __builtin_amdgcn_fmed3f(x, -30.0f, 30.0f); }
__device__ __forceinline__ float gelu_fast(float x) {
  const float h = gelu_h(x);
  const float xh = gelu_clamp(x) * h;
  return x < 0.0f ? xh : x - xh;  // NaN takes the x - xh side (v_med3 drops a NaN)
}
__device__ __forceinline__ float dgelu_fast(float x) {
  const float h = gelu_h(x);
  const float cdf = x >= 0.0f ? 1.0f - h : h;
  // phi(x) = 2^(-x^2 log2(e) / 2 - log2(sqrt(2 pi)))
  // x * x (not xc * xc) in the exponent: a NaN x gives a NaN pdf and result, an infinite one pdf = 0
  const float pdf = __builtin_amdgcn_exp2f(fmaf(x * x, -0.72134752044448170f, -1.3257480647361593f));
  return fmaf(gelu_clamp(x), pdf, cdf);
}

__device__ __forceinline__ void gelu4(const float (&x)[4], float (&y)[4]) {
  float h[4];
  gelu_h4(x, h);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float xh = gelu_clamp(x[i]) * h[i];
    y[i] = x[i] < 0.0f ? xh : x[i] - xh;
  }
}
__device__ __forceinline__ void dgelu4(const float (&x)[4], float (&y)[4]) {
  float h[4];
  gelu_h4(x, h);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float cdf = x[i] >= 0.0f ? 1.0f - h[i] : h[i];
    const float pdf = __builtin_amdgcn_exp2f(fmaf(x[i] * x[i], -0.72134752044448170f, -1.3257480647361593f));
    y[i] = fmaf(gelu_clamp(x[i]), pdf, cdf);
  }
}

}  // namespace vv
