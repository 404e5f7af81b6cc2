// erf-GELU for the hand GEMM epilogues (exact-erf form, as torch.nn.functional.gelu's default).
//
// Abramowitz & Stegun 7.1.26, |erf error| <= 1.5e-7, rearranged for the VALU: with h = x / 2,
//   x Phi(x) = h (1 + sign(x) erf(|x| / sqrt2)) = h + |h| - |h| P(t) e^{-x^2/2}
//            = max(x, 0) - |x| (P(t) / 2) e^{-x^2/2},   t = 1 / (1 + p |x| / sqrt2)
// (the 1/2 and 1/sqrt2 folded into the constants): 12 VALU + rcp + exp2 per value, against 14 + 2
// transcendental-rate ops for the textbook 0.5 x (1 + erf) form.  |x| is clamped to 1e30 so
// that x = +-inf gives inf / 0 instead of inf * 0.
#pragma once

namespace amd_dft {

__device__ __forceinline__ float gelu_erf(float x) {
  const float ax = fminf(fabsf(x), 1e30f);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, ax, 1.f));
  float p = fmaf(0.5f * 1.061405429f, t, 0.5f * -1.453152027f);
  p = fmaf(p, t, 0.5f * 1.421413741f);
  p = fmaf(p, t, 0.5f * -0.284496736f);
  p = fmaf(p, t, 0.5f * 0.254829592f);
  p *= t;
  const float ex = __builtin_amdgcn_exp2f(x * x * (-0.5f * 1.4426950408889634f));
  return fmaf(-ax * p, ex, fmaxf(x, 0.f));
}

}  // namespace amd_dft
